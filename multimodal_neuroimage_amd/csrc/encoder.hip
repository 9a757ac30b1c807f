// Crossmodal-encoder dense layers on the f32 matrix cores (reference:
// TransformerEncoderLayer.forward crossmodal_transformer.py:133-165 and the in/out projections of
// MultiheadAttention.forward multihead_attention.py:71-84,129).
//
//   rowgemm      Y[r][n] = epi( sum_k X'[r][k] W(n, k) )   on time-major token rows (T*B, K)
//                  X' = LayerNorm(X) (prologue: row statistics in-kernel, written for the
//                  backward) or X;  W(n, k) = w[n*w_sn + k*w_sk] (an nn.Linear weight, or its
//                  transpose for dX = dY W);  epi: + bias, ReLU, x (aux > 0) (ReLU backward),
//                  + residual.  Replaces LN -> F.linear (-> F.relu) (-> + residual): one launch.
//   rowgemm_dw   dW[n][k] = sum_r dY[r][n] X'[r][k], db[n] = sum_r dY[r][n] (X' = LN(X) recomputed
//                  from the saved row statistics, or X): row chunks per workgroup, one partial row
//                  per chunk, fixed-order column sum (deterministic).
//   row_ln_bwd   dX = LN_bwd(dXn) + dres, dgamma / dbeta (per-block partial rows, fixed order).
//
// Every contraction is v_mfma_f32_16x16x4_f32: exact fp32 products (an fmaf chain per output,
// cdna_hip_programming.md §FP32-input MFMA), so the layers keep the reference's fp32 arithmetic.
// Lane l = 16 g + t supplies A[row t][k g] and B[k g][col t]; the accumulator holds D[row 4 g + i]
// [col t] in register i.  Tiles: a 256-thread workgroup owns 64 rows x 64 outputs, each wave a
// 32 x 32 quarter (2 x 2 MFMA tiles, 4 independent accumulator chains); K goes through LDS in
// chunks of 32 with the next chunk's global loads issued before the current chunk's MFMAs.
#include "mmni_common.h"

namespace mmni {
namespace enc {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 zero4() { return (f4){0.f, 0.f, 0.f, 0.f}; }

// Contraction order.  The sum over k is order-free between the operands, so k-step s of the
// MFMA takes k = 16 (s / 4) + 4 g + (s % 4) on lane group g: the four k-steps of group j = s / 4
// are one 16-byte piece k = 16 j + 4 g .. + 3 of a lane's row, loaded straight from global memory
// (L2-resident weights and activations) with no LDS staging and no barriers.  Per wave a 32 x 32
// output tile (2 x 2 MFMA tiles, four independent accumulator chains); a 256-thread block 64 x 64.
constexpr int BM = 64, BN = 64;
constexpr int KG = 16;       // k per group (4 k-steps)
constexpr int KMAX_LN = 176; // LN prologue: the whole row (K <= 176, 11 groups) held in registers
constexpr int DEPTH = 4;     // groups in flight

struct RGArgs {
    int64_t rows, ldx, ldy, ldres, ldaux, w_sn, w_sk;
    int K, N, ln, relu;
    float eps;
    const float* x;
    const float* gamma;
    const float* beta;
    const float* w;
    const float* bias;
    const float* aux;
    const float* res;
    float* y;
    float* mean;
    float* rstd;
};

// 4 consecutive k (from k0) of row r of a (rows, ld) matrix; zeros past K / past the rows
__device__ __forceinline__ f4 load_k4(const float* base, int64_t r, int64_t ld, bool rok, int k0, int K) {
    const float* p = base + r * ld + k0;
    if (rok && k0 + 3 < K && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) return *reinterpret_cast<const f4*>(p);
    f4 v = zero4();
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (rok && k0 + i < K) ? p[i] : 0.f;
    return v;
}

// W(n, k0 .. k0 + 3): k-contiguous (w_sk = 1) as a 16-byte piece, n-contiguous (the transpose) as
// four scalars of rows k0 .. k0 + 3 (lanes of a group read 16 consecutive n: coalesced)
__device__ __forceinline__ f4 load_w4(const RGArgs& a, int n, int k0) {
    const bool nok = n < a.N;
    if (a.w_sk == 1) return load_k4(a.w, n, a.w_sn, nok, k0, a.K);
    f4 v = zero4();
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (nok && k0 + i < a.K) ? a.w[(int64_t)(k0 + i) * a.w_sk + n] : 0.f;
    return v;
}

template <bool LN>
__global__ __launch_bounds__(256) void rowgemm_kernel(RGArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = lane & 15, g = lane >> 4;
    const int64_t m0 = (int64_t)blockIdx.x * BM + (wave & 1) * 32;     // the wave's 32 rows
    const int n0 = blockIdx.y * BN + (wave >> 1) * 32;                 // and 32 outputs
    const int64_t ra = m0 + t, rb = m0 + 16 + t;                       // A rows of the two m tiles
    const bool oka = ra < a.rows, okb = rb < a.rows;
    const int na = n0 + t, nb = n0 + 16 + t;                           // B columns of the two n tiles
    const int NG = (a.K + KG - 1) / KG;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
    auto mma_group = [&](f4 xa, f4 xb, f4 wa, f4 wb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[0][0] = mfma(xa[i], wa[i], acc[0][0]);
            acc[0][1] = mfma(xa[i], wb[i], acc[0][1]);
            acc[1][0] = mfma(xb[i], wa[i], acc[1][0]);
            acc[1][1] = mfma(xb[i], wb[i], acc[1][1]);
        }
    };
    if constexpr (LN) {
        // the two rows' whole K extent in registers, LayerNorm statistics by the 4 lane groups
        constexpr int MG = KMAX_LN / KG;
        f4 xa[MG], xb[MG];
#pragma unroll
        for (int j = 0; j < MG; ++j) {
            if (j < NG) {
                xa[j] = load_k4(a.x, ra, a.ldx, oka, KG * j + 4 * g, a.K);
                xb[j] = load_k4(a.x, rb, a.ldx, okb, KG * j + 4 * g, a.K);
            } else {
                xa[j] = xb[j] = zero4();
            }
        }
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int j = 0; j < MG; ++j) {
            sa += (xa[j][0] + xa[j][1]) + (xa[j][2] + xa[j][3]);
            sb += (xb[j][0] + xb[j][1]) + (xb[j][2] + xb[j][3]);
        }
        sa += __shfl_xor(sa, 16); sa += __shfl_xor(sa, 32);
        sb += __shfl_xor(sb, 16); sb += __shfl_xor(sb, 32);
        const float invK = 1.0f / (float)a.K;
        const float ma = sa * invK, mb = sb * invK;
        float va = 0.f, vb = 0.f;
#pragma unroll
        for (int j = 0; j < MG; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool in = KG * j + 4 * g + i < a.K;
                const float da = in ? xa[j][i] - ma : 0.f, db = in ? xb[j][i] - mb : 0.f;
                va = fmaf(da, da, va);
                vb = fmaf(db, db, vb);
            }
        va += __shfl_xor(va, 16); va += __shfl_xor(va, 32);
        vb += __shfl_xor(vb, 16); vb += __shfl_xor(vb, 32);
        const float rsa = 1.0f / sqrtf(va * invK + a.eps), rsb = 1.0f / sqrtf(vb * invK + a.eps);
        if (a.mean != nullptr && blockIdx.y == 0 && (wave >> 1) == 0 && g == 0) {
            if (oka) { a.mean[ra] = ma; a.rstd[ra] = rsa; }
            if (okb) { a.mean[rb] = mb; a.rstd[rb] = rsb; }
        }
        f4 wa[DEPTH], wb[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            wa[d] = d < NG ? load_w4(a, na, KG * d + 4 * g) : zero4();
            wb[d] = d < NG ? load_w4(a, nb, KG * d + 4 * g) : zero4();
        }
#pragma unroll
        for (int j = 0; j < MG; ++j) {
            if (j < NG) {
            f4 ga, gb, xna, xnb;
            const int k0 = KG * j + 4 * g;
            ga = load_k4(a.gamma, 0, 0, true, k0, a.K);
            gb = load_k4(a.beta, 0, 0, true, k0, a.K);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xna[i] = fmaf((xa[j][i] - ma) * rsa, ga[i], gb[i]);
                xnb[i] = fmaf((xb[j][i] - mb) * rsb, ga[i], gb[i]);
            }
            const f4 wcur_a = wa[j % DEPTH], wcur_b = wb[j % DEPTH];
            if (j + DEPTH < NG) {
                wa[j % DEPTH] = load_w4(a, na, KG * (j + DEPTH) + 4 * g);
                wb[j % DEPTH] = load_w4(a, nb, KG * (j + DEPTH) + 4 * g);
            }
            mma_group(xna, xnb, wcur_a, wcur_b);
            }
        }
    } else {
        // stream K in groups, DEPTH groups of all four operands in flight
        f4 xa[DEPTH], xb[DEPTH], wa[DEPTH], wb[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int k0 = KG * d + 4 * g;
            const bool v = d < NG;
            xa[d] = v ? load_k4(a.x, ra, a.ldx, oka, k0, a.K) : zero4();
            xb[d] = v ? load_k4(a.x, rb, a.ldx, okb, k0, a.K) : zero4();
            wa[d] = v ? load_w4(a, na, k0) : zero4();
            wb[d] = v ? load_w4(a, nb, k0) : zero4();
        }
        for (int j0 = 0; j0 < NG; j0 += DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                const int j = j0 + d;
                if (j >= NG) break;
                const f4 ca = xa[d], cb = xb[d], cwa = wa[d], cwb = wb[d];
                if (j + DEPTH < NG) {
                    const int k0 = KG * (j + DEPTH) + 4 * g;
                    xa[d] = load_k4(a.x, ra, a.ldx, oka, k0, a.K);
                    xb[d] = load_k4(a.x, rb, a.ldx, okb, k0, a.K);
                    wa[d] = load_w4(a, na, k0);
                    wb[d] = load_w4(a, nb, k0);
                }
                mma_group(ca, cb, cwa, cwb);
            }
        }
    }
    // epilogue: D[row 4 g + i][col t] of tile (mi, ni)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        const int n = n0 + 16 * ni + t;
        if (n >= a.N) continue;
        const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = m0 + 16 * mi + 4 * g + i;
                if (r >= a.rows) continue;
                float v = acc[mi][ni][i] + b;
                if (a.relu) v = fmaxf(v, 0.f);
                if (a.aux != nullptr && !(a.aux[r * a.ldaux + n] > 0.f)) v = 0.f;
                if (a.res != nullptr) v += a.res[r * a.ldres + n];
                a.y[r * a.ldy + n] = v;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// weight gradient: dW[n][k] = sum_r dY[r][n] X'[r][k] (+ db[n] as the extra column k = K of ones)
// per (64 x 64 output tile, row chunk) block; partials [chunk][N * K + N] reduced in chunk order
// ---------------------------------------------------------------------------------------------
struct DWArgs {
    int64_t rows, ldx, lddy;
    int K, N, ln, rows_per_chunk;
    const float* x;
    const float* gamma;
    const float* beta;
    const float* mean;
    const float* rstd;
    const float* dy;
    float* part;   // [chunk][N * K + N]: dW row-major, then db
};

// rows r0 + 16 j + 4 g + i (i = 0..3) of column c (scalars; the 16 lanes of a group read 16
// consecutive columns of each row)
__device__ __forceinline__ f4 load_rows4(const float* base, int64_t ld, int64_t r0, int64_t rend, int c, int C) {
    f4 v = zero4();
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (r0 + i < rend && c < C) ? base[(r0 + i) * ld + c] : 0.f;
    return v;
}

__global__ __launch_bounds__(256) void rowgemm_dw_kernel(DWArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = lane & 15, g = lane >> 4;
    const int n0 = blockIdx.x * BN + (wave & 1) * 32, k0 = blockIdx.y * BN + (wave >> 1) * 32;
    const int64_t rbeg = (int64_t)blockIdx.z * a.rows_per_chunk;
    const int64_t rend = rbeg + a.rows_per_chunk < a.rows ? rbeg + a.rows_per_chunk : a.rows;
    const int na = n0 + t, nb = n0 + 16 + t, ka = k0 + t, kb = k0 + 16 + t;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
    // X' column k of rows r..r+3: LayerNorm recompute, the ones column k == K (db), zeros past it
    auto load_x = [&](int64_t r, int k) {
        f4 v = zero4();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t rr = r + i;
            if (rr < rend && k < a.K) {
                float xv = a.x[rr * a.ldx + k];
                if (a.ln) xv = fmaf((xv - a.mean[rr]) * a.rstd[rr], a.gamma[k], a.beta[k]);
                v[i] = xv;
            } else if (rr < rend && k == a.K) {
                v[i] = 1.0f;
            }
        }
        return v;
    };
    const int NG = (int)((rend - rbeg + KG - 1) / KG);
    f4 da[DEPTH], db[DEPTH], xa[DEPTH], xb[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const int64_t r = rbeg + KG * d + 4 * g;
        da[d] = load_rows4(a.dy, a.lddy, r, rend, na, a.N);
        db[d] = load_rows4(a.dy, a.lddy, r, rend, nb, a.N);
        xa[d] = load_x(r, ka);
        xb[d] = load_x(r, kb);
    }
    for (int j0 = 0; j0 < NG; j0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int j = j0 + d;
            if (j >= NG) break;
            const f4 ca = da[d], cb = db[d], cxa = xa[d], cxb = xb[d];
            if (j + DEPTH < NG) {
                const int64_t r = rbeg + KG * (j + DEPTH) + 4 * g;
                da[d] = load_rows4(a.dy, a.lddy, r, rend, na, a.N);
                db[d] = load_rows4(a.dy, a.lddy, r, rend, nb, a.N);
                xa[d] = load_x(r, ka);
                xb[d] = load_x(r, kb);
            }
            // A[row n][kk = row]: dY;  B[kk = row][col k]: X'
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[0][0] = mfma(ca[i], cxa[i], acc[0][0]);
                acc[0][1] = mfma(ca[i], cxb[i], acc[0][1]);
                acc[1][0] = mfma(cb[i], cxa[i], acc[1][0]);
                acc[1][1] = mfma(cb[i], cxb[i], acc[1][1]);
            }
        }
    }
    // D[row n = 4 g + i][col k = t]
    float* p = a.part + (int64_t)blockIdx.z * ((int64_t)a.N * a.K + a.N);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int ki = 0; ki < 2; ++ki) {
            const int k = k0 + 16 * ki + t;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + 16 * ni + 4 * g + i;
                if (n >= a.N) continue;
                if (k < a.K) p[(int64_t)n * a.K + k] = acc[ni][ki][i];
                else if (k == a.K) p[(int64_t)a.N * a.K + n] = acc[ni][ki][i];
            }
        }
}

// out[j] = sum_c part[c][j] in chunk order (deterministic); columns [0, split) -> out, [split, ncols)
// -> out2 (nullable).  One thread per 4 columns, every chunk's load issued before the adds.
__global__ __launch_bounds__(256) void chunk_sum_kernel(const float* __restrict__ part, int nchunks, int ncols,
                                                        int split, float* out, float* out2) {
    const int j4 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (j4 >= ncols) return;
    f4 s = zero4();
    const bool vec = j4 + 3 < ncols && (ncols & 3) == 0;
    for (int c0 = 0; c0 < nchunks; c0 += 8) {
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            v[u] = zero4();
            if (c0 + u < nchunks) {
                const float* p = part + (int64_t)(c0 + u) * ncols + j4;
                if (vec) v[u] = *reinterpret_cast<const f4*>(p);
                else
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[u][i] = j4 + i < ncols ? p[i] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = j4 + i;
        if (j >= ncols) break;
        if (j < split) out[j] = s[i];
        else if (out2 != nullptr) out2[j - split] = s[i];
    }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm backward on rows of C <= 256: one wave per row, 4 columns per lane
// ---------------------------------------------------------------------------------------------
struct LNBArgs {
    int64_t rows, lddxn, ldx, ldres, lddx;
    int C;
    const float* dxn;
    const float* x;
    const float* gamma;
    const float* mean;
    const float* rstd;
    const float* dres;
    float* dx;
    float* part;   // [block][2C]: dgamma | dbeta
};

__global__ __launch_bounds__(256) void row_ln_bwd_kernel(LNBArgs a) {
    __shared__ float red[4][2][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f}, gm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j;
        gm[j] = c < a.C ? a.gamma[c] : 0.f;
    }
    const float invC = 1.0f / (float)a.C;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.rows; r += (int64_t)gridDim.x * 4) {
        const float m = a.mean[r], rs = a.rstd[r];
        float d[4], xh[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j;
            d[j] = c < a.C ? a.dxn[r * a.lddxn + c] : 0.f;
            xh[j] = c < a.C ? (a.x[r * a.ldx + c] - m) * rs : 0.f;
            const float gd = d[j] * gm[j];
            s1 += gd;
            s2 = fmaf(gd, xh[j], s2);
            dg[j] = fmaf(d[j], xh[j], dg[j]);
            db[j] += d[j];
        }
        for (int o = 32; o > 0; o >>= 1) {
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
        }
        s1 *= invC;
        s2 *= invC;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j;
            if (c >= a.C) continue;
            float v = rs * (d[j] * gm[j] - s1 - xh[j] * s2);
            if (a.dres != nullptr) v += a.dres[r * a.ldres + c];
            a.dx[r * a.lddx + c] = v;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        red[wave][0][lane + 64 * j] = dg[j];
        red[wave][1][lane + 64 * j] = db[j];
    }
    __syncthreads();
    float* p = a.part + (int64_t)blockIdx.x * 2 * a.C;
    for (int c = threadIdx.x; c < a.C; c += 256) {
        p[c] = ((red[0][0][c] + red[1][0][c]) + red[2][0][c]) + red[3][0][c];
        p[a.C + c] = ((red[0][1][c] + red[1][1][c]) + red[2][1][c]) + red[3][1][c];
    }
}

constexpr int kLnbBlocks = 128;

// row chunks of a weight gradient: >= 64 rows each (4 groups per wave), at most 256, and a
// partial slab of at most 8 MB (the chunk-order reduction reads it once)
int dw_chunks(int64_t rows, int N, int K) {
    int64_t c = rows / 64;
    const int64_t cap = (int64_t)(8 << 20) / (((int64_t)N * K + N) * 4);
    if (c > cap) c = cap;
    if (c > 256) c = 256;
    if (c < 1) c = 1;
    return (int)c;
}

void chunk_sum(const float* part, int nchunks, int ncols, int split, float* out, float* out2, hipStream_t s) {
    const int threads = (ncols + 3) / 4;
    chunk_sum_kernel<<<(threads + 255) / 256, 256, 0, s>>>(part, nchunks, ncols, split, out, out2);
}

}  // namespace enc
}  // namespace mmni

using namespace mmni;

extern "C" int mmni_rowgemm(const mmni_rowgemm_desc* d, const float* x, const float* gamma, const float* beta,
                            const float* w, const float* bias, const float* aux, const float* res, float* y,
                            float* mean, float* rstd, void* stream) {
    MMNI_ARG_CHECK(d != nullptr && x && w && y, "rowgemm: null descriptor or pointer");
    MMNI_ARG_CHECK(d->rows > 0 && d->K > 0 && d->N > 0, "rowgemm: bad extents rows=%lld K=%d N=%d",
                   (long long)d->rows, d->K, d->N);
    MMNI_ARG_CHECK(d->ldx >= d->K && d->ldy >= d->N, "rowgemm: leading dimensions below K / N");
    MMNI_ARG_CHECK((d->w_sk == 1 && d->w_sn >= d->K) || (d->w_sn == 1 && d->w_sk >= d->N),
                   "rowgemm: weight must be k-contiguous (w_sk = 1) or n-contiguous (w_sn = 1)");
    MMNI_ARG_CHECK(!d->ln || (gamma && beta), "rowgemm: LayerNorm prologue needs gamma and beta");
    MMNI_ARG_CHECK(!d->ln || ((mean == nullptr) == (rstd == nullptr)), "rowgemm: mean and rstd go together");
    MMNI_ARG_CHECK(!d->ln || d->K <= enc::KMAX_LN, "rowgemm: LayerNorm prologue over K=%d > %d columns", d->K,
                   enc::KMAX_LN);
    MMNI_ARG_CHECK(aux == nullptr || d->ldaux >= d->N, "rowgemm: aux leading dimension below N");
    MMNI_ARG_CHECK(res == nullptr || d->ldres >= d->N, "rowgemm: residual leading dimension below N");
    enc::RGArgs a{};
    a.rows = d->rows; a.ldx = d->ldx; a.ldy = d->ldy; a.ldres = d->ldres; a.ldaux = d->ldaux;
    a.w_sn = d->w_sn; a.w_sk = d->w_sk; a.K = d->K; a.N = d->N; a.ln = d->ln; a.relu = d->relu; a.eps = d->eps;
    a.x = x; a.gamma = gamma; a.beta = beta; a.w = w; a.bias = bias; a.aux = aux; a.res = res; a.y = y;
    a.mean = d->ln ? mean : nullptr; a.rstd = d->ln ? rstd : nullptr;
    const dim3 grid((unsigned)((d->rows + enc::BM - 1) / enc::BM), (unsigned)((d->N + enc::BN - 1) / enc::BN));
    if (d->ln) enc::rowgemm_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    else enc::rowgemm_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return launch_status("rowgemm");
}

extern "C" size_t mmni_rowgemm_dw_workspace_bytes(const mmni_rowgemm_desc* d) {
    if (d == nullptr || d->rows <= 0 || d->K <= 0 || d->N <= 0) return 0;
    return (size_t)enc::dw_chunks(d->rows, d->N, d->K) * ((size_t)d->N * d->K + d->N) * sizeof(float);
}

extern "C" int mmni_rowgemm_dw(const mmni_rowgemm_desc* d, const float* x, const float* gamma, const float* beta,
                               const float* mean, const float* rstd, const float* dy, float* dw, float* db,
                               void* workspace, void* stream) {
    MMNI_ARG_CHECK(d != nullptr && x && dy && dw && workspace, "rowgemm_dw: null descriptor or pointer");
    MMNI_ARG_CHECK(d->rows > 0 && d->K > 0 && d->N > 0, "rowgemm_dw: bad extents");
    MMNI_ARG_CHECK(d->ldx >= d->K && d->ldy >= d->N, "rowgemm_dw: leading dimensions below K / N (ldy: dY)");
    MMNI_ARG_CHECK(!d->ln || (gamma && beta && mean && rstd), "rowgemm_dw: LayerNorm recompute needs its inputs");
    enc::DWArgs a{};
    a.rows = d->rows; a.ldx = d->ldx; a.lddy = d->ldy; a.K = d->K; a.N = d->N; a.ln = d->ln;
    const int chunks = enc::dw_chunks(d->rows, d->N, d->K);
    a.rows_per_chunk = (int)((d->rows + chunks - 1) / chunks);
    a.x = x; a.gamma = gamma; a.beta = beta; a.mean = mean; a.rstd = rstd; a.dy = dy;
    a.part = static_cast<float*>(workspace);
    const dim3 grid((unsigned)((d->N + enc::BN - 1) / enc::BN), (unsigned)((d->K + 1 + enc::BN - 1) / enc::BN),
                    (unsigned)chunks);
    enc::rowgemm_dw_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a);
    int rc = launch_status("rowgemm_dw");
    if (rc) return rc;
    // dW = columns [0, N K), db = [N K, N K + N) (a null db drops them)
    enc::chunk_sum(a.part, chunks, d->N * d->K + d->N, d->N * d->K, dw, db, (hipStream_t)stream);
    return launch_status("rowgemm_dw_sum");
}

extern "C" size_t mmni_row_layernorm_bwd_workspace_bytes(int64_t rows, int C) {
    (void)rows;
    return (size_t)enc::kLnbBlocks * 2 * C * sizeof(float);
}

extern "C" int mmni_row_layernorm_bwd(int64_t rows, int C, const float* dxn, int64_t lddxn, const float* x,
                                      int64_t ldx, const float* gamma, const float* mean, const float* rstd,
                                      const float* dres, int64_t ldres, float* dx, int64_t lddx, float* dgamma,
                                      float* dbeta, void* workspace, void* stream) {
    MMNI_ARG_CHECK(dxn && x && gamma && mean && rstd && dx && dgamma && dbeta && workspace,
                   "row_layernorm_bwd: null pointer");
    MMNI_ARG_CHECK(rows > 0 && C > 0 && C <= 256, "row_layernorm_bwd: C=%d outside 1..256", C);
    MMNI_ARG_CHECK(lddxn >= C && ldx >= C && lddx >= C && (dres == nullptr || ldres >= C),
                   "row_layernorm_bwd: leading dimensions below C");
    enc::LNBArgs a{};
    a.rows = rows; a.lddxn = lddxn; a.ldx = ldx; a.ldres = ldres; a.lddx = lddx; a.C = C;
    a.dxn = dxn; a.x = x; a.gamma = gamma; a.mean = mean; a.rstd = rstd; a.dres = dres; a.dx = dx;
    a.part = static_cast<float*>(workspace);
    int64_t blocks = (rows + 3) / 4;
    if (blocks > enc::kLnbBlocks) blocks = enc::kLnbBlocks;
    enc::row_ln_bwd_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(a);
    int rc = launch_status("row_layernorm_bwd");
    if (rc) return rc;
    enc::chunk_sum(a.part, (int)blocks, 2 * C, C, dgamma, dbeta, (hipStream_t)stream);
    return launch_status("row_layernorm_bwd_sum");
}
