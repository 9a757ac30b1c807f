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

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int LDW = BK + 2;   // LDS row stride in floats: t * 34 + g hits 32 distinct banks per 32 lanes

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

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

// LayerNorm statistics (nn.LayerNorm: biased variance, eps inside the root) of the block's 64
// rows, 4 threads per row, two passes over the row (mean, then centred squares).
__device__ __forceinline__ void block_row_stats(const RGArgs& a, int64_t r0, float* mean_s, float* rstd_s) {
    const int tid = threadIdx.x, rr = tid >> 2, q = tid & 3;
    const int64_t r = r0 + rr;
    const float* xr = a.x + r * a.ldx;
    float s = 0.f;
    if (r < a.rows)
        for (int k = q; k < a.K; k += 4) s += xr[k];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    const float mean = s / (float)a.K;
    float v = 0.f;
    if (r < a.rows)
        for (int k = q; k < a.K; k += 4) {
            const float d = xr[k] - mean;
            v = fmaf(d, d, v);
        }
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    const float rstd = 1.0f / sqrtf(v / (float)a.K + a.eps);
    if (q == 0) {
        mean_s[rr] = mean;
        rstd_s[rr] = rstd;
        if (a.mean != nullptr && blockIdx.y == 0 && r < a.rows) {
            a.mean[r] = mean;
            a.rstd[r] = rstd;
        }
    }
}

// One K chunk of the block's operands into registers: 8 x-values and 8 w-values per thread.
// x: thread -> row tid / 4, columns 8 (tid % 4) .. +7 of the chunk.  w: thread -> output n,
// 8 consecutive k (k-contiguous weights) or output group / k (n-contiguous, the transposed use).
struct Chunk {
    float x[8], w[8];
};

__device__ __forceinline__ void load_chunk(const RGArgs& a, int64_t r0, int n0, int k0, Chunk& c) {
    const int tid = threadIdx.x;
    {
        const int rr = tid >> 2, kk = (tid & 3) * 8;
        const int64_t r = r0 + rr;
        const float* xr = a.x + r * a.ldx + k0 + kk;
#pragma unroll
        for (int j = 0; j < 8; ++j) c.x[j] = (r < a.rows && k0 + kk + j < a.K) ? xr[j] : 0.f;
    }
    if (a.w_sk == 1) {   // W rows along k: thread -> n = tid / 4, 8 consecutive k
        const int nn = tid >> 2, kk = (tid & 3) * 8;
        const int n = n0 + nn;
        const float* wr = a.w + (int64_t)n * a.w_sn + k0 + kk;
#pragma unroll
        for (int j = 0; j < 8; ++j) c.w[j] = (n < a.N && k0 + kk + j < a.K) ? wr[j] : 0.f;
    } else {             // W columns along n (w_sn == 1): thread -> k = tid / 8, 8 consecutive n
        const int kk = tid >> 3, nn = (tid & 7) * 8;
        const int k = k0 + kk;
        const float* wr = a.w + (int64_t)k * a.w_sk + n0 + nn;
#pragma unroll
        for (int j = 0; j < 8; ++j) c.w[j] = (k < a.K && n0 + nn + j < a.N) ? wr[j] : 0.f;
    }
}

__device__ __forceinline__ void store_chunk(const RGArgs& a, int k0, const Chunk& c, float (*xs)[LDW],
                                            float (*ws)[LDW], const float* mean_s, const float* rstd_s) {
    const int tid = threadIdx.x;
    {
        const int rr = tid >> 2, kk = (tid & 3) * 8;
        if (a.ln) {
            const float m = mean_s[rr], rs = rstd_s[rr];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = k0 + kk + j;
                xs[rr][kk + j] = k < a.K ? fmaf((c.x[j] - m) * rs, a.gamma[k], a.beta[k]) : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[rr][kk + j] = c.x[j];
        }
    }
    if (a.w_sk == 1) {
        const int nn = tid >> 2, kk = (tid & 3) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) ws[nn][kk + j] = c.w[j];
    } else {
        const int kk = tid >> 3, nn = (tid & 7) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) ws[nn + j][kk] = c.w[j];
    }
}

__global__ __launch_bounds__(256) void rowgemm_kernel(RGArgs a) {
    __shared__ float xs[BM][LDW];
    __shared__ float ws[BN][LDW];
    __shared__ float mean_s[BM], rstd_s[BM];
    const int64_t r0 = (int64_t)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = lane & 15, g = lane >> 4;
    const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
    if (a.ln) block_row_stats(a, r0, mean_s, rstd_s);
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};
    Chunk cur;
    load_chunk(a, r0, n0, 0, cur);
    for (int k0 = 0; k0 < a.K; k0 += BK) {
        __syncthreads();   // previous chunk's MFMA reads done (and the row statistics, first time)
        store_chunk(a, k0, cur, xs, ws, mean_s, rstd_s);
        __syncthreads();
        if (k0 + BK < a.K) load_chunk(a, r0, n0, k0 + BK, cur);   // in flight during the MFMAs
        const int rem = a.K - k0 < BK ? a.K - k0 : BK;
        const int ks = (rem + 3) / 4;   // k-steps of this chunk (columns past K are zero)
        auto step = [&](int s) {
            const float x0 = xs[wm + t][4 * s + g], x1 = xs[wm + 16 + t][4 * s + g];
            const float w0 = ws[wn + t][4 * s + g], w1 = ws[wn + 16 + t][4 * s + g];
            acc[0][0] = mfma(x0, w0, acc[0][0]);
            acc[0][1] = mfma(x0, w1, acc[0][1]);
            acc[1][0] = mfma(x1, w0, acc[1][0]);
            acc[1][1] = mfma(x1, w1, acc[1][1]);
        };
        if (ks == BK / 4) {
#pragma unroll
            for (int s = 0; s < BK / 4; ++s) step(s);
        } else {
            for (int s = 0; s < ks; ++s) step(s);
        }
    }
    // epilogue: D[row 4 g + i][col t] of tile (mi, ni)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        const int n = n0 + wn + 16 * ni + t;
        if (n >= a.N) continue;
        const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = r0 + wm + 16 * mi + 4 * g + i;
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

constexpr int DR = 32;   // rows staged per LDS round

__global__ __launch_bounds__(256) void rowgemm_dw_kernel(DWArgs a) {
    // block: outputs n0..n0+63 x k0..k0+63 (k = K is the ones column), rows of chunk blockIdx.z
    // row stride 80 floats: lanes (t, g) reading [4 s + g][t] hit banks 16 g + t, all distinct
    __shared__ float ds[DR][BN + 16];   // dY[r][n]
    __shared__ float xs[DR][BN + 16];   // X'[r][k]
    const int n0 = blockIdx.x * BN, k0 = blockIdx.y * BN;
    const int64_t rbeg = (int64_t)blockIdx.z * a.rows_per_chunk;
    const int64_t rend = rbeg + a.rows_per_chunk < a.rows ? rbeg + a.rows_per_chunk : a.rows;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t = lane & 15, g = lane >> 4;
    const int wn = (wave & 1) * 32, wk = (wave >> 1) * 32;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};
    for (int64_t rb = rbeg; rb < rend; rb += DR) {
        __syncthreads();
        // stage DR rows x 64 columns of dY and X' (thread -> row tid / 8, 8 consecutive columns)
        const int rr = tid >> 3, cc = (tid & 7) * 8;
        const int64_t r = rb + rr;
        const bool rok = r < rend;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = n0 + cc + j;
            ds[rr][cc + j] = (rok && n < a.N) ? a.dy[r * a.lddy + n] : 0.f;
            const int k = k0 + cc + j;
            float xv = 0.f;
            if (rok && k < a.K) {
                xv = a.x[r * a.ldx + k];
                if (a.ln) xv = fmaf((xv - a.mean[r]) * a.rstd[r], a.gamma[k], a.beta[k]);
            } else if (rok && k == a.K) {
                xv = 1.0f;   // db
            }
            xs[rr][cc + j] = xv;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < DR / 4; ++s) {
            // A[row n = t][kk = row g]: dY[4 s + g][n]; B[kk = row g][col k = t]: X'[4 s + g][k]
            const float d0 = ds[4 * s + g][wn + t], d1 = ds[4 * s + g][wn + 16 + t];
            const float x0 = xs[4 * s + g][wk + t], x1 = xs[4 * s + g][wk + 16 + t];
            acc[0][0] = mfma(d0, x0, acc[0][0]);
            acc[0][1] = mfma(d0, x1, acc[0][1]);
            acc[1][0] = mfma(d1, x0, acc[1][0]);
            acc[1][1] = mfma(d1, x1, acc[1][1]);
        }
    }
    // D[row n = 4 g + i][col k = t]
    float* p = a.part + (int64_t)blockIdx.z * ((int64_t)a.N * a.K + a.N);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int ki = 0; ki < 2; ++ki) {
            const int k = k0 + wk + 16 * ki + t;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + wn + 16 * ni + 4 * g + i;
                if (n >= a.N) continue;
                if (k < a.K) p[(int64_t)n * a.K + k] = acc[ni][ki][i];
                else if (k == a.K) p[(int64_t)a.N * a.K + n] = acc[ni][ki][i];
            }
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

constexpr int kLnbBlocks = 512;

int dw_chunks(int64_t rows) {
    // >= 256 rows per chunk, at most 64 chunks: the partial slab stays small and the column sum short
    int64_t c = rows / 256;
    if (c > 64) c = 64;
    if (c < 1) c = 1;
    return (int)c;
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
    MMNI_ARG_CHECK(aux == nullptr || d->ldaux >= d->N, "rowgemm: aux leading dimension below N");
    MMNI_ARG_CHECK(res == nullptr || d->ldres >= d->N, "rowgemm: residual leading dimension below N");
    enc::RGArgs a{};
    a.rows = d->rows; a.ldx = d->ldx; a.ldy = d->ldy; a.ldres = d->ldres; a.ldaux = d->ldaux;
    a.w_sn = d->w_sn; a.w_sk = d->w_sk; a.K = d->K; a.N = d->N; a.ln = d->ln; a.relu = d->relu; a.eps = d->eps;
    a.x = x; a.gamma = gamma; a.beta = beta; a.w = w; a.bias = bias; a.aux = aux; a.res = res; a.y = y;
    a.mean = d->ln ? mean : nullptr; a.rstd = d->ln ? rstd : nullptr;
    const dim3 grid((unsigned)((d->rows + enc::BM - 1) / enc::BM), (unsigned)((d->N + enc::BN - 1) / enc::BN));
    enc::rowgemm_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return launch_status("rowgemm");
}

extern "C" size_t mmni_rowgemm_dw_workspace_bytes(const mmni_rowgemm_desc* d) {
    if (d == nullptr || d->rows <= 0 || d->K <= 0 || d->N <= 0) return 0;
    return (size_t)enc::dw_chunks(d->rows) * ((size_t)d->N * d->K + d->N) * sizeof(float);
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
    const int chunks = enc::dw_chunks(d->rows);
    a.rows_per_chunk = (int)((d->rows + chunks - 1) / chunks);
    a.x = x; a.gamma = gamma; a.beta = beta; a.mean = mean; a.rstd = rstd; a.dy = dy;
    a.part = static_cast<float*>(workspace);
    const dim3 grid((unsigned)((d->N + enc::BN - 1) / enc::BN), (unsigned)((d->K + 1 + enc::BN - 1) / enc::BN),
                    (unsigned)chunks);
    enc::rowgemm_dw_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a);
    int rc = launch_status("rowgemm_dw");
    if (rc) return rc;
    ColSegs segs{};
    segs.n = 2;
    segs.end[0] = d->N * d->K;
    segs.end[1] = d->N * d->K + d->N;
    segs.dst[0] = dw;
    segs.dst[1] = db;   // null: the bias gradient is dropped
    segs.accumulate = 0;
    column_sum_segs(a.part, chunks, d->N * d->K + d->N, segs, (hipStream_t)stream);
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
    ColSegs segs{};
    segs.n = 2;
    segs.end[0] = C;
    segs.end[1] = 2 * C;
    segs.dst[0] = dgamma;
    segs.dst[1] = dbeta;
    segs.accumulate = 0;
    column_sum_segs(a.part, (int)blocks, 2 * C, segs, (hipStream_t)stream);
    return launch_status("row_layernorm_bwd_sum");
}
