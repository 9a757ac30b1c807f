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
constexpr int DEPTH = 4;     // groups in flight (LN rows, weight gradient)
constexpr int SDEPTH = 8;    // groups in flight for plain rows: 7 groups (~3.5k cycles of MFMA) cover a
                             // first-touch HBM latency at ~1 wave per SIMD

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

// Operand loads are branch-free and select-free: an element outside the tensor (row past the
// end, k past K, n past N) is read from a 16-byte zero page instead, so every load is
// unconditional and its value is first touched by the MFMA that consumes it.  (Loads under per-lane
// branches got a full vmcnt(0) wait each, and a select right after a load pins the wait there too:
// both serialised the DEPTH groups that are meant to be in flight.)
__device__ __attribute__((aligned(16))) float g_zero4[4];

// VEC: K, the leading dimension and the base are multiples of 4 floats (16-byte pieces).
// 4 consecutive k (from k0) of row r (rok = the row exists); zeros past K
template <bool VEC>
__device__ __forceinline__ f4 load_k4(const float* base, int64_t r, int64_t ld, bool rok, int k0, int K) {
    if constexpr (VEC) {
        // k0 and K are multiples of 4: k0 < K means all four are in
        const float* p = (rok && k0 < K) ? base + r * ld + k0 : g_zero4;
        return *reinterpret_cast<const f4*>(p);
    } else {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *((rok && k0 + i < K) ? base + r * ld + k0 + i : g_zero4);
        return v;
    }
}

// W(n, k0 .. k0 + 3): k-contiguous (an nn.Linear weight) as load_k4, or n-contiguous (TW, the
// transpose for dX = dY W) as four scalars of rows k0 .. k0 + 3 (16 lanes of a group read 16
// consecutive n: 64-byte pieces)
template <bool VEC, bool TW>
__device__ __forceinline__ f4 load_w4(const RGArgs& a, int n, int k0) {
    const bool nok = n < a.N;
    if constexpr (!TW) {
        return load_k4<VEC>(a.w, n, a.w_sn, nok, k0, a.K);
    } else {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            v[i] = *((nok && k0 + i < a.K) ? a.w + (int64_t)(k0 + i) * a.w_sk + n : g_zero4);
        return v;
    }
}

struct Tile {
    f4 acc[2][2];   // [m tile][n tile], D[row 4 g + i][col t]
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
    }
    // one group: 4 k-steps x (2 x 2) tiles, four independent accumulator chains
    __device__ __forceinline__ void group(f4 xa, f4 xb, f4 wa, f4 wb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[0][0] = mfma(xa[i], wa[i], acc[0][0]);
            acc[0][1] = mfma(xa[i], wb[i], acc[0][1]);
            acc[1][0] = mfma(xb[i], wa[i], acc[1][0]);
            acc[1][1] = mfma(xb[i], wb[i], acc[1][1]);
        }
    }
};

// Plain rows: X and W stream through a D-slot register ring over groups [g0, g0 + ng).  Whole laps
// of D groups run in a loop with no exits (a slot is refilled right after its MFMAs, so the ring
// keeps its registers and the wait before each group leaves the other D - 1 groups in flight), the
// ng % D tail after it.
template <bool VEC, bool TW, int D>
__device__ __forceinline__ void stream_rows(const RGArgs& a, Tile& T, int64_t ra, int64_t rb, bool oka, bool okb,
                                            int na, int nb, int g, int g0, int ng) {
    f4 xa[D], xb[D], wa[D], wb[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int k0 = KG * (g0 + d) + 4 * g;   // groups past K load as zeros
        xa[d] = load_k4<VEC>(a.x, ra, a.ldx, oka, k0, a.K);
        xb[d] = load_k4<VEC>(a.x, rb, a.ldx, okb, k0, a.K);
        wa[d] = load_w4<VEC, TW>(a, na, k0);
        wb[d] = load_w4<VEC, TW>(a, nb, k0);
    }
    const int laps = ng / D;
    for (int l = 0; l < laps; ++l) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            T.group(xa[d], xb[d], wa[d], wb[d]);
            const int k0 = KG * (g0 + (l + 1) * D + d) + 4 * g;
            xa[d] = load_k4<VEC>(a.x, ra, a.ldx, oka, k0, a.K);
            xb[d] = load_k4<VEC>(a.x, rb, a.ldx, okb, k0, a.K);
            wa[d] = load_w4<VEC, TW>(a, na, k0);
            wb[d] = load_w4<VEC, TW>(a, nb, k0);
        }
    }
    const int rem = ng - laps * D;
#pragma unroll
    for (int d = 0; d < D - 1; ++d)
        if (d < rem) T.group(xa[d], xb[d], wa[d], wb[d]);
}

// LayerNorm rows (K <= KMAX_LN): the two rows' whole K extent in registers (NG groups, a template
// constant so every index is static and nothing branches), statistics by the 4 lane groups, and
// W, gamma, beta streaming through the ring; the W / gamma / beta prologue is issued before the
// statistics so it lands while they are computed.
template <bool VEC, int NG>
__device__ __forceinline__ void ln_rows(const RGArgs& a, Tile& T, int64_t ra, int64_t rb, bool oka, bool okb,
                                        int na, int nb, int g, bool write_stats) {
    f4 xa[NG], xb[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
        xa[j] = load_k4<VEC>(a.x, ra, a.ldx, oka, KG * j + 4 * g, a.K);
        xb[j] = load_k4<VEC>(a.x, rb, a.ldx, okb, KG * j + 4 * g, a.K);
    }
    constexpr int D = NG < DEPTH ? NG : DEPTH;
    f4 wa[D], wb[D], ga[D], be[D];
    auto refill = [&](int slot, int j) {
        const int k0 = KG * j + 4 * g;   // zeros past K
        wa[slot] = load_w4<VEC, false>(a, na, k0);
        wb[slot] = load_w4<VEC, false>(a, nb, k0);
        ga[slot] = load_k4<VEC>(a.gamma, 0, 0, true, k0, a.K);
        be[slot] = load_k4<VEC>(a.beta, 0, 0, true, k0, a.K);
    };
#pragma unroll
    for (int d = 0; d < D; ++d) refill(d, d);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
        sa += (xa[j][0] + xa[j][1]) + (xa[j][2] + xa[j][3]);
        sb += (xb[j][0] + xb[j][1]) + (xb[j][2] + xb[j][3]);
    }
    sa += __shfl_xor(sa, 16); sa += __shfl_xor(sa, 32);
    sb += __shfl_xor(sb, 16); sb += __shfl_xor(sb, 32);
    const float invK = 1.0f / (float)a.K;
    const float ma = sa * invK, mb = sb * invK;
    float va = 0.f, vb = 0.f;
#pragma unroll
    for (int j = 0; j < NG; ++j)
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
    if (write_stats && g == 0) {
        if (oka) { a.mean[ra] = ma; a.rstd[ra] = rsa; }
        if (okb) { a.mean[rb] = mb; a.rstd[rb] = rsb; }
    }
#pragma unroll
    for (int j = 0; j < NG; ++j) {
        const int s = j % D;
        f4 xna, xnb;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            xna[i] = fmaf((xa[j][i] - ma) * rsa, ga[s][i], be[s][i]);
            xnb[i] = fmaf((xb[j][i] - mb) * rsb, ga[s][i], be[s][i]);
        }
        T.group(xna, xnb, wa[s], wb[s]);
        if (j + D < NG) refill(s, j + D);   // compile-time condition
    }
}

// KS = 1: a workgroup owns 64 rows x 64 outputs (2 x 2 waves of 32 x 32).  KS = 2 / 4 (long K, few
// output tiles): the 4 waves split K instead — 32 rows x 64 outputs with 2 K-halves, or 32 x 32 with
// 4 K-quarters — and the partial tiles are added through LDS in K order (deterministic), so a
// 6,912-row GEMM with N = 84 runs ~2,600 waves instead of ~650.
template <bool LN, bool VEC, bool TW, int KS>
__global__ __launch_bounds__(256) void rowgemm_kernel(RGArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = lane & 15, g = lane >> 4;
    constexpr int BMK = KS == 1 ? 64 : 32, BNK = KS == 4 ? 32 : 64;
    const int mw = KS == 1 ? (wave & 1) : 0;
    const int nw = KS == 1 ? (wave >> 1) : (KS == 2 ? (wave & 1) : 0);
    const int kp = KS == 1 ? 0 : (KS == 2 ? (wave >> 1) : wave);
    const int64_t m0 = (int64_t)blockIdx.x * BMK + mw * 32;             // the wave's 32 rows
    const int n0 = blockIdx.y * BNK + nw * 32;                         // and 32 outputs
    const int64_t ra = m0 + t, rb = m0 + 16 + t;                       // A rows of the two m tiles
    const bool oka = ra < a.rows, okb = rb < a.rows;
    const int na = n0 + t, nb = n0 + 16 + t;                           // B columns of the two n tiles
    const bool active = m0 < a.rows && n0 < a.N;
    if (KS == 1 && !active) return;   // a wave wholly past the edge (KS = 1 has no barrier)
    const int NG = (a.K + KG - 1) / KG;
    Tile T;
    T.zero();
    if constexpr (LN) {
        const bool ws = a.mean != nullptr && blockIdx.y == 0 && (wave >> 1) == 0;
        switch (NG) {
#define MMNI_LN_CASE(n) case n: ln_rows<VEC, n>(a, T, ra, rb, oka, okb, na, nb, g, ws); break;
            MMNI_LN_CASE(1) MMNI_LN_CASE(2) MMNI_LN_CASE(3) MMNI_LN_CASE(4) MMNI_LN_CASE(5) MMNI_LN_CASE(6)
            MMNI_LN_CASE(7) MMNI_LN_CASE(8) MMNI_LN_CASE(9) MMNI_LN_CASE(10) MMNI_LN_CASE(11)
#undef MMNI_LN_CASE
            default: break;   // K > KMAX_LN is refused by the host
        }
    } else if constexpr (KS == 1) {
        stream_rows<VEC, TW, SDEPTH>(a, T, ra, rb, oka, okb, na, nb, g, 0, NG);
    } else {
        const int per = (NG + KS - 1) / KS, g0 = kp * per;
        const int ng = NG - g0 < per ? NG - g0 : per;
        if (active && ng > 0) stream_rows<VEC, TW, DEPTH>(a, T, ra, rb, oka, okb, na, nb, g, g0, ng);
        // K parts 1 .. KS-1 hand their tiles to part 0 through LDS; part 0 adds them in order
        __shared__ f4 red[3][4][64];
        const int slot = nw * (KS - 1) + kp - 1;
        if (kp > 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) red[slot][i][lane] = T.acc[i >> 1][i & 1];
        }
        __syncthreads();
        if (kp > 0 || !active) return;
#pragma unroll
        for (int p = 0; p < KS - 1; ++p)
#pragma unroll
            for (int i = 0; i < 4; ++i) T.acc[i >> 1][i & 1] += red[nw * (KS - 1) + p][i][lane];
    }
    auto& acc = T.acc;
    // epilogue: D[row 4 g + i][col t] of tile (mi, ni).  The residual / ReLU-mask operands load
    // unconditionally first (absent ones read y's first row, clamped addresses; the host passes
    // ld 0) and are selected, so the stores wait once, not per element.
    const bool has_aux = a.aux != nullptr, has_res = a.res != nullptr;
    const float* auxp = has_aux ? a.aux : a.y;
    const float* resp = has_res ? a.res : a.y;
    float ev[2][2][4], rv[2][2][4];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        const int n = n0 + 16 * ni + t;
        const int nc = n < a.N ? n : a.N - 1;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = m0 + 16 * mi + 4 * g + i;
                const int64_t rc = r < a.rows ? r : a.rows - 1;
                ev[ni][mi][i] = auxp[rc * a.ldaux + nc];
                rv[ni][mi][i] = resp[rc * a.ldres + nc];
            }
    }
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        const int n = n0 + 16 * ni + t;
        const float b = a.bias ? a.bias[n < a.N ? n : a.N - 1] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = m0 + 16 * mi + 4 * g + i;
                float v = acc[mi][ni][i] + b;
                if (a.relu) v = fmaxf(v, 0.f);
                if (has_aux && !(ev[ni][mi][i] > 0.f)) v = 0.f;
                if (has_res) v += rv[ni][mi][i];
                if (r < a.rows && n < a.N) a.y[r * a.ldy + n] = v;
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

// rows r0 .. r0 + 3 of column c (scalars; the 16 lanes of a group read 16 consecutive columns of
// each row); the zero page past the chunk end / past C
__device__ __forceinline__ f4 load_rows4(const float* base, int64_t ld, int64_t r0, int64_t rend, int c, int C) {
    f4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = *((r0 + i < rend && c < C) ? base + (r0 + i) * ld + c : g_zero4);
    return v;
}

// the row statistics of rows r0 .. r0 + 3 (zero page past the chunk: those rows are masked later)
__device__ __forceinline__ f4 load_stat4(const float* p, int64_t r0, int64_t rend) {
    f4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = *(r0 + i < rend ? p + r0 + i : g_zero4);
    return v;
}

template <bool LN>
__global__ __launch_bounds__(256) void rowgemm_dw_kernel(DWArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = lane & 15, g = lane >> 4;
    const int n0 = blockIdx.x * BN + (wave & 1) * 32, k0 = blockIdx.y * BN + (wave >> 1) * 32;
    const int64_t rbeg = (int64_t)blockIdx.z * a.rows_per_chunk;
    const int64_t rend = rbeg + a.rows_per_chunk < a.rows ? rbeg + a.rows_per_chunk : a.rows;
    if (n0 >= a.N || k0 > a.K) return;   // a wave wholly past the edge (its partials are never read)
    const int na = n0 + t, nb = n0 + 16 + t, ka = k0 + t, kb = k0 + 16 + t;
    // X' columns ka, kb: LN affine per column (hoisted), the ones column k == K (db), zeros past it
    const float ga = LN ? a.gamma[ka < a.K ? ka : a.K - 1] : 1.f, ba = LN ? a.beta[ka < a.K ? ka : a.K - 1] : 0.f;
    const float gb = LN ? a.gamma[kb < a.K ? kb : a.K - 1] : 1.f, bb = LN ? a.beta[kb < a.K ? kb : a.K - 1] : 0.f;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
    // raw X -> X' at the consuming step (k >= K reads the zero page; the ones column set here)
    auto xform = [&](f4 xv, f4 m, f4 rs, int64_t r, int k, float gk, float bk) {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float xn = LN ? fmaf((xv[i] - m[i]) * rs[i], gk, bk) : xv[i];
            xn = k < a.K ? xn : (k == a.K ? 1.f : 0.f);
            v[i] = r + i < rend ? xn : 0.f;
        }
        return v;
    };
    const int NG = (int)((rend - rbeg + KG - 1) / KG);
    f4 da[DEPTH], db[DEPTH], xa[DEPTH], xb[DEPTH], mr[DEPTH], rr[DEPTH];
    auto issue = [&](int d, int64_t r) {
        da[d] = load_rows4(a.dy, a.lddy, r, rend, na, a.N);
        db[d] = load_rows4(a.dy, a.lddy, r, rend, nb, a.N);
        xa[d] = load_rows4(a.x, a.ldx, r, rend, ka, a.K);
        xb[d] = load_rows4(a.x, a.ldx, r, rend, kb, a.K);
        if (LN) {
            mr[d] = load_stat4(a.mean, r, rend);
            rr[d] = load_stat4(a.rstd, r, rend);
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) issue(d, rbeg + KG * d + 4 * g);   // rows past the chunk: zeros
    // A[row n][kk = row]: dY;  B[kk = row][col k]: X'.  Whole laps in an exit-free loop, slots
    // refilled after their MFMAs (as stream_rows), then the tail.
    auto step = [&](int d, int j) {
        const int64_t r = rbeg + KG * j + 4 * g;
        const f4 cxa = xform(xa[d], mr[d], rr[d], r, ka, ga, ba), cxb = xform(xb[d], mr[d], rr[d], r, kb, gb, bb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[0][0] = mfma(da[d][i], cxa[i], acc[0][0]);
            acc[0][1] = mfma(da[d][i], cxb[i], acc[0][1]);
            acc[1][0] = mfma(db[d][i], cxa[i], acc[1][0]);
            acc[1][1] = mfma(db[d][i], cxb[i], acc[1][1]);
        }
    };
    const int laps = NG / DEPTH;
    for (int l = 0; l < laps; ++l) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            step(d, l * DEPTH + d);
            issue(d, rbeg + KG * ((l + 1) * DEPTH + d) + 4 * g);
        }
    }
    const int rem = NG - laps * DEPTH;
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
        if (d < rem) step(d, laps * DEPTH + d);
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

// out[j] = sum_c part[c][j] (deterministic: fixed slices and a fixed tree); columns [0, split) ->
// out, [split, ncols) -> out2 (nullable).  A block owns Q float4 column quads and splits the chunks
// over SL = 256 / Q slices (slice s sums chunks s, s + SL, ... in order, 8 loads in flight), then
// adds the slices by a fixed LDS tree.  Q = 8 for wide slabs (weight gradients); Q = 2 for narrow
// ones (a LayerNorm's 2C dgamma | dbeta columns over 768 chunks: 6 blocks of 32 columns took
// ~9.4 us a call, 21 blocks of 8 columns one load round).  One thread per column quad looping over
// 100+ chunks was a chain of dependent load waits (~10 us per call).
template <int Q>
__global__ __launch_bounds__(256) void chunk_sum_kernel(const float* __restrict__ part, int nchunks, int ncols,
                                                        int split, float* out, float* out2) {
    constexpr int SL = 256 / Q;
    __shared__ f4 red[SL][Q];
    const int q = threadIdx.x % Q, sl = threadIdx.x / Q;
    const int j4 = (blockIdx.x * Q + q) * 4;
    const bool vec = (ncols & 3) == 0;
    f4 s = zero4();
    for (int c0 = sl; c0 < nchunks; c0 += 8 * SL) {
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = c0 + u * SL;
            const float* p = part + (int64_t)(c < nchunks ? c : nchunks - 1) * ncols;
            if (vec) {
                v[u] = *reinterpret_cast<const f4*>(p + (j4 < ncols ? j4 : ncols - 4));
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[u][i] = p[j4 + i < ncols ? j4 + i : ncols - 1];
            }
            if (c >= nchunks) v[u] = zero4();
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    red[sl][q] = s;
    __syncthreads();
#pragma unroll
    for (int h = SL / 2; h > 0; h >>= 1) {
        if (sl < h) red[sl][q] += red[sl + h][q];
        __syncthreads();
    }
    if (sl == 0) {
        const f4 r = red[0][q];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = j4 + i;
            if (j >= ncols) break;
            if (j < split) out[j] = r[i];
            else if (out2 != nullptr) out2[j - split] = r[i];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm backward on rows of C <= 256: one wave per row, 4 columns per lane
// ---------------------------------------------------------------------------------------------
struct LNBArgs {
    int64_t rows, lddxn, ldx, ldres, lddx;
    int C;
    const void* dxn;   // float, or __bf16 (the bf16 head's linears hand back bf16 input gradients)
    const float* x;
    const float* gamma;
    const float* mean;
    const float* rstd;
    const float* dres;
    float* dx;
    float* part;   // [block][2C]: dgamma | dbeta
};

template <typename TI>
__device__ __forceinline__ float ln_ld(const TI* p) { return (float)*p; }

template <bool RES, typename TI = float>
__global__ __launch_bounds__(256) void row_ln_bwd_kernel(LNBArgs a) {
    __shared__ float red[4][2][256];
    const TI* dxn = static_cast<const TI*>(a.dxn);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f}, gm[4];
    int cc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j;
        cc[j] = c < a.C ? c : a.C - 1;   // clamped column: every load unconditional
        gm[j] = c < a.C ? a.gamma[cc[j]] : 0.f;
    }
    const float invC = 1.0f / (float)a.C;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.rows; r += (int64_t)gridDim.x * 4) {
        const float m = a.mean[r], rs = a.rstd[r];
        float d[4], xv[4], rv[4], xh[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            d[j] = ln_ld<TI>(dxn + r * a.lddxn + cc[j]);
            xv[j] = a.x[r * a.ldx + cc[j]];
            rv[j] = RES ? a.dres[r * a.ldres + cc[j]] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool in = lane + 64 * j < a.C;
            d[j] = in ? d[j] : 0.f;
            xh[j] = in ? (xv[j] - m) * rs : 0.f;
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
            const float v = rs * (d[j] * gm[j] - s1 - xh[j] * s2) + rv[j];
            if (c < a.C) a.dx[r * a.lddx + c] = v;
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

// LayerNorm forward on rows of C <= 256: a wave per row, 4 columns per lane (two butterfly sums:
// mean, then the centred second moment); (mean, rstd) written for the backward.
template <typename TO = float>
__global__ __launch_bounds__(256) void row_ln_fwd_kernel(int64_t rows, int C, const float* __restrict__ x,
                                                         int64_t ldx, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps, TO* y,
                                                         int64_t ldy, float* mean, float* rstd) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float gm[4], bt[4];
    bool in[4];
    const float* zp = g_zero4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j;
        in[j] = c < C;
        gm[j] = *(in[j] ? gamma + c : zp);
        bt[j] = *(in[j] ? beta + c : zp);
    }
    const float invC = 1.0f / (float)C;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += (int64_t)gridDim.x * 4) {
        float v[4], s = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = *(in[j] ? x + r * ldx + lane + 64 * j : zp);
            s += v[j];
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        const float mu = s * invC;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float d = in[j] ? v[j] - mu : 0.f;
            q = fmaf(d, d, q);
        }
        for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
        const float rs = 1.0f / sqrtf(q * invC + eps);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (in[j]) y[r * ldy + lane + 64 * j] = (TO)fmaf((v[j] - mu) * rs, gm[j], bt[j]);
        if (lane == 0) {
            mean[r] = mu;
            rstd[r] = rs;
        }
    }
}

// Quad-lane variants for C % 4 == 0 (the crossmodal widths 84 / 168): a row takes LPR lanes (32 for
// C <= 128, 64 for C <= 256), each holding 4 consecutive columns from one 16-byte load, so a wave
// covers 64 / LPR rows at once (84: two rows of 21 live lanes, against one row of 64 + 20 four-byte
// loads in the scalar kernels).  Row sums: xor butterflies inside the LPR-lane segment.
template <typename TO>
__device__ __forceinline__ void st4(TO* p, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void st4<float>(float* p, float a, float b, float c, float d) {
    *reinterpret_cast<f4*>(p) = (f4){a, b, c, d};
}
template <>
__device__ __forceinline__ void st4<__bf16>(__bf16* p, float a, float b, float c, float d) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<b4*>(p) = (b4){(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
}
template <typename TI>
__device__ __forceinline__ f4 ld4v(const TI* p);
template <>
__device__ __forceinline__ f4 ld4v<float>(const float* p) { return *reinterpret_cast<const f4*>(p); }
template <>
__device__ __forceinline__ f4 ld4v<__bf16>(const __bf16* p) {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    return (f4){__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
                __uint_as_float(q.y & 0xffff0000u)};
}
template <int LPR>
__device__ __forceinline__ float seg_sum(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <typename TO, int LPR>
__global__ __launch_bounds__(256) void row_ln_fwd_q_kernel(int64_t rows, int C, const float* __restrict__ x,
                                                           int64_t ldx, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps, TO* y,
                                                           int64_t ldy, float* mean, float* rstd) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane / LPR, c0 = (lane % LPR) * 4;
    const bool live = c0 < C;
    const f4 gm = live ? *reinterpret_cast<const f4*>(gamma + c0) : zero4();
    const f4 bt = live ? *reinterpret_cast<const f4*>(beta + c0) : zero4();
    const float invC = 1.0f / (float)C;
    for (int64_t rb = ((int64_t)blockIdx.x * 4 + wave) * RPW; rb < rows; rb += (int64_t)gridDim.x * 4 * RPW) {
        const int64_t r = rb + sub;
        const bool ok = live & (r < rows);
        const f4 v = ok ? *reinterpret_cast<const f4*>(x + r * ldx + c0) : zero4();
        const float mu = seg_sum<LPR>((v[0] + v[1]) + (v[2] + v[3])) * invC;
        const f4 d = ok ? v - mu : zero4();
        const float q = seg_sum<LPR>((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]));
        const float rs = 1.0f / sqrtf(q * invC + eps);
        if (ok)
            st4<TO>(y + r * ldy + c0, fmaf(d[0] * rs, gm[0], bt[0]), fmaf(d[1] * rs, gm[1], bt[1]),
                    fmaf(d[2] * rs, gm[2], bt[2]), fmaf(d[3] * rs, gm[3], bt[3]));
        if (c0 == 0 && r < rows) {
            mean[r] = mu;
            rstd[r] = rs;
        }
    }
}

template <bool RES, typename TI, int LPR>
__global__ __launch_bounds__(256) void row_ln_bwd_q_kernel(LNBArgs a) {
    constexpr int RPW = 64 / LPR;
    __shared__ f4 red[4 * RPW][2][64];
    const TI* dxn = static_cast<const TI*>(a.dxn);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane / LPR, cq = lane % LPR, c0 = cq * 4;
    const bool live = c0 < a.C;
    const f4 gm = live ? *reinterpret_cast<const f4*>(a.gamma + c0) : zero4();
    f4 dg = zero4(), db = zero4();
    const float invC = 1.0f / (float)a.C;
    for (int64_t rb = ((int64_t)blockIdx.x * 4 + wave) * RPW; rb < a.rows; rb += (int64_t)gridDim.x * 4 * RPW) {
        const int64_t r = rb + sub;
        const bool ok = live & (r < a.rows);
        const int64_t rr = r < a.rows ? r : a.rows - 1;
        const float m = a.mean[rr], rs = a.rstd[rr];
        f4 d = ok ? ld4v<TI>(dxn + r * a.lddxn + c0) : zero4();
        const f4 xv = ok ? *reinterpret_cast<const f4*>(a.x + r * a.ldx + c0) : zero4();
        f4 rv = zero4();
        if (RES && ok) rv = *reinterpret_cast<const f4*>(a.dres + r * a.ldres + c0);
        const f4 xh = ok ? (xv - m) * rs : zero4();
        const f4 gd = d * gm;
        const float s1 = seg_sum<LPR>((gd[0] + gd[1]) + (gd[2] + gd[3])) * invC;
        const float s2 = seg_sum<LPR>((gd[0] * xh[0] + gd[1] * xh[1]) + (gd[2] * xh[2] + gd[3] * xh[3])) * invC;
        dg += d * xh;
        db += d;
        if (ok) {
            const f4 o = rs * (gd - s1 - xh * s2) + rv;
            *reinterpret_cast<f4*>(a.dx + r * a.lddx + c0) = o;
        }
    }
    red[wave * RPW + sub][0][cq] = dg;
    red[wave * RPW + sub][1][cq] = db;
    __syncthreads();
    float* p = a.part + (int64_t)blockIdx.x * 2 * a.C;
    for (int c = threadIdx.x; c < a.C; c += 256) {
        float tg = 0.f, tb = 0.f;
#pragma unroll
        for (int k = 0; k < 4 * RPW; ++k) {   // fixed order: wave-major, then row group
            tg += red[k][0][c >> 2][c & 3];
            tb += red[k][1][c >> 2][c & 3];
        }
        p[c] = tg;
        p[a.C + c] = tb;
    }
}

constexpr int kLnbBlocks = 768;   // ~2 rows per wave at 6,912 rows: a short dependent chain per wave

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
    if (ncols <= 1024 && nchunks >= 256) {
        chunk_sum_kernel<2><<<(ncols + 7) / 8, 256, 0, s>>>(part, nchunks, ncols, split, out, out2);
    } else {
        chunk_sum_kernel<8><<<(ncols + 31) / 32, 256, 0, s>>>(part, nchunks, ncols, split, out, out2);
    }
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
    if (aux == nullptr) a.ldaux = 0;
    if (res == nullptr) a.ldres = 0;
    const bool tw = d->w_sk != 1;
    const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    // 16-byte operand pieces when every row of x (and of a k-contiguous weight) starts aligned
    const bool vec = d->K % 4 == 0 && d->ldx % 4 == 0 && al(x) && (!d->ln || (al(gamma) && al(beta))) &&
                     (tw || (d->w_sn % 4 == 0 && al(w)));
    hipStream_t s = (hipStream_t)stream;
    // K split across the workgroup's waves when the 32 x 32 output tiles alone leave the SIMDs
    // mostly idle and K is long enough to share (<= 4 waves per SIMD in flight either way)
    const int64_t tiles = ((d->rows + 31) / 32) * ((d->N + 31) / 32);
    const int NG = (d->K + enc::KG - 1) / enc::KG;
    int ks = 1;
    if (!d->ln) {
        if (tiles * 4 <= 4096 && NG >= 12) ks = 4;
        else if (tiles * 2 <= 4096 && NG >= 6) ks = 2;
    }
    const int bm = ks == 1 ? 64 : 32, bn = ks == 4 ? 32 : 64;
    const dim3 grid((unsigned)((d->rows + bm - 1) / bm), (unsigned)((d->N + bn - 1) / bn));
#define MMNI_RG(LN, VEC, TW, KS) enc::rowgemm_kernel<LN, VEC, TW, KS><<<grid, 256, 0, s>>>(a)
#define MMNI_RG_KS(VEC, TW)                                   \
    do {                                                      \
        if (ks == 4) MMNI_RG(false, VEC, TW, 4);              \
        else if (ks == 2) MMNI_RG(false, VEC, TW, 2);         \
        else MMNI_RG(false, VEC, TW, 1);                      \
    } while (0)
    if (d->ln) {
        MMNI_ARG_CHECK(!tw, "rowgemm: the LayerNorm prologue takes a k-contiguous weight");
        if (vec) MMNI_RG(true, true, false, 1); else MMNI_RG(true, false, false, 1);
    } else if (tw) {
        if (vec) MMNI_RG_KS(true, true); else MMNI_RG_KS(false, true);
    } else {
        if (vec) MMNI_RG_KS(true, false); else MMNI_RG_KS(false, false);
    }
#undef MMNI_RG_KS
#undef MMNI_RG
    return launch_status("rowgemm");
}

namespace mmni {

size_t enc_rowgemm_dw_workspace(int64_t rows, int N, int K) {
    return (size_t)enc::dw_chunks(rows, N, K) * ((size_t)N * K + N) * sizeof(float);
}

int enc_rowgemm_dw(int64_t rows, int N, int K, const float* x, int64_t ldx, const float* dy, int64_t lddy,
                   const float* gamma, const float* beta, const float* mean, const float* rstd, float* dw, float* db,
                   void* workspace, hipStream_t s) {
    enc::DWArgs a{};
    a.rows = rows; a.ldx = ldx; a.lddy = lddy; a.K = K; a.N = N; a.ln = gamma != nullptr;
    const int chunks = enc::dw_chunks(rows, N, K);
    a.rows_per_chunk = (int)((rows + chunks - 1) / chunks);
    a.x = x; a.gamma = gamma; a.beta = beta; a.mean = mean; a.rstd = rstd; a.dy = dy;
    a.part = static_cast<float*>(workspace);
    const dim3 grid((unsigned)((N + enc::BN - 1) / enc::BN), (unsigned)((K + 1 + enc::BN - 1) / enc::BN),
                    (unsigned)chunks);
    if (a.ln) enc::rowgemm_dw_kernel<true><<<grid, 256, 0, s>>>(a);
    else enc::rowgemm_dw_kernel<false><<<grid, 256, 0, s>>>(a);
    int rc = launch_status("rowgemm_dw");
    if (rc) return rc;
    // dW = columns [0, N K), db = [N K, N K + N) (a null db drops them)
    enc::chunk_sum(a.part, chunks, N * K + N, N * K, dw, db, s);
    return launch_status("rowgemm_dw_sum");
}

size_t enc_row_ln_bwd_workspace(int64_t rows, int C) {
    int64_t blocks = (rows + 3) / 4;
    if (blocks > enc::kLnbBlocks) blocks = enc::kLnbBlocks;
    return (size_t)blocks * 2 * C * sizeof(float);
}

int enc_row_ln_bwd(int64_t rows, int C, const float* dxn, int64_t lddxn, const float* x, int64_t ldx,
                   const float* gamma, const float* mean, const float* rstd, const float* dres, int64_t ldres,
                   float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace, hipStream_t s) {
    return enc_row_ln_bwd_t(rows, C, dxn, 0, lddxn, x, ldx, gamma, mean, rstd, dres, ldres, dx, lddx, dgamma, dbeta,
                            workspace, s);
}

int enc_row_ln_bwd_t(int64_t rows, int C, const void* dxn, int dxn_bf16, int64_t lddxn, const float* x, int64_t ldx,
                     const float* gamma, const float* mean, const float* rstd, const float* dres, int64_t ldres,
                     float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace, hipStream_t s) {
    enc::LNBArgs a{};
    a.rows = rows; a.lddxn = lddxn; a.ldx = ldx; a.ldres = ldres; a.lddx = lddx; a.C = C;
    a.dxn = dxn; a.x = x; a.gamma = gamma; a.mean = mean; a.rstd = rstd; a.dres = dres; a.dx = dx;
    a.part = static_cast<float*>(workspace);
    int64_t blocks = (rows + 3) / 4;
    if (blocks > enc::kLnbBlocks) blocks = enc::kLnbBlocks;
    const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool quad = C % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 && lddxn % 4 == 0 &&
                      (dres == nullptr || ldres % 4 == 0) && al16(x) && al16(dx) && al16(gamma) &&
                      (reinterpret_cast<uintptr_t>(dxn) & (dxn_bf16 ? 7 : 15)) == 0 && (dres == nullptr || al16(dres));
    if (quad) {
#define MMNI_LNBQ(LPR)                                                                                          \
    do {                                                                                                        \
        if (dxn_bf16) {                                                                                         \
            if (dres != nullptr) enc::row_ln_bwd_q_kernel<true, __bf16, LPR><<<(unsigned)blocks, 256, 0, s>>>(a); \
            else enc::row_ln_bwd_q_kernel<false, __bf16, LPR><<<(unsigned)blocks, 256, 0, s>>>(a);             \
        } else {                                                                                                \
            if (dres != nullptr) enc::row_ln_bwd_q_kernel<true, float, LPR><<<(unsigned)blocks, 256, 0, s>>>(a);  \
            else enc::row_ln_bwd_q_kernel<false, float, LPR><<<(unsigned)blocks, 256, 0, s>>>(a);              \
        }                                                                                                       \
    } while (0)
        if (C <= 128) MMNI_LNBQ(32);
        else MMNI_LNBQ(64);
#undef MMNI_LNBQ
    } else if (dxn_bf16) {
        if (dres != nullptr) enc::row_ln_bwd_kernel<true, __bf16><<<(unsigned)blocks, 256, 0, s>>>(a);
        else enc::row_ln_bwd_kernel<false, __bf16><<<(unsigned)blocks, 256, 0, s>>>(a);
    } else {
        if (dres != nullptr) enc::row_ln_bwd_kernel<true><<<(unsigned)blocks, 256, 0, s>>>(a);
        else enc::row_ln_bwd_kernel<false><<<(unsigned)blocks, 256, 0, s>>>(a);
    }
    int rc = launch_status("row_layernorm_bwd");
    if (rc) return rc;
    enc::chunk_sum(a.part, (int)blocks, 2 * C, C, dgamma, dbeta, s);
    return launch_status("row_layernorm_bwd_sum");
}

}  // namespace mmni

extern "C" size_t mmni_rowgemm_dw_workspace_bytes(const mmni_rowgemm_desc* d) {
    if (d == nullptr || d->rows <= 0 || d->K <= 0 || d->N <= 0) return 0;
    return enc_rowgemm_dw_workspace(d->rows, d->N, d->K);
}

extern "C" int mmni_rowgemm_dw(const mmni_rowgemm_desc* d, const float* x, const float* gamma, const float* beta,
                               const float* mean, const float* rstd, const float* dy, float* dw, float* db,
                               void* workspace, void* stream) {
    MMNI_ARG_CHECK(d != nullptr && x && dy && dw && workspace, "rowgemm_dw: null descriptor or pointer");
    MMNI_ARG_CHECK(d->rows > 0 && d->K > 0 && d->N > 0, "rowgemm_dw: bad extents");
    MMNI_ARG_CHECK(d->ldx >= d->K && d->ldy >= d->N, "rowgemm_dw: leading dimensions below K / N (ldy: dY)");
    MMNI_ARG_CHECK(!d->ln || (gamma && beta && mean && rstd), "rowgemm_dw: LayerNorm recompute needs its inputs");
    return enc_rowgemm_dw(d->rows, d->N, d->K, x, d->ldx, dy, d->ldy, d->ln ? gamma : nullptr, beta, mean, rstd, dw,
                          db, workspace, (hipStream_t)stream);
}

extern "C" size_t mmni_row_layernorm_bwd_workspace_bytes(int64_t rows, int C) {
    return enc_row_ln_bwd_workspace(rows, C);
}

extern "C" int mmni_row_layernorm_bwd(int64_t rows, int C, const float* dxn, int64_t lddxn, const float* x,
                                      int64_t ldx, const float* gamma, const float* mean, const float* rstd,
                                      const float* dres, int64_t ldres, float* dx, int64_t lddx, float* dgamma,
                                      float* dbeta, void* workspace, void* stream) {
    return mmni_row_layernorm_bwd_t(rows, C, dxn, 0, lddxn, x, ldx, gamma, mean, rstd, dres, ldres, dx, lddx, dgamma,
                                    dbeta, workspace, stream);
}

extern "C" int mmni_row_layernorm_bwd_t(int64_t rows, int C, const void* dxn, int dxn_dtype, int64_t lddxn,
                                        const float* x, int64_t ldx, const float* gamma, const float* mean,
                                        const float* rstd, const float* dres, int64_t ldres, float* dx, int64_t lddx,
                                        float* dgamma, float* dbeta, void* workspace, void* stream) {
    MMNI_ARG_CHECK(dxn && x && gamma && mean && rstd && dx && dgamma && dbeta && workspace,
                   "row_layernorm_bwd: null pointer");
    MMNI_ARG_CHECK(rows > 0 && C > 0 && C <= 256, "row_layernorm_bwd: C=%d outside 1..256", C);
    MMNI_ARG_CHECK(lddxn >= C && ldx >= C && lddx >= C && (dres == nullptr || ldres >= C),
                   "row_layernorm_bwd: leading dimensions below C");
    MMNI_ARG_CHECK(dxn_dtype == 0 || dxn_dtype == 1, "row_layernorm_bwd: dxn dtype %d (0 fp32, 1 bf16)", dxn_dtype);
    return enc_row_ln_bwd_t(rows, C, dxn, dxn_dtype, lddxn, x, ldx, gamma, mean, rstd, dres, ldres, dx, lddx, dgamma,
                            dbeta, workspace, (hipStream_t)stream);
}

extern "C" int mmni_row_layernorm_fwd(int64_t rows, int C, const float* x, int64_t ldx, const float* gamma,
                                      const float* beta, float eps, float* y, int64_t ldy, float* mean, float* rstd,
                                      void* stream) {
    return mmni_row_layernorm_fwd_t(rows, C, x, ldx, gamma, beta, eps, y, 0, ldy, mean, rstd, stream);
}

extern "C" int mmni_row_layernorm_fwd_t(int64_t rows, int C, const float* x, int64_t ldx, const float* gamma,
                                        const float* beta, float eps, void* y, int y_dtype, int64_t ldy, float* mean,
                                        float* rstd, void* stream) {
    MMNI_ARG_CHECK(x && gamma && beta && y && mean && rstd, "row_layernorm_fwd: null pointer");
    MMNI_ARG_CHECK(rows > 0 && C > 0 && C <= 256, "row_layernorm_fwd: C=%d outside 1..256", C);
    MMNI_ARG_CHECK(ldx >= C && ldy >= C, "row_layernorm_fwd: leading dimensions below C");
    MMNI_ARG_CHECK(y_dtype == 0 || y_dtype == 1, "row_layernorm_fwd: y dtype %d (0 fp32, 1 bf16)", y_dtype);
    int64_t blocks = (rows + 7) / 8;   // ~2 rows per wave
    if (blocks > 4096) blocks = 4096;
    hipStream_t s = (hipStream_t)stream;
    const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) && al16(gamma) && al16(beta) &&
        (reinterpret_cast<uintptr_t>(y) & (y_dtype == 1 ? 7 : 15)) == 0) {
        int64_t qb = (rows + (C <= 128 ? 7 : 3)) / (C <= 128 ? 8 : 4);   // one row group per wave
        if (qb > 4096) qb = 4096;
#define MMNI_LNFQ(TO, LPR)                                                                                      \
    enc::row_ln_fwd_q_kernel<TO, LPR><<<(unsigned)qb, 256, 0, s>>>(rows, C, x, ldx, gamma, beta, eps,             \
                                                                   static_cast<TO*>(y), ldy, mean, rstd)
        if (y_dtype == 1) {
            if (C <= 128) MMNI_LNFQ(__bf16, 32);
            else MMNI_LNFQ(__bf16, 64);
        } else {
            if (C <= 128) MMNI_LNFQ(float, 32);
            else MMNI_LNFQ(float, 64);
        }
#undef MMNI_LNFQ
        return launch_status("row_layernorm_fwd");
    }
    if (y_dtype == 1)
        enc::row_ln_fwd_kernel<__bf16><<<(unsigned)blocks, 256, 0, s>>>(rows, C, x, ldx, gamma, beta, eps,
                                                                         static_cast<__bf16*>(y), ldy, mean, rstd);
    else
        enc::row_ln_fwd_kernel<float><<<(unsigned)blocks, 256, 0, s>>>(rows, C, x, ldx, gamma, beta, eps,
                                                                        static_cast<float*>(y), ldy, mean, rstd);
    return launch_status("row_layernorm_fwd");
}
