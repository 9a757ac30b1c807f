// Fused token ops around the window attention of a SwinFusion block,
// C = 12 channels, on the f32 MFMA (tile maps: tokentile.h).
//
// Replaces, per SwinTransformerBlock_fusion (modules/swinfusion_module.py:340-380):
//   norm1 + attn.qkv  (swinfusion_module.py:346, 121)   -> ln_linear_fwd   x -> qkv, (mean, rstd)
//   backward of both + the residual gradient            -> ln_linear_bwd   dqkv, x, dres -> dx, dW, db, dgamma, dbeta
//   backward of attn.proj (swinfusion_module.py:143)    -> linear_bwd      dy, o -> do, dW, db
// The LayerNorm output is never stored: the backward recomputes it from x and the saved
// (mean, rstd), so the qkv weight gradient, the qkv input gradient, the LayerNorm backward and
// the residual add that autograd would issue separately are one pass over the token rows.
// Weight / affine gradients are per-wave partials reduced in a fixed order (column_sum):
// deterministic.
#include "tokentile.h"

namespace mmni {
namespace blk {

using namespace tt;

constexpr int kLlfU = 4;   // tiles per step, ln_linear_fwd
constexpr int kLlbU = 2;   // tiles per step, ln_linear_bwd (N = 12, 24)
// N = 36 keeps one tile per step: two would take it to 2 waves / SIMD (measured 270 vs 257 us)
constexpr int llb_u(int n) { return n == 36 ? 1 : kLlbU; }
// N > 12: ln_linear_fwd stages its outputs and ln_linear_bwd its dy tiles through LDS (N = 12
// rows are 48 B: the accumulator layout already writes / reads them whole)

struct TokArgs {
    int64_t rows;
    float eps;
    const float* x;      // (rows, C)
    const float* gamma;  // (C)
    const float* beta;   // (C)
    const float* w;      // (N, C) nn.Linear weight
    const float* b;      // (N) or null
    float* y;            // fwd: (rows, N)
    float* mean;         // (rows)
    float* rstd;         // (rows)
    const float* dy;     // bwd: (rows, N)
    const float* dres;   // bwd: (rows, C) residual gradient added to dx, or null
    const float* dres2;  // bwd: a second one (the residual group's skip), or null
    float* dx;           // bwd: (rows, C)
    float* partA;        // [waves][N*C + N (+ 2C)]  dW | db (| dgamma | dbeta)
    float* partB;        // unused (dgamma | dbeta follow dW | db in partA's rows)
};

// ------------------------------------------------------------------------------------
// y = LN(x) W^T + b, per 16-token tile: LN on the feature-major operand, NT MFMA output tiles
// ------------------------------------------------------------------------------------
template <int N, int U>
__global__ __launch_bounds__(256) void ln_linear_fwd_kernel(TokArgs a) {
    constexpr int NT = (N + 15) / 16;
    const int lane = threadIdx.x & 63;
    const Tile tl{a.rows, lane & 15, lane >> 4};
    const int t = tl.t, g = tl.g;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float wa[NT][CS], gm[CS], bt[CS];
    f4 bc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int n = nt * 16 + t;
#pragma unroll
        for (int s = 0; s < CS; ++s) wa[nt][s] = n < N ? a.w[n * C + 4 * s + g] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int nr = nt * 16 + 4 * g + i;
            bc[nt][i] = (a.b && nr < N) ? a.b[nr] : 0.f;
        }
    }
#pragma unroll
    for (int s = 0; s < CS; ++s) { gm[s] = a.gamma[4 * s + g]; bt[s] = a.beta[4 * s + g]; }
    __shared__ __attribute__((aligned(16))) float ys_all[N > 12 ? 4 * 16 * N : 4];
    float* ys = ys_all + (N > 12 ? (threadIdx.x >> 6) * 16 * N : 0);
    const int64_t tiles = (a.rows + 15) / 16;
    // U consecutive tiles per step: their loads are issued together (one tile's 768 B per wave
    // in flight leaves the HBM latency exposed at this register budget)
    for (int64_t tb = wave * U; tb < tiles; tb += nwaves * U) {
        float v[U][CS];
#pragma unroll
        for (int u = 0; u < U; ++u) tl.load_fm<CS, C>(a.x, (tb + u) * 16, v[u]);   // rows past the end load 0
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t0 = (tb + u) * 16;
            float mean, rstd;
            ln_stats(v[u], a.eps, mean, rstd);
            float xn[CS];
#pragma unroll
            for (int s = 0; s < CS; ++s) xn[s] = fmaf((v[u][s] - mean) * rstd, gm[s], bt[s]);
            const bool ok = tl.token_ok(t0);
            if constexpr (N > 12) {
                // the tile's 16 x N outputs go through the wave's LDS slab, then out as contiguous
                // 16-B stores (the accumulator layout writes each token row in N / 16 pieces)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    f4 acc = bc[nt];
#pragma unroll
                    for (int s = 0; s < CS; ++s) acc = mfma(wa[nt][s], xn[s], acc);
                    if (nt * 16 + 4 * g < N) *reinterpret_cast<f4*>(ys + t * N + nt * 16 + 4 * g) = acc;
                }
                const int64_t nvec = (a.rows - t0 < 16 ? a.rows - t0 : 16) * (N / 4);
#pragma unroll
                for (int k = 0; k < (4 * N + 63) / 64; ++k) {
                    const int e = k * 64 + lane;
                    if (e < nvec) *reinterpret_cast<f4*>(a.y + t0 * N + 4 * e) = *reinterpret_cast<const f4*>(ys + 4 * e);
                }
            } else {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    f4 acc = bc[nt];
#pragma unroll
                    for (int s = 0; s < CS; ++s) acc = mfma(wa[nt][s], xn[s], acc);
                    if (ok && nt * 16 + 4 * g < N) *reinterpret_cast<f4*>(a.y + (t0 + t) * N + nt * 16 + 4 * g) = acc;
                }
            }
            if (ok && g == 0) {
                a.mean[t0 + t] = mean;
                a.rstd[t0 + t] = rstd;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// dx = LN_bwd(dy W) + dres;  dW = dy^T LN(x),  db = colsum dy,  dgamma, dbeta
// ------------------------------------------------------------------------------------
template <int N, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(N == 36 ? 3 : 1)))
void ln_linear_bwd_kernel(TokArgs a) {
    constexpr int NT = (N + 15) / 16;
    constexpr int NS = N / 4;   // k-steps over the N gradient columns
    constexpr bool kEarlyRes = N == 36;   // (N = 12 would drop to 3 waves / SIMD)
    const int lane = threadIdx.x & 63;
    const Tile tl{a.rows, lane & 15, lane >> 4};
    const int t = tl.t, g = tl.g;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float wt[NS];                 // W^T[c = t][n = 4 s + g]
#pragma unroll
    for (int s = 0; s < NS; ++s) wt[s] = t < C ? a.w[(4 * s + g) * C + t] : 0.f;
    f4 gm4, bt4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        gm4[i] = g < 3 ? a.gamma[4 * g + i] : 0.f;
        bt4[i] = g < 3 ? a.beta[4 * g + i] : 0.f;
    }
    const float gmt = t < C ? a.gamma[t] : 0.f, btt = t < C ? a.beta[t] : 0.f;
    f4 dw[NT], dg = zero4(), dbt = zero4();
    float db[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) { dw[nt] = zero4(); db[nt] = 0.f; }

    constexpr bool kDyLds = N > 12;
    constexpr int DYV = (4 * N + 63) / 64;   // 16-B vectors per lane per dy tile
    __shared__ __attribute__((aligned(16))) float dys_all[kDyLds ? 4 * U * 16 * N : 4];
    float* dys = dys_all + (kDyLds ? (threadIdx.x >> 6) * U * 16 * N : 0);
    const int64_t tiles = (a.rows + 15) / 16;
    // U consecutive tiles per step, all loads first (see ln_linear_fwd_kernel)
    for (int64_t tb = wave * U; tb < tiles; tb += nwaves * U) {
        float dyb[U][NS], xa[U][4], mt[U][4], rt[U][4], dya[U][NT][4], mu[U], ru[U];
        f4 xc[U], rs[U], rs2[U];
        if constexpr (kDyLds) {
            // dy tiles (16 x N floats, contiguous) in with 16-B loads, both operand maps out of LDS
            f4 dv[U][DYV];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t t0 = (tb + u) * 16;
                const int64_t nvec = (a.rows - t0 < 16 ? a.rows - t0 : 16) * (N / 4);
#pragma unroll
                for (int k = 0; k < DYV; ++k) {
                    const int e = k * 64 + lane;
                    dv[u][k] = e < nvec ? *reinterpret_cast<const f4*>(a.dy + t0 * N + 4 * e) : zero4();
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < DYV; ++k) {
                    const int e = k * 64 + lane;
                    if (e < 4 * N) *reinterpret_cast<f4*>(dys + u * 16 * N + 4 * e) = dv[u][k];
                }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float* ds = dys + u * 16 * N;
#pragma unroll
                for (int s = 0; s < NS; ++s) dyb[u][s] = ds[t * N + 4 * s + g];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int s = 0; s < 4; ++s) dya[u][nt][s] = nt * 16 + t < N ? ds[(4 * s + g) * N + nt * 16 + t] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t0 = (tb + u) * 16;
            if constexpr (!kDyLds) tl.load_fm<NS, N>(a.dy, t0, dyb[u]);
            const bool ok = tl.chunk_ok(t0);
            const bool tok = tl.token_ok(t0);
            mu[u] = tok ? a.mean[t0 + t] : 0.f;
            ru[u] = tok ? a.rstd[t0 + t] : 0.f;
            xc[u] = ok ? *reinterpret_cast<const f4*>(a.x + (t0 + t) * C + 4 * g) : zero4();
            if (kEarlyRes) {   // the residual gradients travel with the tile's other loads
                rs[u] = (a.dres != nullptr && ok) ? *reinterpret_cast<const f4*>(a.dres + (t0 + t) * C + 4 * g) : zero4();
                rs2[u] = (a.dres2 != nullptr && ok) ? *reinterpret_cast<const f4*>(a.dres2 + (t0 + t) * C + 4 * g) : zero4();
            }
            tl.load_tm<C>(a.x, t0, 0, C, xa[u]);
            tl.load_tm_scalar(a.mean, t0, mt[u]);
            tl.load_tm_scalar(a.rstd, t0, rt[u]);
            if constexpr (!kDyLds) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) tl.load_tm<N>(a.dy, t0, nt * 16, N - nt * 16, dya[u][nt]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t0 = (tb + u) * 16;
            // dxn^T = W^T dy^T: accumulator chunk = dL/dLN(x) of channels 4 g + i of token t0 + t
            f4 dxn = zero4();
#pragma unroll
            for (int s = 0; s < NS; ++s) dxn = mfma(wt[s], dyb[u][s], dxn);
            // LayerNorm backward on the chunk (+ residual gradient)
            const bool ok = tl.chunk_ok(t0);
            const f4 xh = ok ? (xc[u] - mu[u]) * ru[u] : zero4();
            f4 dx = ln_bwd_chunk(dxn, xh, gm4, ru[u]);
            if (kEarlyRes) {
                dx += rs[u] + rs2[u];
            } else {
                if (a.dres != nullptr && ok) dx += *reinterpret_cast<const f4*>(a.dres + (t0 + t) * C + 4 * g);
                if (a.dres2 != nullptr && ok) dx += *reinterpret_cast<const f4*>(a.dres2 + (t0 + t) * C + 4 * g);
            }
            if (ok) *reinterpret_cast<f4*>(a.dx + (t0 + t) * C + 4 * g) = dx;
            dg += dxn * xh;
            dbt += dxn;
            // dW = dy^T xn over the tile's tokens (token-major operands; xn recomputed)
            float xnt[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) xnt[s] = t < C ? fmaf((xa[u][s] - mt[u][s]) * rt[u][s], gmt, btt) : 0.f;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    dw[nt] = mfma(dya[u][nt][s], xnt[s], dw[nt]);
                    db[nt] += dya[u][nt][s];
                }
            }
        }
    }
    // per-wave partial row: [dW (N x C) | db (N) | dgamma (C) | dbeta (C)] (one column sum)
    float* pa = a.partA + wave * (N * C + N + 2 * C);
    float* pb = pa + (N * C + N);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = nt * 16 + 4 * g + i;
            if (n < N && t < C) pa[n * C + t] = dw[nt][i];
        }
        const float v = sum_groups(db[nt]);
        if (g == 0 && nt * 16 + t < N) pa[N * C + nt * 16 + t] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float a1 = sum_tokens(dg[i]), a2 = sum_tokens(dbt[i]);
        if (t == 0 && g < 3) {
            pb[4 * g + i] = a1;
            pb[C + 4 * g + i] = a2;
        }
    }
}

// ------------------------------------------------------------------------------------
// dx = dy W;  dW = dy^T x;  db = colsum dy   (a C -> C Linear: the attention proj)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void linear_bwd_kernel(TokArgs a) {
    const int lane = threadIdx.x & 63;
    const Tile tl{a.rows, lane & 15, lane >> 4};
    const int t = tl.t, g = tl.g;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float wt[CS];
#pragma unroll
    for (int s = 0; s < CS; ++s) wt[s] = t < C ? a.w[(4 * s + g) * C + t] : 0.f;   // W^T[c = t][o = 4 s + g]
    f4 dw = zero4();
    float db = 0.f;
    const int64_t tiles = (a.rows + 15) / 16;
    for (int64_t tile = wave; tile < tiles; tile += nwaves) {
        const int64_t t0 = tile * 16;
        float dyb[CS];
        tl.load_fm<CS, C>(a.dy, t0, dyb);
        f4 dx = zero4();
#pragma unroll
        for (int s = 0; s < CS; ++s) dx = mfma(wt[s], dyb[s], dx);
        if (tl.chunk_ok(t0)) *reinterpret_cast<f4*>(a.dx + (t0 + t) * C + 4 * g) = dx;
        float dya[4], xa[4];
        tl.load_tm<C>(a.dy, t0, 0, C, dya);
        tl.load_tm<C>(a.x, t0, 0, C, xa);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            dw = mfma(dya[s], xa[s], dw);
            db += dya[s];
        }
    }
    float* pa = a.partA + wave * (C * C + C);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int o = 4 * g + i;
        if (o < C && t < C) pa[o * C + t] = dw[i];
    }
    db = sum_groups(db);
    if (g == 0 && t < C) pa[C * C + t] = db;
}

}  // namespace blk

namespace {
template <typename K>
int waves_of(K kern) {
    static_assert(sizeof(K) > 0, "");
    return tt::resident_blocks(reinterpret_cast<const void*>(kern), 256, 0) * 4;
}
}  // namespace

}  // namespace mmni

using namespace mmni;

static int tok_check(const mmni_tok_desc* d, bool ln) {
    MMNI_ARG_CHECK(d != nullptr && d->rows > 0, "token op: empty descriptor");
    MMNI_ARG_CHECK(d->C == 12, "token op: fused kernels cover C = 12 (got %d)", d->C);
    MMNI_ARG_CHECK(ln ? (d->N == 12 || d->N == 24 || d->N == 36) : d->N == 12,
                   "token op: unsupported N = %d", d->N);
    return 0;
}

static bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

extern "C" int mmni_ln_linear_fwd(const mmni_tok_desc* d, const float* x, const float* gamma, const float* beta,
                                  const float* w, const float* b, float* y, float* mean, float* rstd, void* stream) {
    int rc = tok_check(d, true);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && gamma && beta && w && y && mean && rstd, "ln_linear_fwd: null pointer");
    MMNI_ARG_CHECK(al16(x) && al16(y), "ln_linear_fwd: x / y must be 16-byte aligned");
    blk::TokArgs a{};
    a.rows = d->rows; a.eps = d->eps; a.x = x; a.gamma = gamma; a.beta = beta; a.w = w; a.b = b;
    a.y = y; a.mean = mean; a.rstd = rstd;
    const int64_t tiles = (d->rows + 15) / 16;
    hipStream_t s = (hipStream_t)stream;
#define MMNI_LLF(NN)                                                                                  \
    if (d->N == NN) {                                                                                 \
        static const int waves = waves_of(&blk::ln_linear_fwd_kernel<NN, blk::kLlfU>);                   \
        const int64_t need = (tiles + 4 * blk::kLlfU - 1) / (4 * blk::kLlfU);                                  \
        const int64_t grid = need < waves / 4 ? need : waves / 4;                                    \
        blk::ln_linear_fwd_kernel<NN, blk::kLlfU><<<(int)grid, 256, 0, s>>>(a);                           \
    }
    MMNI_LLF(12) MMNI_LLF(24) MMNI_LLF(36)
#undef MMNI_LLF
    return launch_status("ln_linear_fwd");
}

extern "C" size_t mmni_tok_bwd_workspace_bytes(const mmni_tok_desc* d) {
    if (!d) return 0;
    // the widest grid any of the backward kernels uses: resident blocks of 4 waves, at most 8 per CU
    const size_t waves = (size_t)kNumCU * 8 * 4;
    return waves * ((size_t)d->N * d->C + d->N + 2 * d->C) * sizeof(float);
}

static int ln_linear_bwd_impl(const mmni_tok_desc* d, const float* dy, const float* x, const float* mean,
                              const float* rstd, const float* gamma, const float* beta, const float* w,
                              const float* dres, const float* dres2, float* dx, float* dw, float* db, float* dgamma,
                              float* dbeta, void* workspace, void* stream) {
    int rc = tok_check(d, true);
    if (rc) return rc;
    MMNI_ARG_CHECK(dy && x && mean && rstd && gamma && beta && w && dx && dw && dgamma && dbeta && workspace,
                   "ln_linear_bwd: null pointer");
    MMNI_ARG_CHECK(al16(x) && al16(dx) && (!dres || al16(dres)) && (!dres2 || al16(dres2)),
                   "ln_linear_bwd: rows must be 16-byte aligned");
    const int N = d->N, C = d->C;
    blk::TokArgs a{};
    a.rows = d->rows; a.x = x; a.gamma = gamma; a.beta = beta; a.w = w; a.mean = const_cast<float*>(mean);
    a.rstd = const_cast<float*>(rstd); a.dy = dy; a.dres = dres; a.dres2 = dres2; a.dx = dx;
    hipStream_t s = (hipStream_t)stream;
    const int64_t tiles = (d->rows + 15) / 16;
    int waves = 0;
#define MMNI_LLB(NN)                                                                                  \
    if (N == NN) {                                                                                    \
        static const int wv = waves_of(&blk::ln_linear_bwd_kernel<NN, blk::llb_u(NN)>);                      \
        waves = wv < kNumCU * 8 * 4 ? wv : kNumCU * 8 * 4;                                           \
        a.partA = reinterpret_cast<float*>(workspace);                                              \
        blk::ln_linear_bwd_kernel<NN, blk::llb_u(NN)><<<waves / 4, 256, 0, s>>>(a);                           \
    }
    MMNI_LLB(12) MMNI_LLB(24) MMNI_LLB(36)
#undef MMNI_LLB
    (void)tiles;
    rc = launch_status("ln_linear_bwd");
    if (rc) return rc;
    ColSegs segs{};
    segs.n = 4;
    segs.end[0] = N * C;
    segs.end[1] = N * C + N;
    segs.end[2] = N * C + N + C;
    segs.end[3] = N * C + N + 2 * C;
    segs.dst[0] = dw;
    segs.dst[1] = db;
    segs.dst[2] = dgamma;
    segs.dst[3] = dbeta;
    column_sum_segs(a.partA, waves, N * C + N + 2 * C, segs, s);
    return launch_status("ln_linear_bwd_colsum");
}

extern "C" int mmni_ln_linear_bwd(const mmni_tok_desc* d, const float* dy, const float* x, const float* mean,
                                  const float* rstd, const float* gamma, const float* beta, const float* w,
                                  const float* dres, float* dx, float* dw, float* db, float* dgamma, float* dbeta,
                                  void* workspace, void* stream) {
    return ln_linear_bwd_impl(d, dy, x, mean, rstd, gamma, beta, w, dres, nullptr, dx, dw, db, dgamma, dbeta,
                              workspace, stream);
}

extern "C" int mmni_ln_linear_bwd2(const mmni_tok_desc* d, const float* dy, const float* x, const float* mean,
                                   const float* rstd, const float* gamma, const float* beta, const float* w,
                                   const float* dres, const float* dres2, float* dx, float* dw, float* db,
                                   float* dgamma, float* dbeta, void* workspace, void* stream) {
    return ln_linear_bwd_impl(d, dy, x, mean, rstd, gamma, beta, w, dres, dres2, dx, dw, db, dgamma, dbeta,
                              workspace, stream);
}

extern "C" int mmni_linear_bwd(const mmni_tok_desc* d, const float* dy, const float* x, const float* w, float* dx,
                               float* dw, float* db, void* workspace, void* stream) {
    int rc = tok_check(d, false);
    if (rc) return rc;
    MMNI_ARG_CHECK(dy && x && w && dx && dw && workspace, "linear_bwd: null pointer");
    MMNI_ARG_CHECK(al16(dx), "linear_bwd: dx must be 16-byte aligned");
    const int C = d->C;
    blk::TokArgs a{};
    a.rows = d->rows; a.x = x; a.w = w; a.dy = dy; a.dx = dx;
    static const int wv = waves_of(&blk::linear_bwd_kernel);
    const int waves = wv < kNumCU * 8 * 4 ? wv : kNumCU * 8 * 4;
    a.partA = reinterpret_cast<float*>(workspace);
    hipStream_t s = (hipStream_t)stream;
    blk::linear_bwd_kernel<<<waves / 4, 256, 0, s>>>(a);
    rc = launch_status("linear_bwd");
    if (rc) return rc;
    column_sum(a.partA, waves, C * C + C, dw, C * C, db, s);
    return launch_status("linear_bwd_colsum");
}
