// Fused token MLP of the Swin blocks on the f32 MFMA.
//
// Replaces Mlp / Mlp_fusion (modules/swin_v2_module.py:16-32, modules/swinfusion_module.py:14-30):
//   y = fc2(GELU(fc1(x))) (+ residual)           nn.GELU exact (erf), dropout inactive
// at the SwinFusion shape C = 12, hidden 48, over every token of a 96^3 volume (3.5M rows).
//
// The unfused path (tokenlinear.hip + linear_dw) moves the 48-wide hidden activation through HBM
// five times per block (fc1 out, fc2 in, dW2 in, dpre out/in); here it never leaves registers:
//   forward   per 16-token tile: pre^T = W1 x^T + b1 (9 MFMAs), GELU in registers,
//             y^T = W2 g^T + b2 (+ residual) (12 MFMAs); reads x (+ residual), writes y.
//   backward  per tile: recompute pre^T (9), dg^T = W2^T dy^T (9), dpre = dg * GELU'(pre),
//             dx^T = W1^T dpre^T (12); the weight gradients contract over tokens, which sit on the
//             lanes of the accumulator layout, so g and dpre take one LDS transpose per tile and
//             dW2 = dy^T g, dW1 = dpre^T x accumulate over the wave's tiles (24 MFMAs).  Per-wave
//             partials are summed in a fixed order (column_sum): deterministic.  Reads x and dy,
//             writes dx.
// With a LayerNorm prologue (LN template flag) the same kernels compute y = res + MLP(LN(x)),
// the second half of a pre-norm SwinFusion block (norm2 + mlp + residual,
// swinfusion_module.py:374-377): the LN statistics are computed in the tile (never stored),
// the backward recomputes them from x and adds the LN backward, dgamma / dbeta and the residual
// gradient (res = x) in the same pass.
// v_mfma_f32_16x16x4_f32 is exact f32 (an fmaf chain per output, cdna_hip_programming.md §FP32-
// input MFMA) at the f32 VALU rate, and leaves the VALU to the GELU polynomial.
//
// Operand maps (16x16x4 f32): A[l&15][k=l>>4], B[k=l>>4][l&15], C/D row (l>>4)*4+i, col l&15.
// A product that contracts over the ROW index of an accumulator tile takes it as an operand with
// no data movement when the k-step's 4 rows are chosen as {4g + i : g = 0..3} (fixed i): lane
// group g then supplies its own register i.  Hidden tiles are ht = 0..2 (48 = 3 x 16).
#include "mmni_common.h"

namespace mmni {

namespace mlpk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int C = 12, H = 48, HT = 3, CS = 3;   // channels, hidden, hidden tiles, channel k-steps
constexpr float kSqrtHalf = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f2 splat(float x) { return (f2){x, x}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Normal CDF Phi(v) of two values via Abramowitz & Stegun 7.1.26 (|erf err| <= 1.5e-7; measured
// in fp32 over [-12, 12]: |Phi err| <= 3.0e-7, |GELU err| <= 4.2e-7, |GELU' err| <= 3.0e-7):
//   erfc(z) = t (a1 + a2 t + ... + a5 t^4) exp(-z^2),  t = 1 / (1 + p z),  z = |v| / sqrt2,
// computed as the small tail term h = erfc / 2 so the negative tail has no cancellation.
// e = exp(-v^2 / 2) is returned for GELU' = Phi + v e / sqrt(2 pi).  5 packed FMAs + 1 rcp +
// 1 exp per value (the erfcc fit of tokenlinear.hip needs 9 FMAs and 2 exps).
__device__ __forceinline__ f2 norm_cdf2(f2 v, f2& e) {
    const f2 z = (f2){fabsf(v.x), fabsf(v.y)} * splat(kSqrtHalf);
    const f2 den = pfma(splat(0.3275911f), z, splat(1.0f));
    const f2 t = (f2){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    f2 p = splat(0.5f * 1.061405429f);
    p = pfma(p, t, splat(0.5f * -1.453152027f));
    p = pfma(p, t, splat(0.5f * 1.421413741f));
    p = pfma(p, t, splat(0.5f * -0.284496736f));
    p = pfma(p, t, splat(0.5f * 0.254829592f));
    const f2 w = z * (z * splat(-kLog2e));
    e = (f2){fast_exp2(w.x), fast_exp2(w.y)};
    const f2 h = (p * t) * e;                  // erfc(z) / 2 = Phi(-|v|)
    const f2 u = splat(0.5f) - h;              // |Phi(v) - 1/2|
    return splat(0.5f) + (f2){__builtin_copysignf(u.x, v.x), __builtin_copysignf(u.y, v.y)};
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
struct MlpArgs {
    int64_t rows;
    const float* x;    // (rows, C) contiguous
    const float* w1;   // (H, C)
    const float* b1;   // (H)
    const float* w2;   // (C, H)
    const float* b2;   // (C)
    const float* res;  // (rows, C) contiguous, or null
    const float* res2; // forward: a second addend (the residual group's skip), or null
    float* y;
    // LayerNorm prologue (LN kernels): x -> (x - mean) * rstd * gamma + beta over the C channels
    const float* gamma;
    const float* beta;
    float eps;
    int res_x;         // backward: the residual was x itself (dx += dy)
    // backward
    const float* dy;
    float* dx;
    float* partA;      // [waves][H*C + H]  dW1 | db1
    float* partB;      // [waves][C*H + C]  dW2 | db2
    float* partC;      // [waves][2C]       dgamma | dbeta (LN kernels)
};

__device__ __forceinline__ float sum_groups(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// LN statistics of the lane's token from its feature-major channels (nn.LayerNorm: biased
// variance, eps inside the root); all four lane groups end with the same values.
__device__ __forceinline__ void ln_stats(const float (&v)[CS], float eps, float& mean, float& rstd) {
    mean = sum_groups(v[0] + v[1] + v[2]) * (1.0f / C);
    float q = 0.f;
#pragma unroll
    for (int s = 0; s < CS; ++s) q = fmaf(v[s] - mean, v[s] - mean, q);
    rstd = 1.0f / sqrtf(sum_groups(q) * (1.0f / C) + eps);
}

// Rows are contiguous 48-byte token rows: a tile's data sits at a wave-uniform base (SGPR) plus a
// fixed per-lane offset, so every load / store is one instruction with an immediate offset.
// Only the last, partial tile takes the clamped path.
struct TileIO {
    int64_t rows;
    int li, lg;
    // feature-major B operand x[t0 + li][4 s + lg]
    __device__ __forceinline__ void load_fm(const float* base, int64_t t0, float (&v)[CS]) const {
        const float* p = base + t0 * C;
        if (t0 + 16 <= rows) {
#pragma unroll
            for (int s = 0; s < CS; ++s) v[s] = p[li * C + 4 * s + lg];
        } else {
            const bool ok = t0 + li < rows;
#pragma unroll
            for (int s = 0; s < CS; ++s) v[s] = ok ? p[li * C + 4 * s + lg] : 0.f;
        }
    }
    // token-major operand x[t0 + 4 s + lg][li] (li < C), for the weight gradients
    __device__ __forceinline__ void load_tm(const float* base, int64_t t0, float (&v)[4]) const {
        const float* p = base + t0 * C;
        const int cc = li < C ? li : 0;
        if (t0 + 16 <= rows) {
#pragma unroll
            for (int s = 0; s < 4; ++s) v[s] = li < C ? p[(4 * s + lg) * C + cc] : 0.f;
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) v[s] = (li < C && t0 + 4 * s + lg < rows) ? p[(4 * s + lg) * C + cc] : 0.f;
        }
    }
    // row chunk [t0 + li][4 lg .. 4 lg + 3] of the accumulator layout (lg < 3 holds the 12 channels)
    __device__ __forceinline__ bool row_ok(int64_t t0) const { return lg < 3 && t0 + li < rows; }
};

template <bool LN>
__global__ __launch_bounds__(256) void mlp_fwd_kernel(MlpArgs a) {
    const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const TileIO io{a.rows, li, lg};
    // weights in operand layout (loop invariant)
    float w1a[HT][CS], w2a[HT][4];
    f4 b1c[HT], b2c;
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
        for (int s = 0; s < CS; ++s) w1a[ht][s] = a.w1[(ht * 16 + li) * C + 4 * s + lg];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            w2a[ht][i] = li < C ? a.w2[li * H + ht * 16 + 4 * lg + i] : 0.f;
            b1c[ht][i] = a.b1 ? a.b1[ht * 16 + 4 * lg + i] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) b2c[i] = (lg < 3 && a.b2) ? a.b2[4 * lg + i] : 0.f;
    float gm[CS], bt[CS];
#pragma unroll
    for (int s = 0; s < CS; ++s) {
        gm[s] = LN ? a.gamma[4 * s + lg] : 1.f;
        bt[s] = LN ? a.beta[4 * s + lg] : 0.f;
    }

    const int64_t tiles = (a.rows + 15) / 16;
    // the next tile's x and residual are loaded while this tile computes (one tile in flight per
    // wave otherwise leaves the chain load -> LN -> MFMA -> GELU -> MFMA exposed)
    float xn[CS] = {0.f, 0.f, 0.f};
    f4 rn = (f4){0.f, 0.f, 0.f, 0.f}, sn = rn;
    auto fetch = [&](int64_t tile) {
        const int64_t t0 = tile * 16;
        io.load_fm(a.x, t0, xn);
        if (a.res != nullptr && io.row_ok(t0)) rn = *reinterpret_cast<const f4*>(a.res + (t0 + li) * C + 4 * lg);
        if (a.res2 != nullptr && io.row_ok(t0)) sn = *reinterpret_cast<const f4*>(a.res2 + (t0 + li) * C + 4 * lg);
    };
    if (wave < tiles) fetch(wave);
    for (int64_t tile = wave; tile < tiles; tile += nwaves) {
        const int64_t t0 = tile * 16;
        float xb[CS];
#pragma unroll
        for (int s = 0; s < CS; ++s) xb[s] = xn[s];
        const f4 rv = rn, sv = sn;
        if (tile + nwaves < tiles) fetch(tile + nwaves);
        if constexpr (LN) {
            float mean, rstd;
            ln_stats(xb, a.eps, mean, rstd);
#pragma unroll
            for (int s = 0; s < CS; ++s) xb[s] = fmaf((xb[s] - mean) * rstd, gm[s], bt[s]);
        }
        const bool ok = io.row_ok(t0);
        const int64_t roff = (t0 + li) * C + 4 * lg;
        f4 acc = b2c;
        if (a.res != nullptr && ok) acc += rv;
        if (a.res2 != nullptr && ok) acc += sv;
        // three independent accumulator chains (one per hidden tile), summed at the end
        f4 out[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f4 pre = b1c[ht];
#pragma unroll
            for (int s = 0; s < CS; ++s) pre = mfma(w1a[ht][s], xb[s], pre);
            f4 g;
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                f2 e;
                const f2 v = (f2){pre[i], pre[i + 1]};
                const f2 gv = v * norm_cdf2(v, e);
                g[i] = gv.x;
                g[i + 1] = gv.y;
            }
            out[ht] = ht == 0 ? acc : (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) out[ht] = mfma(w2a[ht][i], g[i], out[ht]);
        }
        if (ok) *reinterpret_cast<f4*>(a.y + roff) = out[0] + out[1] + out[2];
    }
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
constexpr int kBwdWaves = 4;   // waves per block (LDS transpose slab per wave)

constexpr int kMlpBwdOcc = 3;   // min waves per SIMD (caps VGPRs at 168)
// (the LN variant carries ~20 more live values: 2 waves per SIMD, no spills)
template <bool LN>
__global__ __launch_bounds__(256, kMlpBwdOcc) void mlp_bwd_kernel(MlpArgs a) {
    __shared__ float tr[kBwdWaves][2][16][H + 4];   // per wave: g and dpre as [token][hidden]
    const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
    const int wib = threadIdx.x >> 6;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const TileIO io{a.rows, li, lg};
    float w1a[HT][CS], w2ta[HT][CS], w1ta[HT][4];
    f4 b1c[HT];
    // the 42 per-lane weight values live in LDS ([value][lane]: conflict-free) and are re-read per
    // tile, which frees their VGPRs for a third wave per SIMD
    constexpr int NWV = HT * (2 * CS + 8);
    __shared__ float wv_s[NWV * 64];
    auto wload = [&]() {
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
            for (int s = 0; s < CS; ++s) {
                w1a[ht][s] = a.w1[(ht * 16 + li) * C + 4 * s + lg];      // W1[hid][c]
                w2ta[ht][s] = a.w2[(4 * s + lg) * H + ht * 16 + li];     // W2^T[hid][o] = W2[o][hid]
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w1ta[ht][i] = li < C ? a.w1[(ht * 16 + 4 * lg + i) * C + li] : 0.f;   // W1^T[c][hid]
                b1c[ht][i] = a.b1 ? a.b1[ht * 16 + 4 * lg + i] : 0.f;
            }
        }
    };
    auto wslot = [&](int ht, int k) -> float& { return wv_s[(ht * (2 * CS + 8) + k) * 64 + lane]; };
    if (wib == 0) {
        wload();
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
            for (int s = 0; s < CS; ++s) { wslot(ht, s) = w1a[ht][s]; wslot(ht, CS + s) = w2ta[ht][s]; }
#pragma unroll
            for (int i = 0; i < 4; ++i) { wslot(ht, 2 * CS + i) = w1ta[ht][i]; wslot(ht, 2 * CS + 4 + i) = b1c[ht][i]; }
        }
    }
    __syncthreads();
    f4 dw1[HT], dw2[HT];   // dW1 tile ht: rows hid, cols c;  dW2 tile ht: rows o, cols hid
    f4 db1[HT];            // per-lane partial column sums of dpre (rows hid, this lane's tokens)
    float db2 = 0.f;       // per-lane partial of dy[., o = li]
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        dw1[ht] = (f4){0.f, 0.f, 0.f, 0.f};
        dw2[ht] = (f4){0.f, 0.f, 0.f, 0.f};
        db1[ht] = (f4){0.f, 0.f, 0.f, 0.f};
    }
    // LN: gamma / beta in the feature-major (s), accumulator-chunk (i) and token-major (li) maps
    float gm[CS], bt[CS];
    f4 gm4, dgm = (f4){0.f, 0.f, 0.f, 0.f}, dbt = (f4){0.f, 0.f, 0.f, 0.f};
    float gml = 0.f, btl = 0.f;
    if constexpr (LN) {
#pragma unroll
        for (int s = 0; s < CS; ++s) { gm[s] = a.gamma[4 * s + lg]; bt[s] = a.beta[4 * s + lg]; }
#pragma unroll
        for (int i = 0; i < 4; ++i) gm4[i] = lg < 3 ? a.gamma[4 * lg + i] : 0.f;
        gml = li < C ? a.gamma[li] : 0.f;
        btl = li < C ? a.beta[li] : 0.f;
    }
    float (*gT)[H + 4] = tr[wib][0];
    float (*dT)[H + 4] = tr[wib][1];

    const int64_t tiles = (a.rows + 15) / 16;
    for (int64_t tile = wave; tile < tiles; tile += nwaves) {
        const int64_t t0 = tile * 16;
        asm volatile("" ::: "memory");   // keep the weight reads in the loop (not hoisted)
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
            for (int s = 0; s < CS; ++s) { w1a[ht][s] = wslot(ht, s); w2ta[ht][s] = wslot(ht, CS + s); }
#pragma unroll
            for (int i = 0; i < 4; ++i) { w1ta[ht][i] = wslot(ht, 2 * CS + i); b1c[ht][i] = wslot(ht, 2 * CS + 4 + i); }
        }
        float xb[CS], dyb[CS], xa[4], dya[4];
        io.load_fm(a.x, t0, xb);
        io.load_fm(a.dy, t0, dyb);
        io.load_tm(a.x, t0, xa);
        io.load_tm(a.dy, t0, dya);
        // LN variant: the chunk-layout x and dy rows of the LN backward / residual gradient load
        // with the tile's operands (after the MFMAs their latency was exposed once per tile)
        f4 xc_e = (f4){0.f, 0.f, 0.f, 0.f}, dyr_e = xc_e;
        if constexpr (LN) {
            if (io.row_ok(t0)) {
                const int64_t roff = (t0 + li) * C + 4 * lg;
                xc_e = *reinterpret_cast<const f4*>(a.x + roff);
                if (a.res_x) dyr_e = *reinterpret_cast<const f4*>(a.dy + roff);
            }
        }
        float mean = 0.f, rstd = 0.f;
        if constexpr (LN) {
            // recompute the LN of the tile: feature-major operand, and the token-major copy for
            // dW1 with the statistics of token 4 s + lg fetched from the lane that owns it
            ln_stats(xb, a.eps, mean, rstd);
#pragma unroll
            for (int s = 0; s < CS; ++s) xb[s] = fmaf((xb[s] - mean) * rstd, gm[s], bt[s]);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float ms = __shfl(mean, 4 * s + lg), rs = __shfl(rstd, 4 * s + lg);
                xa[s] = li < C ? fmaf((xa[s] - ms) * rs, gml, btl) : 0.f;
            }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) db2 += dya[s];
        f4 dxo[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f4 pre = b1c[ht], dg = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < CS; ++s) {
                pre = mfma(w1a[ht][s], xb[s], pre);
                dg = mfma(w2ta[ht][s], dyb[s], dg);
            }
            f4 g, dp;
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                f2 e;
                const f2 v = (f2){pre[i], pre[i + 1]};
                const f2 cdf = norm_cdf2(v, e);
                const f2 gv = v * cdf;
                const f2 gp = pfma(v * splat(kInvSqrt2Pi), e, cdf);   // GELU' = Phi + v phi
                const f2 d = (f2){dg[i], dg[i + 1]} * gp;
                g[i] = gv.x; g[i + 1] = gv.y;
                dp[i] = d.x; dp[i + 1] = d.y;
            }
            db1[ht] += dp;
            dxo[ht] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) dxo[ht] = mfma(w1ta[ht][i], dp[i], dxo[ht]);
            // transpose through LDS: lane (lg, li) holds hidden ht*16 + 4 lg + i of token li
            *reinterpret_cast<f4*>(&gT[li][ht * 16 + 4 * lg]) = g;
            *reinterpret_cast<f4*>(&dT[li][ht * 16 + 4 * lg]) = dp;
        }
        if constexpr (LN) {
            // LN backward on the lane's chunk (channels 4 lg + i of token li) + residual gradient
            const bool ok = io.row_ok(t0);
            const int64_t roff = (t0 + li) * C + 4 * lg;
            const f4 dxn = dxo[0] + dxo[1] + dxo[2];
            const f4 xc = xc_e;
            const f4 xh = ok ? (xc - mean) * rstd : (f4){0.f, 0.f, 0.f, 0.f};
            const f4 gd = dxn * gm4;
            const float s1 = sum_groups(gd[0] + gd[1] + gd[2] + gd[3]) * (1.0f / C);
            const float s2 = sum_groups(gd[0] * xh[0] + gd[1] * xh[1] + gd[2] * xh[2] + gd[3] * xh[3]) * (1.0f / C);
            f4 dxv = (gd - s1 - xh * s2) * rstd;
            dxv += dyr_e;
            if (ok) *reinterpret_cast<f4*>(a.dx + roff) = dxv;
            dgm += dxn * xh;
            dbt += dxn;
        } else {
            if (io.row_ok(t0)) *reinterpret_cast<f4*>(a.dx + (t0 + li) * C + 4 * lg) = dxo[0] + dxo[1] + dxo[2];
        }
        // weight gradients over the tile's 16 tokens (k-steps of 4 tokens: rows 4 s' + lg)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                const float gv = gT[4 * s + lg][ht * 16 + li];
                const float dv = dT[4 * s + lg][ht * 16 + li];
                dw2[ht] = mfma(dya[s], gv, dw2[ht]);   // dW2[o][hid] += dy[t][o] g[t][hid]
                dw1[ht] = mfma(dv, xa[s], dw1[ht]);    // dW1[hid][c] += dpre[t][hid] x[t][c]
            }
        }
    }
    // per-wave partial rows: A = [dW1 (H x C) | db1 (H)], B = [dW2 (C x H) | db2 (C)]
    // one partial row per wave: [dW1 | db1 | dW2 | db2 (| dgamma | dbeta)] (one column sum)
    constexpr int RW = H * C + H + C * H + C + (LN ? 2 * C : 0);
    float* pa = a.partA + wave * RW;
    float* pb = pa + (H * C + H);
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int hid_r = ht * 16 + 4 * lg + i;   // C/D row of the dW1 tile
            if (li < C) pa[hid_r * C + li] = dw1[ht][i];
            const int o = 4 * lg + i;                 // C/D row of the dW2 tile
            if (o < C) pb[o * H + ht * 16 + li] = dw2[ht][i];
            // db1: sum the 16 token lanes of this lane group
            float v = db1[ht][i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (li == 0) pa[H * C + hid_r] = v;
        }
    }
    db2 += __shfl_xor(db2, 16);
    db2 += __shfl_xor(db2, 32);
    if (lg == 0 && li < C) pb[C * H + li] = db2;
    if constexpr (LN) {
        float* pc = pb + (C * H + C);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float u = dgm[i], v = dbt[i];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) { u += __shfl_xor(u, o); v += __shfl_xor(v, o); }
            if (li == 0 && lg < 3) { pc[4 * lg + i] = u; pc[C + 4 * lg + i] = v; }
        }
    }
}

}  // namespace mlpk

// Persistent grids sized to what is resident at once (occupancy query, cached): a grid-stride
// launch of more blocks runs a partial second wave of blocks at a fraction of the occupancy.
static int resident_blocks(const void* kern, int threads, size_t lds) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    return per_cu * kNumCU;
}

template <bool LN>
static int mlp_bwd_waves() {
    static const int waves = resident_blocks(reinterpret_cast<const void*>(&mlpk::mlp_bwd_kernel<LN>),
                                             64 * mlpk::kBwdWaves, 0) * mlpk::kBwdWaves;
    return waves;
}

}  // namespace mmni

using namespace mmni;

static int mlp_check(const mmni_mlp_desc* d) {
    MMNI_ARG_CHECK(d != nullptr && d->rows > 0, "mlp: empty descriptor");
    MMNI_ARG_CHECK(d->C == 12 && d->H == 48, "mlp: fused kernel covers C=12, hidden 48 (got C=%d H=%d)", d->C, d->H);
    MMNI_ARG_CHECK(d->ldx == d->C && d->ldy == d->C, "mlp: rows must be contiguous (ldx = ldy = C)");
    return 0;
}

extern "C" int mmni_mlp_supported(int C, int H) { return C == 12 && H == 48; }

template <bool LN>
static int mlp_fwd_launch(const mmni_mlp_desc* d, const mlpk::MlpArgs& a, hipStream_t s) {
    static const int resident = resident_blocks(reinterpret_cast<const void*>(&mlpk::mlp_fwd_kernel<LN>), 256, 0);
    const int64_t tiles = (d->rows + 15) / 16;
    int64_t grid = (tiles + 3) / 4;
    if (grid > resident) grid = resident;
    mlpk::mlp_fwd_kernel<LN><<<(int)grid, 256, 0, s>>>(a);
    return launch_status(LN ? "ln_mlp_fwd" : "mlp_fwd");
}

extern "C" int mmni_mlp_fwd(const mmni_mlp_desc* d, const float* x, const float* w1, const float* b1,
                            const float* w2, const float* b2, const float* residual, float* y, void* stream) {
    int rc = mlp_check(d);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && w1 && w2 && y, "mlp_fwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(y) % 16 == 0 && (!residual || reinterpret_cast<uintptr_t>(residual) % 16 == 0),
                   "mlp_fwd: y / residual must be 16-byte aligned");
    mlpk::MlpArgs a{};
    a.rows = d->rows;
    a.x = x; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.res = residual; a.y = y;
    return mlp_fwd_launch<false>(d, a, (hipStream_t)stream);
}

static int ln_mlp_fwd_impl(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma, const float* beta,
                           const float* w1, const float* b1, const float* w2, const float* b2, int residual_x,
                           const float* skip, float* y, void* stream) {
    int rc = mlp_check(d);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && gamma && beta && w1 && w2 && y, "ln_mlp_fwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(y) % 16 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(skip) % 16 == 0, "ln_mlp_fwd: x / skip / y must be 16-byte aligned");
    mlpk::MlpArgs a{};
    a.rows = d->rows;
    a.x = x; a.gamma = gamma; a.beta = beta; a.eps = eps;
    a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.res = residual_x ? x : nullptr; a.res2 = skip; a.y = y;
    return mlp_fwd_launch<true>(d, a, (hipStream_t)stream);
}

extern "C" int mmni_ln_mlp_fwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma,
                               const float* beta, const float* w1, const float* b1, const float* w2, const float* b2,
                               int residual_x, float* y, void* stream) {
    return ln_mlp_fwd_impl(d, eps, x, gamma, beta, w1, b1, w2, b2, residual_x, nullptr, y, stream);
}

extern "C" int mmni_ln_mlp_skip_fwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma,
                                    const float* beta, const float* w1, const float* b1, const float* w2,
                                    const float* b2, int residual_x, const float* skip, float* y, void* stream) {
    MMNI_ARG_CHECK(skip != nullptr && skip != y, "ln_mlp_skip_fwd: skip must be a separate (rows, C) buffer");
    return ln_mlp_fwd_impl(d, eps, x, gamma, beta, w1, b1, w2, b2, residual_x, skip, y, stream);
}

extern "C" size_t mmni_mlp_bwd_workspace_bytes(const mmni_mlp_desc* d) {
    if (!d) return 0;
    const int waves = mlp_bwd_waves<false>() > mlp_bwd_waves<true>() ? mlp_bwd_waves<false>() : mlp_bwd_waves<true>();
    return (size_t)waves * ((size_t)d->H * d->C + d->H + (size_t)d->C * d->H + d->C + 2 * (size_t)d->C) * sizeof(float);
}

template <bool LN>
static int mlp_bwd_launch(const mmni_mlp_desc* d, mlpk::MlpArgs& a, float* dw1, float* db1, float* dw2, float* db2,
                          float* dgamma, float* dbeta, void* workspace, hipStream_t s) {
    const int C = d->C, H = d->H, waves = mlp_bwd_waves<LN>();
    a.partA = reinterpret_cast<float*>(workspace);   // [waves][dW1 | db1 | dW2 | db2 (| dgamma | dbeta)]
    mlpk::mlp_bwd_kernel<LN><<<waves / mlpk::kBwdWaves, 64 * mlpk::kBwdWaves, 0, s>>>(a);
    int rc = launch_status(LN ? "ln_mlp_bwd" : "mlp_bwd");
    if (rc) return rc;
    ColSegs segs{};
    segs.n = LN ? 6 : 4;
    const int e1 = H * C, e2 = e1 + H, e3 = e2 + C * H, e4 = e3 + C;
    segs.end[0] = e1; segs.end[1] = e2; segs.end[2] = e3; segs.end[3] = e4;
    segs.end[4] = e4 + C; segs.end[5] = e4 + 2 * C;
    segs.dst[0] = dw1; segs.dst[1] = db1; segs.dst[2] = dw2; segs.dst[3] = db2;
    segs.dst[4] = dgamma; segs.dst[5] = dbeta;
    column_sum_segs(a.partA, waves, LN ? e4 + 2 * C : e4, segs, s);
    return launch_status("mlp_colsum");
}

extern "C" int mmni_mlp_bwd(const mmni_mlp_desc* d, const float* x, const float* w1, const float* b1, const float* w2,
                            const float* dy, float* dx, float* dw1, float* db1, float* dw2, float* db2,
                            void* workspace, void* stream) {
    int rc = mlp_check(d);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && w1 && w2 && dy && dx && dw1 && dw2 && workspace, "mlp_bwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(dx) % 16 == 0, "mlp_bwd: dx must be 16-byte aligned");
    mlpk::MlpArgs a{};
    a.rows = d->rows;
    a.x = x; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.dy = dy; a.dx = dx;
    return mlp_bwd_launch<false>(d, a, dw1, db1, dw2, db2, nullptr, nullptr, workspace, (hipStream_t)stream);
}

extern "C" int mmni_ln_mlp_bwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma,
                               const float* beta, const float* w1, const float* b1, const float* w2, const float* dy,
                               int residual_x, float* dx, float* dgamma, float* dbeta, float* dw1, float* db1,
                               float* dw2, float* db2, void* workspace, void* stream) {
    int rc = mlp_check(d);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && gamma && beta && w1 && w2 && dy && dx && dgamma && dbeta && dw1 && dw2 && workspace,
                   "ln_mlp_bwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(dx) % 16 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(dy) % 16 == 0, "ln_mlp_bwd: x / dy / dx must be 16-byte aligned");
    mlpk::MlpArgs a{};
    a.rows = d->rows;
    a.x = x; a.gamma = gamma; a.beta = beta; a.eps = eps; a.res_x = residual_x;
    a.w1 = w1; a.b1 = b1; a.w2 = w2; a.dy = dy; a.dx = dx;
    return mlp_bwd_launch<true>(d, a, dw1, db1, dw2, db2, dgamma, dbeta, workspace, (hipStream_t)stream);
}
