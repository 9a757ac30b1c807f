// Token Linear forward / input gradient for the skinny Linears of the Swin blocks (gfx950).
//
// The reference's block Linears (qkv 12->36, proj 12->12, q/kv 12->12/24, fc1 12->48, fc2
// 48->12; swinfusion_module.py:25-31,104-110,203-205) run over every token of a 96^3 volume:
// M = 3.5M rows with K, N <= 48.  These are pure streams (AI < 6 FLOP/B): hipBLASLt's tiles
// (rocprof r02: MT16x256x16 at 350 us per call) run them at about a quarter of the HBM floor.
// Here one lane owns one row: the row is read with 16-byte loads, the weight matrix sits in LDS
// (W[k][n], read as wave-uniform broadcasts) and the epilogue is fused:
//   EPI 0  y = x W^T (+ b)
//   EPI 1  y = gelu(x W^T + b)                                   (Mlp fc1 + nn.GELU, exact erf)
//   EPI 2  y = (x W^T) * gelu'(aux W2^T + b2)                     (Mlp backward through fc2 and
//          the GELU, the fc1 pre-activation recomputed from the fc1 input `aux`, so it is never
//          stored)
// The weight is addressed as W(n, k) = w[n*w_sn + k*w_sk]: (K, 1) is an nn.Linear weight, (1, Nw)
// its transpose, used for dX = dY W.
#include "mmni_common.h"
#include "tokentile.h"

namespace mmni {

struct TLinArgs {
    int64_t rows, ldx, ldy, ldaux;
    int64_t w_sn, w_sk;
    const float* x;
    const float* w;
    const float* bias;
    const float* aux;
    const float* w2;   // fc1 weight (N, K2), nn.Linear layout
    const float* b2;
    const float* res;  // optional residual added in the epilogue (epi 0/1), row stride ldy
    float* y;
};

constexpr float kSqrtHalf = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

// Normal CDF without the device libm erff: ocml's erff takes two divergent branches (~35 VALU
// per value with both paths live), which made the fused fc1 + GELU kernel compute-bound.
// Phi(x) = erfc(-x / sqrt2) / 2 with the Chebyshev erfc fit of Numerical Recipes (erfcc,
// fractional error < 1.2e-7): one rcp, nine FMAs and one exp, no branch.  Measured in fp32
// emulation over [-12, 12]: |Phi err| <= 2.2e-7, |GELU err| <= 1.6e-7 absolute (torch's fp32
// 0.5x(1 + erf(x/sqrt2)) cancels catastrophically in the negative tail; this form does not).
__device__ __forceinline__ float norm_cdf(float x) {
    const float z = fabsf(x) * kSqrtHalf;
    const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);
    float p = 0.17087277f;
    p = fmaf(p, t, -0.82215223f);
    p = fmaf(p, t, 1.48851587f);
    p = fmaf(p, t, -1.13520398f);
    p = fmaf(p, t, 0.27886807f);
    p = fmaf(p, t, -0.18628806f);
    p = fmaf(p, t, 0.09678418f);
    p = fmaf(p, t, 0.37409196f);
    p = fmaf(p, t, 1.00002368f);
    const float half = 0.5f * t * __expf(fmaf(t, p, fmaf(-z, z, -1.26551223f)));
    return x >= 0.f ? 1.0f - half : half;
}
__device__ __forceinline__ float gelu_exact(float v) { return v * norm_cdf(v); }
__device__ __forceinline__ float gelu_grad(float v) {
    return norm_cdf(v) + v * kInvSqrt2Pi * __expf(-0.5f * v * v);
}

template <int K>
__device__ __forceinline__ void ld_row(float (&d)[K], const float* s) {
#pragma unroll
    for (int c = 0; c < K; c += 4) {
        const float4 t = *reinterpret_cast<const float4*>(s + c);
        d[c] = t.x; d[c + 1] = t.y; d[c + 2] = t.z; d[c + 3] = t.w;
    }
}

template <int K, int N, int EPI, int K2>
__global__ __launch_bounds__(256) void token_linear_kernel(TLinArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[K * N];            // W[k][n]
    __shared__ __attribute__((aligned(16))) float bl[N];
    __shared__ __attribute__((aligned(16))) float w2l[EPI == 2 ? K2 * N : 4];   // W2[k2][n]
    __shared__ __attribute__((aligned(16))) float b2l[EPI == 2 ? N : 4];
    for (int e = threadIdx.x; e < K * N; e += blockDim.x) {
        const int k = e / N, n = e - k * N;
        wl[e] = a.w[n * a.w_sn + k * a.w_sk];
    }
    for (int n = threadIdx.x; n < N; n += blockDim.x) bl[n] = a.bias ? a.bias[n] : 0.f;
    if constexpr (EPI == 2) {
        for (int e = threadIdx.x; e < K2 * N; e += blockDim.x) {
            const int k = e / N, n = e - k * N;
            w2l[e] = a.w2[n * K2 + k];
        }
        for (int n = threadIdx.x; n < N; n += blockDim.x) b2l[n] = a.b2 ? a.b2[n] : 0.f;
    }
    __syncthreads();
    if constexpr (K == 12 && N == 12 && EPI == 0) {
        if (a.ldx == K && a.ldy == N) {
            // Contiguous rows: the block's 256 x 12 tile moves between HBM and LDS as contiguous
            // 16-B vectors (a lane's own 48-B row, read and written directly, leaves every
            // instruction touching a third of each line: the measured write traffic doubled).
            // The residual is added on the way out.
            __shared__ __attribute__((aligned(16))) float tile[256 * 12];
            float4* t4 = reinterpret_cast<float4*>(tile);
            const float4* x4 = reinterpret_cast<const float4*>(a.x);
            const float4* r4 = reinterpret_cast<const float4*>(a.res);
            float4* y4 = reinterpret_cast<float4*>(a.y);
            for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < a.rows; r0 += (int64_t)gridDim.x * 256) {
                const int nr = a.rows - r0 < 256 ? (int)(a.rows - r0) : 256;
                const int nv = nr * 3;
                float4 xin[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int e = k * 256 + threadIdx.x;
                    if (e < nv) xin[k] = x4[r0 * 3 + e];
                }
                __syncthreads();   // the previous tile's stores have read the LDS tile
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int e = k * 256 + threadIdx.x;
                    if (e < nv) t4[e] = xin[k];
                }
                __syncthreads();
                if ((int)threadIdx.x < nr) {
                    float xr[12];
                    ld_row<12>(xr, tile + threadIdx.x * 12);
                    float o[12];
#pragma unroll
                    for (int n = 0; n < 12; n += 4) {
                        float acc[4] = {bl[n], bl[n + 1], bl[n + 2], bl[n + 3]};
#pragma unroll
                        for (int k = 0; k < 12; ++k) {
                            const float4 wv = *reinterpret_cast<const float4*>(wl + k * N + n);
                            acc[0] = fmaf(xr[k], wv.x, acc[0]);
                            acc[1] = fmaf(xr[k], wv.y, acc[1]);
                            acc[2] = fmaf(xr[k], wv.z, acc[2]);
                            acc[3] = fmaf(xr[k], wv.w, acc[3]);
                        }
                        o[n] = acc[0]; o[n + 1] = acc[1]; o[n + 2] = acc[2]; o[n + 3] = acc[3];
                    }
#pragma unroll
                    for (int n = 0; n < 12; n += 4)
                        t4[threadIdx.x * 3 + n / 4] = make_float4(o[n], o[n + 1], o[n + 2], o[n + 3]);
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int e = k * 256 + threadIdx.x;
                    if (e < nv) {
                        float4 v = t4[e];
                        if (r4 != nullptr) {
                            const float4 rv = r4[r0 * 3 + e];
                            v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
                        }
                        y4[r0 * 3 + e] = v;
                    }
                }
            }
            return;
        }
    }
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.rows; r += (int64_t)gridDim.x * blockDim.x) {
        // keep the LDS weight reads inside the loop: hoisted, K*N weights would not fit in VGPRs
        asm volatile("" ::: "memory");
        float xr[K];
        ld_row<K>(xr, a.x + r * a.ldx);
        float ar[EPI == 2 ? K2 : 1];
        if constexpr (EPI == 2) ld_row<K2>(ar, a.aux + r * a.ldaux);
        // output columns in chunks of 4: the row stays in registers, each chunk is reduced over
        // k, passed through the epilogue and stored as one 16-byte write
        constexpr int kChunkUnroll = EPI == 0 ? N / 4 : 1;
#pragma unroll kChunkUnroll
        for (int n = 0; n < N; n += 4) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float4 wv = *reinterpret_cast<const float4*>(wl + k * N + n);
                acc[0] = fmaf(xr[k], wv.x, acc[0]);
                acc[1] = fmaf(xr[k], wv.y, acc[1]);
                acc[2] = fmaf(xr[k], wv.z, acc[2]);
                acc[3] = fmaf(xr[k], wv.w, acc[3]);
            }
            const float4 bv = *reinterpret_cast<const float4*>(bl + n);
            float o[4];
            if constexpr (EPI == 0) {
                o[0] = acc[0] + bv.x; o[1] = acc[1] + bv.y; o[2] = acc[2] + bv.z; o[3] = acc[3] + bv.w;
            } else if constexpr (EPI == 1) {
                o[0] = gelu_exact(acc[0] + bv.x); o[1] = gelu_exact(acc[1] + bv.y);
                o[2] = gelu_exact(acc[2] + bv.z); o[3] = gelu_exact(acc[3] + bv.w);
            } else {
                float pre[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < K2; ++k) {
                    const float4 wv = *reinterpret_cast<const float4*>(w2l + k * N + n);
                    pre[0] = fmaf(ar[k], wv.x, pre[0]);
                    pre[1] = fmaf(ar[k], wv.y, pre[1]);
                    pre[2] = fmaf(ar[k], wv.z, pre[2]);
                    pre[3] = fmaf(ar[k], wv.w, pre[3]);
                }
                const float4 cv = *reinterpret_cast<const float4*>(b2l + n);
                o[0] = acc[0] * gelu_grad(pre[0] + cv.x); o[1] = acc[1] * gelu_grad(pre[1] + cv.y);
                o[2] = acc[2] * gelu_grad(pre[2] + cv.z); o[3] = acc[3] * gelu_grad(pre[3] + cv.w);
            }
            if (EPI != 2 && a.res != nullptr) {
                const float4 rv = *reinterpret_cast<const float4*>(a.res + r * a.ldy + n);
                o[0] += rv.x; o[1] += rv.y; o[2] += rv.z; o[3] += rv.w;
            }
            *reinterpret_cast<float4*>(a.y + r * a.ldy + n) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

// 12 -> 12 Linear (+ bias, + residual) on contiguous rows (the attention proj): one 16-token tile
// per wave step on the f32 MFMA in the accumulator-chunk layout of tokentile.h (as blockops'
// linear_bwd), y^T = W x^T.  No LDS staging and no block barriers: the LDS-tiled path above
// moved the same bytes at ~3.7 TB/s.
__global__ __launch_bounds__(256) void linear12_fwd_kernel(TLinArgs a) {
    using namespace tt;
    const int lane = threadIdx.x & 63;
    const Tile tl{a.rows, lane & 15, lane >> 4};
    const int t = tl.t, g = tl.g;
    const int64_t wave = __builtin_amdgcn_readfirstlane(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float wf[CS];   // A operand: W[o = t][c = 4 s + g]
#pragma unroll
    for (int s = 0; s < CS; ++s) wf[s] = t < C ? a.w[t * a.w_sn + (4 * s + g) * a.w_sk] : 0.f;
    f4 bc;
#pragma unroll
    for (int i = 0; i < 4; ++i) bc[i] = (g < 3 && a.bias != nullptr) ? a.bias[4 * g + i] : 0.f;
    const int64_t tiles = (a.rows + 15) / 16;
    for (int64_t tile = wave; tile < tiles; tile += nwaves) {
        const int64_t t0 = tile * 16;
        float xb[CS];
        tl.load_fm<CS, C>(a.x, t0, xb);
        const bool ok = tl.chunk_ok(t0);
        const int64_t off = (t0 + t) * C + 4 * g;
        const f4 r = (a.res != nullptr && ok) ? *reinterpret_cast<const f4*>(a.res + off) : zero4();
        f4 y = bc;
#pragma unroll
        for (int s = 0; s < CS; ++s) y = mfma(wf[s], xb[s], y);
        if (ok) *reinterpret_cast<f4*>(a.y + off) = y + r;
    }
}

}  // namespace mmni

using namespace mmni;

static bool aligned16(const void* p, int64_t ld) {
    return reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0;
}

extern "C" int mmni_token_linear(const mmni_tlin_desc* d, const float* x, const float* w, const float* bias,
                                 const float* aux, const float* w2, const float* b2, const float* residual, float* y,
                                 void* stream) {
    MMNI_ARG_CHECK(d != nullptr && x && w && y, "token_linear: null pointer");
    MMNI_ARG_CHECK(d->rows > 0 && d->K > 0 && d->N > 0, "token_linear: empty shape");
    MMNI_ARG_CHECK(d->epi >= 0 && d->epi <= 2, "token_linear: epi must be 0, 1 or 2");
    MMNI_ARG_CHECK(d->ldx >= d->K && d->ldy >= d->N, "token_linear: leading dimensions too small");
    MMNI_ARG_CHECK(aligned16(x, d->ldx) && aligned16(y, d->ldy),
                   "token_linear: x / y rows must be 16-byte aligned (ld multiple of 4)");
    if (d->epi == 2) {
        MMNI_ARG_CHECK(aux && w2 && d->ldaux >= d->K2 && aligned16(aux, d->ldaux),
                       "token_linear: epi 2 needs aligned aux rows and w2");
    }
    TLinArgs a{};
    a.rows = d->rows; a.ldx = d->ldx; a.ldy = d->ldy; a.ldaux = d->ldaux;
    a.w_sn = d->w_sn; a.w_sk = d->w_sk;
    MMNI_ARG_CHECK(residual == nullptr || (d->epi != 2 && reinterpret_cast<uintptr_t>(residual) % 16 == 0),
                   "token_linear: residual needs epi 0/1 and 16-byte alignment");
    a.x = x; a.w = w; a.bias = bias; a.aux = aux; a.w2 = w2; a.b2 = b2; a.res = residual; a.y = y;
    const int64_t blocks = (d->rows + 255) / 256;
    hipStream_t s = (hipStream_t)stream;
    if (d->K == 12 && d->N == 12 && d->epi == 0 && d->ldx == 12 && d->ldy == 12) {
        static const int resident =
            tt::resident_blocks(reinterpret_cast<const void*>(&linear12_fwd_kernel), 256, 0);
        const int64_t need = (d->rows + 63) / 64;   // 4 waves x 16-token tiles per block
        const int grid = (int)(need < resident ? need : resident);
        linear12_fwd_kernel<<<grid, 256, 0, s>>>(a);
        return launch_status("token_linear");
    }
    // grid-stride loops over row tiles: one resident wave of blocks (a fixed 4096-block grid left
    // a partial second round of blocks on every CU)
#define MMNI_TLIN(K_, N_, E_, K2_)                                                                  \
    if (d->K == K_ && d->N == N_ && d->epi == E_ && (E_ != 2 || d->K2 == K2_)) {                    \
        static const int resident =                                                                \
            tt::resident_blocks(reinterpret_cast<const void*>(&token_linear_kernel<K_, N_, E_, K2_>), 256, 0); \
        const int grid = (int)(blocks < resident ? blocks : resident);                              \
        token_linear_kernel<K_, N_, E_, K2_><<<grid, 256, 0, s>>>(a);                                \
        return launch_status("token_linear");                                                       \
    }
    MMNI_TLIN(12, 36, 0, 0) MMNI_TLIN(12, 12, 0, 0) MMNI_TLIN(12, 24, 0, 0) MMNI_TLIN(12, 48, 0, 0)
    MMNI_TLIN(48, 12, 0, 0) MMNI_TLIN(36, 12, 0, 0) MMNI_TLIN(24, 12, 0, 0)
    MMNI_TLIN(12, 48, 1, 0)
    MMNI_TLIN(12, 48, 2, 12)
#undef MMNI_TLIN
    set_error("token_linear: unsupported shape K=%d N=%d epi=%d K2=%d", d->K, d->N, d->epi, d->K2);
    return -2;
}

extern "C" int mmni_token_linear_supported(int K, int N, int epi, int K2) {
    if (epi == 0)
        return (K == 12 && (N == 36 || N == 12 || N == 24 || N == 48)) ||
               (N == 12 && (K == 48 || K == 36 || K == 24));
    if (epi == 1) return K == 12 && N == 48;
    if (epi == 2) return K == 12 && N == 48 && K2 == 12;
    return 0;
}
