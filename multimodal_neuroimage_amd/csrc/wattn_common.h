// Shared definitions of the window-attention kernels (wattn.hip: generic head_dim, wattn_pk.hip:
// packed-fp32 head_dim 2).  Internal, not part of the ABI.
#pragma once
#include "mmni_common.h"

namespace mmni {

struct WGeom {
    int B, D, H, W;
    int wd, wh, ww, sd, sh, sw;
    int nWd, nWh, nWw;
    int nwin;   // B * nWd * nWh * nWw
    int N;      // tokens per window
    int tw, th; // relative-code strides: (2wh-1)(2ww-1), (2ww-1)
    int off;    // (wd-1)*tw + (wh-1)*th + (ww-1)
    int Tsz;    // bias table rows
};

// Region id of a shifted-frame coordinate (swinfusion_module.py:321-331: slices
// (0,-ws), (-ws,-s), (-s,None) filled with increasing ids).
__device__ __host__ __forceinline__ int shift_region(int c, int L, int ws, int s) {
    return s == 0 ? 0 : (c < L - ws ? 0 : (c < L - s ? 1 : 2));
}

struct TokenInfo {
    int64_t row;  // source token row in the (B, D, H, W) tensor
    int code;     // i*tw + j*th + k  (relative-position code)
    int rc;       // packed per-axis region ids
};

__device__ __forceinline__ TokenInfo token_info(const WGeom& g, int w, int t) {
    int r = w;
    const int wx = r % g.nWw; r /= g.nWw;
    const int wy = r % g.nWh; r /= g.nWh;
    const int wz = r % g.nWd;
    const int b = r / g.nWd;
    const int k = t % g.ww;
    const int r2 = t / g.ww;
    const int j = r2 % g.wh;
    const int i = r2 / g.wh;
    const int cz = wz * g.wd + i, cy = wy * g.wh + j, cx = wx * g.ww + k;
    int z = cz + g.sd; if (z >= g.D) z -= g.D;
    int y = cy + g.sh; if (y >= g.H) y -= g.H;
    int x = cx + g.sw; if (x >= g.W) x -= g.W;
    TokenInfo ti;
    ti.row = ((int64_t)(b * g.D + z) * g.H + y) * g.W + x;
    ti.code = i * g.tw + j * g.th + k;
    ti.rc = (shift_region(cz, g.D, g.wd, g.sd) * 3 + shift_region(cy, g.H, g.wh, g.sh)) * 3 +
            shift_region(cx, g.W, g.ww, g.sw);
    return ti;
}

struct WAArgs {
    WGeom g;
    int KS, WPB, NPAD, ngroups, kind;
    float scale;
    int64_t qs, ks, vs, os;
    const float* q;
    const float* k;
    const float* v;
    const float* table;
    const float* tau;
    float* out;
    float* lse;
    // backward
    const float* o;
    const float* dout;
    float* dq;
    float* dk;
    float* dv;
    float* dtable;
    float* dtau;
    unsigned long long* dtab_fix;   // global int64 fixed-point accumulator (workspace)
    unsigned int* maxbits;          // workspace tail: max|dout|, max|v| bits (fixed-point scale)
    int fix_shift;                  // bits the fixed-point scale is lowered by (0: every kernel here)
    unsigned int* vmax;             // forward (packed kernels): running max|v| (float bits), or null
    int hsplit;                     // head groups per window (blocks split the heads; row-broadcast bwd: head pairs)
    float* dtau_part;               // kind 1 backward: one dtau partial row (NH floats) per block (workspace)
};

// kind 1 backward: the per-wave dtau sums land in LDS slots (no atomics) and each block writes
// one fixed-order partial row; a fixed-order column sum adds the rows into dtau (deterministic).
constexpr int kMaxWaves = 16;                   // 1024-thread blocks
constexpr int kMaxBwdBlocks = 8 * 256;          // resident-grid cap of the generic backward (plan())

constexpr float kMask2 = -100.0f * kLog2e;  // -100 shift mask in the log2 domain
constexpr float kNormEps = 1e-12f;          // F.normalize eps (swin_v2_module.py:153)
constexpr int CH = 4;                       // keys per online-softmax chunk (generic kernels)
constexpr int kDtabPad = 1;   // packed bwd: table-gradient row stride NH + pad (u64)
constexpr int kTabSwz = 1;     // packed bwd: float4 chunks of table row r XOR-ed with (r >> 3)
constexpr int kPkChunk = 6;     // keys per online-softmax chunk (packed kernels)
constexpr int kPk2Chunk = 3;    // keys per online-softmax chunk of the two-query forward
constexpr int kPk2Ks = 1;       // key slices (lanes per query pair) of the two-query forward
constexpr int kPk2FwdWpb = 2;   // windows per block of the two-query forward: two blocks share a CU

// Packed head_dim-2 kernels (wattn_pk.hip): fills kf/kb/maxt and returns 1 when C is covered.
int wattn_pk_kernels(int C, int kind, int N, void*& kf, void*& kb, int& maxt_f, int& maxt_b, int& qpl_f);

// Row-broadcast head_dim-2 backward (wattn_bc.hip): kind 0, head pairs, paired rows t, t + N/2.
bool wattn_bc_supported(const WGeom& g, int C, int heads, int kind);
size_t wattn_bc_workspace_bytes(const WGeom& g, int heads);
int wattn_bc_backward(WAArgs& a, int heads, float* dtable, void* workspace, hipStream_t s);
int wattn_bc_forward(WAArgs& a, int heads, hipStream_t s);   // same geometries; vmax as the packed kernels

// The bias-table gradient is a scatter-add of N*N*heads values per window into a
// (2w-1)^k x heads table.  LDS float atomics (ds_add_f32) run ~5x slower than the rest of the
// backward on gfx950 (measured: 27.8 ms vs 4.8 ms without the table update at the C3 shape),
// integer LDS atomics run at full rate.  So the table gradient is accumulated in 64-bit fixed
// point: exact, order-independent integer adds, i.e. bitwise deterministic, flushed to a global
// int64 workspace and converted once.  The scale 2^S is picked per call from a proven bound:
//   |ds| = p |dO.v - delta| <= 2 * HD * max|dout| * max|v| < 2^ex      (delta is a p-average of dO.v)
//   S = 30 - ex  =>  every contribution rounds to a 32-bit integer below 2^30 (one cvt, no
//   64-bit arithmetic), and an entry takes at most one contribution per query and head, so
//   |entry sum| < T * 2^30 < 2^63 for the T < 2^31 tokens the descriptor allows.
// Resolution is 2^-30 of the largest possible contribution, rounded to nearest (a fixed 2^-32
// scale with truncation was measured at 20% error on BCE-loss-sized table gradients: ~1e4
// contributions of ~1e-10 summing to ~1e-7).
__device__ __forceinline__ int fix_exponent(const unsigned int* maxbits, int hd) {
    const double bound = 2.0 * hd * (double)__uint_as_float(maxbits[0]) * (double)__uint_as_float(maxbits[1]);
    if (!(bound < 1e300)) return 0;       // non-finite inputs: any scale, the result is garbage anyway
    if (bound <= 0.0) return 126;
    int ex;
    frexp(bound, &ex);                    // bound < 2^ex
    return max(-100, min(126, 30 - ex));
}

__device__ __forceinline__ unsigned long long to_fixed(float x, float scale) {
    return (unsigned long long)(long long)__float2int_rn(x * scale);   // |x * scale| < 2^30
}


template <int C>
__device__ __forceinline__ void load_row(float (&dst)[C], const float* src) {
    if constexpr (C % 4 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 4) {
            const float4 t = *reinterpret_cast<const float4*>(src + c);
            dst[c] = t.x; dst[c + 1] = t.y; dst[c + 2] = t.z; dst[c + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) dst[c] = src[c];
    }
}

template <int C>
__device__ __forceinline__ void store_row(float* dst, const float (&src)[C]) {
    if constexpr (C % 4 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 4)
            *reinterpret_cast<float4*>(dst + c) = make_float4(src[c], src[c + 1], src[c + 2], src[c + 3]);
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) dst[c] = src[c];
    }
}

// Per-head L2 normalisation (F.normalize(dim=-1), eps 1e-12); returns the raw norms.
template <int C, int HD>
__device__ __forceinline__ void normalize_heads(float (&x)[C], float (&nrm)[C / HD]) {
#pragma unroll
    for (int h = 0; h < C / HD; ++h) {
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < HD; ++c) ss += x[h * HD + c] * x[h * HD + c];
        nrm[h] = sqrtf(ss);
        const float inv = 1.0f / fmaxf(nrm[h], kNormEps);
#pragma unroll
        for (int c = 0; c < HD; ++c) x[h * HD + c] *= inv;
    }
}

// Backward of y = x / max(||x||, eps) for one head: dx from dy, y and the raw norm.
template <int HD>
__device__ __forceinline__ void normalize_bwd(float* dx, const float* dy, const float* y, float nrm) {
    if (nrm >= kNormEps) {
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < HD; ++c) dot += y[c] * dy[c];
        const float inv = 1.0f / nrm;
#pragma unroll
        for (int c = 0; c < HD; ++c) dx[c] = (dy[c] - y[c] * dot) * inv;
    } else {
#pragma unroll
        for (int c = 0; c < HD; ++c) dx[c] = dy[c] * (1.0f / kNormEps);
    }
}

}  // namespace mmni
