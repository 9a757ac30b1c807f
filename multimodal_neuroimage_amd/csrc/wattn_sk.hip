// Scalar-key window attention for SwinFusion's head_dim 2 (kind 0, pair-interleaved layout).
//
// Replaces, on the device:
//   torch.roll + window_partition_fusion          modules/swinfusion_module.py:33-45,350-357
//   WindowAttention_fusion.forward                modules/swinfusion_module.py:114-145
//   Cross_WindowAttention.forward                 modules/swinfusion_module.py:213-246
//   window_reverse_fusion + reverse roll          modules/swinfusion_module.py:366-373
//
// Why a second formulation (the LDS-staged kernels of wattn.hip / wattn_pk.hip stay for the
// natural channel layout): with K/V rows staged in LDS and read back as 16-byte broadcasts, every
// (query, key) step costs ~34 LDS-array cycles per wave (ds_read_b128 = 4 cycles for any address
// pattern) against ~50 VALU issue cycles per head pair, and the backward's table-gradient atomics
// add ~48 more: measured, the staged backward spends more LDS than VALU time.  Here a wave owns 64
// query rows (or key rows) of ONE window and walks the other side of the window in lock-step, so
// the walked row is wave-uniform: it is fetched with scalar loads (s_load_dwordx4, its own cache,
// no LDS, no VGPRs) and used as the SGPR operand of v_pk_fma_f32.  The only per-lane gather is the
// relative-position bias row, read from the (Tsz, heads) table through the vector L1.  What stays
// in LDS is the backward's table-gradient accumulator.  Waves never synchronise inside a launch.
//
// Layout 1 ("pairs"): channel (head h, dim c) of a q/k/v/out row sits at (h/2)*4 + c*2 + (h%2),
// so a row is an array of float2 {head 2P, head 2P+1} per dim: one v_pk_* instruction serves two
// heads.  The modules produce it for free by permuting the rows of the qkv / q / kv Linear weights
// and the columns of the proj weight (functional.pair_perm).  lse is stored in base 2.
//
// Softmax (forward): online over chunks of KC keys with a lazy rescale — the running max m only
// moves when some score of the wave exceeds m + 8 (log2 domain), so exp2(s - m) <= 256 stays
// finite and the per-chunk rescale (two v_exp_f32 per head pair) is skipped almost always.
// Backward: flash-style recompute of P from lse; pass A (lane = query) -> dq and the table
// gradient (64-bit fixed point LDS atomics, wattn_common.h), pass B (lane = key) -> dk, dv.
#include <type_traits>

#include "wattn_common.h"

namespace mmni {

namespace sk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
// constant address space: a wave-uniform address through it becomes an s_load
typedef __attribute__((address_space(4))) const f4 cf4;
typedef __attribute__((address_space(4))) const f2 cf2;

__device__ __forceinline__ f2 splat(float x) { return (f2){x, x}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 exp2_2(f2 x) { return (f2){fast_exp2(x.x), fast_exp2(x.y)}; }

// wave-uniform row of C floats (pair layout) -> C/2 float2 in SGPRs
template <int C>
__device__ __forceinline__ void sload_row(f2 (&d)[C / 2], const float* p) {
#pragma unroll
    for (int i = 0; i < C / 4; ++i) {
        const f4 t = *(cf4*)(p + 4 * i);
        d[2 * i] = (f2){t.x, t.y};
        d[2 * i + 1] = (f2){t.z, t.w};
    }
}

template <int N2>
__device__ __forceinline__ void sload_pairs(f2 (&d)[N2], const float* p) {
#pragma unroll
    for (int i = 0; i < N2; ++i) {
        d[i] = *(cf2*)(p + 2 * i);
    }
}

// per-lane row of C floats (pair layout) -> C/2 float2 in VGPRs
template <int C>
__device__ __forceinline__ void vload_row(f2 (&d)[C / 2], const float* p) {
#pragma unroll
    for (int i = 0; i < C / 4; ++i) {
        const float4 t = *reinterpret_cast<const float4*>(p + 4 * i);
        d[2 * i] = (f2){t.x, t.y};
        d[2 * i + 1] = (f2){t.z, t.w};
    }
}

template <int C>
__device__ __forceinline__ void vstore_row(float* p, const f2 (&s)[C / 2], float scale) {
#pragma unroll
    for (int i = 0; i < C / 4; ++i)
        *reinterpret_cast<float4*>(p + 4 * i) = make_float4(s[2 * i].x * scale, s[2 * i].y * scale,
                                                            s[2 * i + 1].x * scale, s[2 * i + 1].y * scale);
}

template <int NP>
__device__ __forceinline__ void vload_tab(f2 (&d)[NP], const float* p) {
#pragma unroll
    for (int P = 0; P < NP; ++P) {
        const float2 t = *reinterpret_cast<const float2*>(p + 2 * P);
        d[P] = (f2){t.x, t.y};
    }
}

// Wave-uniform description of one window (all SGPR values).
struct Win {
    int b, wz, wy, wx;
    bool masked;   // last window along a shifted axis: tokens of several shift regions
};

__device__ __forceinline__ Win window_of(const WGeom& g, int w) {
    Win v;
    int r = w;
    v.wx = r % g.nWw; r /= g.nWw;
    v.wy = r % g.nWh; r /= g.nWh;
    v.wz = r % g.nWd;
    v.b = r / g.nWd;
    v.masked = (g.sw && v.wx == g.nWw - 1) || (g.sh && v.wy == g.nWh - 1) || (g.sd && v.wz == g.nWd - 1);
    return v;
}

// Walk the (z, y) rows of window v in window order, calling row_fn(row of x = 0 before the
// shift wrap, code of x = 0, region id of x = 0 without the x part); key_of() completes a token.
// Every value is wave-uniform (SGPRs); the x loop stays in the caller.
template <typename F>
__device__ __forceinline__ void walk_rows(const WGeom& g, const Win& v, F&& row_fn) {
    for (int kz = 0; kz < g.wd; ++kz) {
        const int cz = v.wz * g.wd + kz;
        int z = cz + g.sd;
        if (z >= g.D) z -= g.D;
        const int rz = shift_region(cz, g.D, g.wd, g.sd);
        for (int ky = 0; ky < g.wh; ++ky) {
            const int cy = v.wy * g.wh + ky;
            int y = cy + g.sh;
            if (y >= g.H) y -= g.H;
            const int ry = shift_region(cy, g.H, g.wh, g.sh);
            const int64_t rowb = ((int64_t)(v.b * g.D + z) * g.H + y) * g.W;
            row_fn(rowb, kz * g.tw + ky * g.th, (rz * 3 + ry) * 3);
        }
    }
}

__device__ __forceinline__ void key_of(const WGeom& g, const Win& v, int64_t rowb, int codeb, int rcb, int kx,
                                       int64_t& row, int& code, int& rc) {
    const int cx = v.wx * g.ww + kx;
    int x = cx + g.sw;
    if (x >= g.W) x -= g.W;
    row = rowb + x;
    code = codeb + kx;
    rc = rcb + shift_region(cx, g.W, g.ww, g.sw);
}

__device__ __forceinline__ long long fix_round(float x) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return (long long)r;
}

constexpr float kLazy = 8.0f;   // log2-domain slack of the lazy softmax max

// x-walk of one row of a window: wrapped x coordinate and region id of column c (uniform)
__device__ __forceinline__ void col_of(const WGeom& g, const Win& v, int c, int& x, int& rx) {
    const int cx = v.wx * g.ww + c;
    x = cx + g.sw;
    if (x >= g.W) x -= g.W;
    rx = shift_region(cx, g.W, g.ww, g.sw);
}

// Unit = (window, quarter of 64 rows, head pair): 64 lanes x 2 heads, walking all N tokens of the
// window on the other side.  A block holds the nq * NP units of one window, so its waves fetch
// the same walked rows within a few hundred cycles of each other: scalar-cache hits.
struct Unit {
    int w, qt, P;
};

__device__ __forceinline__ f2 lo2(f4 x) { return (f2){x.x, x.y}; }
__device__ __forceinline__ f2 hi2(f4 x) { return (f2){x.z, x.w}; }
// byte-offset addressing: every buffer a launch touches is < 2 GiB (checked on the host), so row
// offsets are 32-bit SALU products instead of 64-bit multiply chains
__device__ __forceinline__ f4 sload4(const char* base, uint32_t off) { return *(cf4*)(base + off); }
__device__ __forceinline__ f2 sload2(const char* base, uint32_t off) { return *(cf2*)(base + off); }
__device__ __forceinline__ f4 vload4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ f2 vload2(const float* p) { return *reinterpret_cast<const f2*>(p); }

template <bool V>
using bool_c = std::integral_constant<bool, V>;

// Calls body(row_index, code, region) for every token of window v in window order; the x-row of
// WW tokens (compile-time, WW > 0) is handed over as one batch: body_row(rows[], codes0, rcs[]).
template <int WW, typename FR>
__device__ __forceinline__ void walk_window(const WGeom& g, const Win& v, FR&& body_row) {
    const int ww = WW ? WW : g.ww;
    for (int kz = 0; kz < g.wd; ++kz) {
        const int cz = v.wz * g.wd + kz;
        int z = cz + g.sd;
        if (z >= g.D) z -= g.D;
        const int rz = shift_region(cz, g.D, g.wd, g.sd);
        for (int ky = 0; ky < g.wh; ++ky) {
            const int cy = v.wy * g.wh + ky;
            int y = cy + g.sh;
            if (y >= g.H) y -= g.H;
            const int ry = shift_region(cy, g.H, g.wh, g.sh);
            const int rowb = ((v.b * g.D + z) * g.H + y) * g.W;
            const int codeb = kz * g.tw + ky * g.th;
            const int rcb = (rz * 3 + ry) * 3;
            if constexpr (WW > 0) {
                int rows[WW], rcs[WW];
#pragma unroll
                for (int c = 0; c < WW; ++c) {
                    int x, rx;
                    col_of(g, v, c, x, rx);
                    rows[c] = rowb + x;
                    rcs[c] = rcb + rx;
                }
                body_row(rows, codeb, rcs);
            } else {
                for (int c = 0; c < ww; ++c) {
                    int x, rx;
                    col_of(g, v, c, x, rx);
                    int rows[1] = {rowb + x}, rcs[1] = {rcb + rx};
                    body_row(rows, codeb + c, rcs);
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
// WW > 0: window x-extent known at compile time; the x-row of WW keys is one softmax chunk with
// all its K rows (then all its V rows) fetched before use.  WW = 0: runtime extent, 1-key chunks.
template <int NH, int WW>
__global__ __launch_bounds__(1024) void wattn_fwd_sk_kernel(WAArgs a, int nq, int nunits) {
    constexpr int NP = NH / 2;
    constexpr int KC = WW ? WW : 1;
    const WGeom& g = a.g;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;   // = nq * NP: one block walks one window per iteration
    const f2 L2E = splat(kLog2e);
    const float sl2 = a.scale * kLog2e;
    const uint32_t ks4 = (uint32_t)a.ks * 4, vs4 = (uint32_t)a.vs * 4;
    for (int w = blockIdx.x; w < g.nwin; w += gridDim.x) {
        const Unit un = {w, wave / NP, wave % NP};
        const Win v = window_of(g, un.w);
        const int t = un.qt * 64 + lane;
        const bool act = t < g.N;
        const TokenInfo ti = token_info(g, un.w, act ? t : g.N - 1);
        const int cq = ti.code + g.off, rq = ti.rc;
        const f4 q4 = vload4(a.q + ti.row * a.qs + 4 * un.P);
        const f2 aq0 = lo2(q4) * splat(sl2), aq1 = hi2(q4) * splat(sl2);
        const float* tabP = a.table + 2 * un.P;
        const char* kP = reinterpret_cast<const char*>(a.k + 4 * un.P);
        const char* vP = reinterpret_cast<const char*>(a.v + 4 * un.P);
        f2 m = splat(-INFINITY), m8 = splat(-INFINITY), l = splat(0.f), acc0 = splat(0.f), acc1 = splat(0.f);
        auto run = [&](auto masked_c) {
            constexpr bool MASKED = decltype(masked_c)::value;
            walk_window<WW>(g, v, [&](const int (&rows)[KC], int code0, const int (&rcs)[KC]) {
                f4 kk[KC];
                f2 tb[KC];
                const float* tp = tabP + (cq - code0) * NH;   // bias rows of this x-row: tp - c*NH
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    kk[c] = sload4(kP, (uint32_t)rows[c] * ks4);
                    tb[c] = vload2(tp - c * NH);
                }
                f2 s[KC];
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    f2 sc;
                    if constexpr (MASKED) sc = pfma(tb[c], L2E, splat(rcs[c] != rq ? kMask2 : 0.f));
                    else sc = tb[c] * L2E;
                    sc = pfma(aq0, lo2(kk[c]), sc);
                    s[c] = pfma(aq1, hi2(kk[c]), sc);
                }
                // lazy online max: rescale only when a score passes m + 8 (log2 domain)
                f2 cm = s[0];
#pragma unroll
                for (int c = 1; c < KC; ++c) cm = (f2){fmaxf(cm.x, s[c].x), fmaxf(cm.y, s[c].y)};
                if (__any((cm.x > m8.x) | (cm.y > m8.y))) {
                    const f2 mn = (f2){fmaxf(m.x, cm.x), fmaxf(m.y, cm.y)};
                    const f2 al = exp2_2(m - mn);
                    l *= al;
                    acc0 *= al;
                    acc1 *= al;
                    m = mn;
                    m8 = mn + splat(kLazy);
                }
                f4 vv[KC];
#pragma unroll
                for (int c = 0; c < KC; ++c) vv[c] = sload4(vP, (uint32_t)rows[c] * vs4);
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    const f2 pj = exp2_2(s[c] - m);
                    l += pj;
                    acc0 = pfma(pj, lo2(vv[c]), acc0);
                    acc1 = pfma(pj, hi2(vv[c]), acc1);
                }
            });
        };
        if (v.masked) run(bool_c<true>{});
        else run(bool_c<false>{});
        if (act) {
            const f2 inv = (f2){1.0f / l.x, 1.0f / l.y};
            acc0 *= inv;
            acc1 *= inv;
            *reinterpret_cast<f4*>(a.out + ti.row * a.os + 4 * un.P) = (f4){acc0.x, acc0.y, acc1.x, acc1.y};
            const f2 lse2 = m + (f2){fast_log2(l.x), fast_log2(l.y)};
            *reinterpret_cast<f2*>(a.lse + ti.row * NH + 2 * un.P) = lse2;
        }
    }
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
// delta = rowsum(O * dO) per (token, head), and max|dO|, max|V| for the fixed-point bound.
template <int C>
__global__ void wattn_prep_sk_kernel(const float* o, const float* dout, int64_t os, const float* vv, int64_t vs,
                                     int64_t T, float* delta, unsigned int* maxbits) {
    constexpr int NH = C / 2, NP = NH / 2;
    float md = 0.f, mv = 0.f;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < T; r += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int P = 0; P < NP; ++P) {
            const f4 o4 = vload4(o + r * os + 4 * P), g4 = vload4(dout + r * os + 4 * P);
            const f4 v4 = vload4(vv + r * vs + 4 * P);
            const f2 d = pfma(lo2(o4), lo2(g4), hi2(o4) * hi2(g4));
            *reinterpret_cast<f2*>(delta + r * NH + 2 * P) = d;
            md = fmaxf(md, fmaxf(fmaxf(fabsf(g4.x), fabsf(g4.y)), fmaxf(fabsf(g4.z), fabsf(g4.w))));
            mv = fmaxf(mv, fmaxf(fmaxf(fabsf(v4.x), fabsf(v4.y)), fmaxf(fabsf(v4.z), fabsf(v4.w))));
        }
    }
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
        md = fmaxf(md, __shfl_xor(md, o2));
        mv = fmaxf(mv, __shfl_xor(mv, o2));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&maxbits[0], __float_as_uint(md));
        atomicMax(&maxbits[1], __float_as_uint(mv));
    }
}

// pass A: lane = query row -> dq and the bias-table gradient
template <int NH, int WW>
__global__ __launch_bounds__(1024) void wattn_bwdq_sk_kernel(WAArgs a, int nq, int nunits, const float* delta) {
    constexpr int NP = NH / 2;
    constexpr int KC = WW ? WW : 1;
    constexpr int DS = NH + 1;   // odd u64 stride of the table-gradient rows (spreads LDS banks)
    extern __shared__ __attribute__((aligned(16))) unsigned long long dtab_s[];   // [Tsz][DS]
    const WGeom& g = a.g;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;   // = nq * NP: one block walks one window per iteration
    const f2 L2E = splat(kLog2e);
    const float sl2 = a.scale * kLog2e;
    const uint32_t ks4 = (uint32_t)a.ks * 4, vs4 = (uint32_t)a.vs * 4;
    for (int e = threadIdx.x; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0ull;
    const int fexp = fix_exponent(a.maxbits, 2);
    const float fs = exp2f((float)fexp);     // 2^S: |ds| * 2^S < 2^30 (wattn_common.h)
    const float ifs = exp2f((float)-fexp);
    __syncthreads();

    for (int w = blockIdx.x; w < g.nwin; w += gridDim.x) {
        const Unit un = {w, wave / NP, wave % NP};
        const Win v = window_of(g, un.w);
        const int t = un.qt * 64 + lane;
        const bool act = t < g.N;
        const TokenInfo ti = token_info(g, un.w, act ? t : g.N - 1);
        const f4 q4 = vload4(a.q + ti.row * a.qs + 4 * un.P);
        const f4 g4 = vload4(a.dout + ti.row * a.os + 4 * un.P);
        const f2 aq0 = lo2(q4) * splat(sl2), aq1 = hi2(q4) * splat(sl2);
        const float gs = act ? fs : 0.f;
        const f2 dO0 = lo2(g4) * splat(gs), dO1 = hi2(g4) * splat(gs);
        const f2 nlse = act ? -vload2(a.lse + ti.row * NH + 2 * un.P) : splat(-INFINITY);
        const f2 ndl = vload2(delta + ti.row * NH + 2 * un.P) * splat(-gs);
        const int cq = ti.code + g.off, rq = ti.rc;
        const float* tabP = a.table + 2 * un.P;
        const char* kP = reinterpret_cast<const char*>(a.k + 4 * un.P);
        const char* vP = reinterpret_cast<const char*>(a.v + 4 * un.P);
        unsigned long long* dtP = dtab_s + 2 * un.P;
        f2 dq0 = splat(0.f), dq1 = splat(0.f);
        auto run = [&](auto masked_c) {
            constexpr bool MASKED = decltype(masked_c)::value;
            walk_window<WW>(g, v, [&](const int (&rows)[KC], int code0, const int (&rcs)[KC]) {
                f4 kk[KC], vk[KC];
                f2 tb[KC];
                const float* tp = tabP + (cq - code0) * NH;   // bias rows of this x-row: tp - c*NH
                unsigned long long* dtr = dtP + (cq - code0) * DS;
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    kk[c] = sload4(kP, (uint32_t)rows[c] * ks4);
                    vk[c] = sload4(vP, (uint32_t)rows[c] * vs4);
                    tb[c] = vload2(tp - c * NH);
                }
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    f2 sc;
                    if constexpr (MASKED) sc = pfma(tb[c], L2E, nlse + splat(rcs[c] != rq ? kMask2 : 0.f));
                    else sc = pfma(tb[c], L2E, nlse);
                    sc = pfma(aq0, lo2(kk[c]), sc);
                    sc = pfma(aq1, hi2(kk[c]), sc);
                    const f2 pr = exp2_2(sc);
                    f2 tt = pfma(dO0, lo2(vk[c]), ndl);
                    tt = pfma(dO1, hi2(vk[c]), tt);
                    const f2 dsv = pr * tt;
                    dq0 = pfma(dsv, lo2(kk[c]), dq0);
                    dq1 = pfma(dsv, hi2(kk[c]), dq1);
                    unsigned long long* dt = dtr - c * DS;
                    atomicAdd(&dt[0], (unsigned long long)fix_round(dsv.x));
                    atomicAdd(&dt[1], (unsigned long long)fix_round(dsv.y));
                }
            });
        };
        if (v.masked) run(bool_c<true>{});
        else run(bool_c<false>{});
        if (act) {
            const float sc = a.scale * ifs;
            *reinterpret_cast<f4*>(a.dq + ti.row * a.qs + 4 * un.P) =
                (f4){dq0.x * sc, dq0.y * sc, dq1.x * sc, dq1.y * sc};
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < g.Tsz * NH; e += blockDim.x) {
        const unsigned long long x = dtab_s[(e / NH) * DS + e % NH];
        if (x != 0ull) atomicAdd(&a.dtab_fix[e], x);
    }
}

// pass B: lane = key row -> dk, dv (no LDS).  The x-row of queries is fetched in halves (12
// SGPRs of q / dO / lse / delta per query).
template <int NH, int WW>
__global__ __launch_bounds__(1024) void wattn_bwdkv_sk_kernel(WAArgs a, int nq, int nunits, const float* delta) {
    constexpr int NP = NH / 2;
    constexpr int KC = WW ? WW : 1;
    constexpr int HB = (KC % 2 == 0) ? KC / 2 : KC;   // queries fetched per batch
    const WGeom& g = a.g;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;   // = nq * NP: one block walks one window per iteration
    const f2 L2E = splat(kLog2e);
    const float sl2 = a.scale * kLog2e;
    const uint32_t qs4 = (uint32_t)a.qs * 4, os4 = (uint32_t)a.os * 4, ns4 = NH * 4;
    for (int w = blockIdx.x; w < g.nwin; w += gridDim.x) {
        const Unit un = {w, wave / NP, wave % NP};
        const Win v = window_of(g, un.w);
        const int t = un.qt * 64 + lane;
        const bool act = t < g.N;
        const TokenInfo ti = token_info(g, un.w, act ? t : g.N - 1);
        const f4 k4 = vload4(a.k + ti.row * a.ks + 4 * un.P);
        const f4 v4 = vload4(a.v + ti.row * a.vs + 4 * un.P);
        const f2 kr0 = lo2(k4) * splat(sl2), kr1 = hi2(k4) * splat(sl2);
        const f2 vr0 = lo2(v4), vr1 = hi2(v4);
        const int cko = g.off - ti.code, rk = ti.rc;
        const float* tabP = a.table + 2 * un.P;
        const char* qP = reinterpret_cast<const char*>(a.q + 4 * un.P);
        const char* gP = reinterpret_cast<const char*>(a.dout + 4 * un.P);
        const char* lP = reinterpret_cast<const char*>(a.lse + 2 * un.P);
        const char* dP = reinterpret_cast<const char*>(delta + 2 * un.P);
        f2 dk0 = splat(0.f), dk1 = splat(0.f), dv0 = splat(0.f), dv1 = splat(0.f);
        auto run = [&](auto masked_c) {
            constexpr bool MASKED = decltype(masked_c)::value;
            walk_window<WW>(g, v, [&](const int (&rows)[KC], int code0, const int (&rcs)[KC]) {
#pragma unroll
                for (int h0 = 0; h0 < KC; h0 += HB) {
                    f4 qq[HB], gg[HB];
                    f2 ll[HB], dd[HB], tb[HB];
                    const float* tp = tabP + (code0 + h0 + cko) * NH;
#pragma unroll
                    for (int c = 0; c < HB; ++c) {
                        const uint32_t r = (uint32_t)rows[h0 + c];
                        qq[c] = sload4(qP, r * qs4);
                        gg[c] = sload4(gP, r * os4);
                        ll[c] = sload2(lP, r * ns4);
                        dd[c] = sload2(dP, r * ns4);
                        tb[c] = vload2(tp + c * NH);
                    }
#pragma unroll
                    for (int c = 0; c < HB; ++c) {
                        f2 base = pfma(tb[c], L2E, -ll[c]);
                        if constexpr (MASKED) base += splat(rcs[h0 + c] != rk ? kMask2 : 0.f);
                        f2 sc = pfma(lo2(qq[c]), kr0, base);
                        sc = pfma(hi2(qq[c]), kr1, sc);
                        const f2 pr = exp2_2(sc);
                        const f2 tt = pfma(lo2(gg[c]), vr0, hi2(gg[c]) * vr1);
                        const f2 dsv = pr * (tt - dd[c]);
                        dv0 = pfma(pr, lo2(gg[c]), dv0);
                        dv1 = pfma(pr, hi2(gg[c]), dv1);
                        dk0 = pfma(dsv, lo2(qq[c]), dk0);
                        dk1 = pfma(dsv, hi2(qq[c]), dk1);
                    }
                }
            });
        };
        if (v.masked) run(bool_c<true>{});
        else run(bool_c<false>{});
        if (act) {
            *reinterpret_cast<f4*>(a.dk + ti.row * a.ks + 4 * un.P) =
                (f4){dk0.x * a.scale, dk0.y * a.scale, dk1.x * a.scale, dk1.y * a.scale};
            *reinterpret_cast<f4*>(a.dv + ti.row * a.vs + 4 * un.P) = (f4){dv0.x, dv0.y, dv1.x, dv1.y};
        }
    }
}

}  // namespace sk

// ------------------------------------------------------------------------------------
// host side (called from wattn.hip for layout 1)
// ------------------------------------------------------------------------------------
// block = the nq * NP units of one window; grid-stride over windows, sized to the resident capacity
static int sk_units(const WGeom& g, int heads, int& nq) {
    nq = (g.N + 63) / 64;
    return g.nwin * nq * (heads / 2);
}

static int sk_block(const WGeom& g, int heads) { return 64 * ((g.N + 63) / 64) * (heads / 2); }

static int sk_grid(const WGeom& g, int heads, int waves_per_cu) {
    const int wpb = sk_block(g, heads) / 64;
    int per_cu = waves_per_cu / wpb;
    if (per_cu < 1) per_cu = 1;
    return g.nwin < per_cu * kNumCU ? g.nwin : per_cu * kNumCU;
}

#define MMNI_SK_DISPATCH(KERN, NH_, ...)                                           \
    (a.g.ww == 6 ? reinterpret_cast<void*>(&sk::KERN<NH_, 6>) : reinterpret_cast<void*>(&sk::KERN<NH_, 0>))

// 32-bit byte offsets in the kernels: rows * stride * 4 must stay below 2^31 for every buffer
static int sk_check_offsets(const WAArgs& a) {
    const int64_t T = (int64_t)a.g.B * a.g.D * a.g.H * a.g.W;
    int64_t smax = a.qs > a.ks ? a.qs : a.ks;
    if (a.vs > smax) smax = a.vs;
    if (a.os > smax) smax = a.os;
    MMNI_ARG_CHECK(T * smax * 4 < (1ll << 31),
                   "wattn (pair layout): %lld rows x stride %lld exceed the 2 GiB byte-offset range; split the "
                   "batch or use layout 0", (long long)T, (long long)smax);
    return 0;
}

int wattn_sk_fwd(const WAArgs& a0, int C, hipStream_t stream) {
    WAArgs a = a0;
    if (int rc = sk_check_offsets(a)) return rc;
    int nq;
    const int heads = C / 2;
    int units = sk_units(a.g, heads, nq);
    void* kern = nullptr;
    if (C == 12) kern = MMNI_SK_DISPATCH(wattn_fwd_sk_kernel, 6);
    else if (C == 24) kern = MMNI_SK_DISPATCH(wattn_fwd_sk_kernel, 12);
    else { set_error("wattn (pair layout): C=%d unsupported (12 or 24)", C); return -2; }
    void* args[] = {&a, &nq, &units};
    MMNI_ARG_CHECK(sk_block(a.g, heads) <= 1024, "wattn (pair layout): window of %d tokens too large", a.g.N);
    hipError_t e = hipLaunchKernel(kern, dim3(sk_grid(a.g, heads, 32)), dim3(sk_block(a.g, heads)), args, 0, stream);
    if (e != hipSuccess) { set_error("wattn_fwd_sk launch: %s", hipGetErrorString(e)); return (int)e; }
    return 0;
}

size_t wattn_sk_workspace(const WGeom& g, int heads) {
    return (size_t)g.Tsz * heads * 8 + 16 + (size_t)g.nwin * g.N * heads * 4;
}

int wattn_sk_bwd(const WAArgs& a0, int C, int heads, void* workspace, hipStream_t stream) {
    WAArgs a = a0;
    if (int rc = sk_check_offsets(a)) return rc;
    const WGeom& g = a.g;
    const int ntab = g.Tsz * heads;
    a.dtab_fix = reinterpret_cast<unsigned long long*>(workspace);
    a.maxbits = reinterpret_cast<unsigned int*>(a.dtab_fix + ntab);
    const float* delta = reinterpret_cast<const float*>(reinterpret_cast<char*>(workspace) + (size_t)ntab * 8 + 16);
    float* delta_w = const_cast<float*>(delta);
    hipError_t e = hipMemsetAsync(workspace, 0, (size_t)ntab * 8 + 16, stream);
    if (e != hipSuccess) { set_error("wattn_bwd memset: %s", hipGetErrorString(e)); return (int)e; }
    const int64_t T = (int64_t)g.nwin * g.N;
    int nq;
    int units = sk_units(g, heads, nq);
    const size_t lds = (size_t)g.Tsz * (heads + 1) * 8;
    if (lds > 80 * 1024) {
        set_error("wattn_bwd (pair layout): table-gradient LDS %zu B exceeds 80 KiB", lds);
        return -2;
    }
    void *kq = nullptr, *kkv = nullptr;
    if (C == 12) {
        sk::wattn_prep_sk_kernel<12><<<1024, 256, 0, stream>>>(a.o, a.dout, a.os, a.v, a.vs, T, delta_w, a.maxbits);
        kq = MMNI_SK_DISPATCH(wattn_bwdq_sk_kernel, 6);
        kkv = MMNI_SK_DISPATCH(wattn_bwdkv_sk_kernel, 6);
    } else if (C == 24) {
        sk::wattn_prep_sk_kernel<24><<<1024, 256, 0, stream>>>(a.o, a.dout, a.os, a.v, a.vs, T, delta_w, a.maxbits);
        kq = MMNI_SK_DISPATCH(wattn_bwdq_sk_kernel, 12);
        kkv = MMNI_SK_DISPATCH(wattn_bwdkv_sk_kernel, 12);
    } else {
        set_error("wattn (pair layout): C=%d unsupported (12 or 24)", C);
        return -2;
    }
    int rc = launch_status("wattn_prep_sk");
    if (rc) return rc;
    if (lds > 64 * 1024) {
        e = hipFuncSetAttribute(kq, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
        if (e != hipSuccess) { set_error("hipFuncSetAttribute: %s", hipGetErrorString(e)); return (int)e; }
    }
    void* args[] = {&a, &nq, &units, &delta};
    MMNI_ARG_CHECK(sk_block(g, heads) <= 1024, "wattn (pair layout): window of %d tokens too large", g.N);
    const int per_cu_lds = (int)((160 * 1024) / lds);
    const int wpb = sk_block(g, heads) / 64;
    e = hipLaunchKernel(kq, dim3(sk_grid(g, heads, per_cu_lds * wpb < 32 ? per_cu_lds * wpb : 32)),
                        dim3(sk_block(g, heads)), args, lds, stream);
    if (e != hipSuccess) { set_error("wattn_bwdq_sk launch: %s", hipGetErrorString(e)); return (int)e; }
    e = hipLaunchKernel(kkv, dim3(sk_grid(g, heads, 32)), dim3(sk_block(g, heads)), args, 0, stream);
    if (e != hipSuccess) { set_error("wattn_bwdkv_sk launch: %s", hipGetErrorString(e)); return (int)e; }
    return 0;
}

}  // namespace mmni
