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

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
// WW > 0: window x-extent known at compile time (the x walk is unrolled); 0 = runtime.
template <int C, int KC, int WW>
__global__ __launch_bounds__(512, 2) void wattn_fwd_sk_kernel(WAArgs a, int nq, int nunits) {
    constexpr int NH = C / 2, NP = NH / 2;
    const WGeom& g = a.g;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    const f2 L2E = splat(kLog2e);
    const float sl2 = a.scale * kLog2e;
    for (int u = blockIdx.x * wpb + wave; u < nunits; u += gridDim.x * wpb) {
        const int w = u / nq, qt = u - w * nq;
        const Win v = window_of(g, w);
        const int t = qt * 64 + lane;
        const bool act = t < g.N;
        const TokenInfo ti = token_info(g, w, act ? t : g.N - 1);
        const int cq = ti.code + g.off, rq = ti.rc;
        f2 aq[C / 2];
        vload_row<C>(aq, a.q + ti.row * a.qs);
#pragma unroll
        for (int i = 0; i < C / 2; ++i) aq[i] *= splat(sl2);
        f2 m[NP], m8[NP], l[NP], acc[C / 2];
#pragma unroll
        for (int P = 0; P < NP; ++P) { m[P] = splat(-INFINITY); m8[P] = splat(-INFINITY); l[P] = splat(0.f); }
#pragma unroll
        for (int i = 0; i < C / 2; ++i) acc[i] = splat(0.f);

        walk_rows(g, v, [&](int64_t rowb, int codeb, int rcb) {
            const int ww = WW ? WW : g.ww;
#pragma unroll
            for (int kx0 = 0; kx0 < ww; kx0 += KC) {
                f2 s[KC][NP];
                int64_t krow[KC];
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    int code, rc;
                    const int kx = kx0 + c < ww ? kx0 + c : ww - 1;
                    key_of(g, v, rowb, codeb, rcb, kx, krow[c], code, rc);
                    f2 kk[C / 2], tb[NP];
                    sload_row<C>(kk, a.k + krow[c] * a.ks);
                    vload_tab<NP>(tb, a.table + (cq - code) * NH);
                    float madd = 0.f;
                    if (v.masked) madd = rc == rq ? 0.f : kMask2;
                    if (kx0 + c >= ww) madd = -INFINITY;
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        f2 sc = pfma(tb[P], L2E, splat(madd));
                        sc = pfma(aq[2 * P], kk[2 * P], sc);
                        s[c][P] = pfma(aq[2 * P + 1], kk[2 * P + 1], sc);
                    }
                }
                // lazy online max: rescale only when a score passes m + 8
                f2 cm[NP];
                bool need = false;
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    cm[P] = s[0][P];
#pragma unroll
                    for (int c = 1; c < KC; ++c) cm[P] = (f2){fmaxf(cm[P].x, s[c][P].x), fmaxf(cm[P].y, s[c][P].y)};
                    need |= (cm[P].x > m8[P].x) | (cm[P].y > m8[P].y);
                }
                if (__any(need)) {
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        const f2 mn = (f2){fmaxf(m[P].x, cm[P].x), fmaxf(m[P].y, cm[P].y)};
                        const f2 al = exp2_2(m[P] - mn);
                        l[P] *= al;
                        acc[2 * P] *= al;
                        acc[2 * P + 1] *= al;
                        m[P] = mn;
                        m8[P] = mn + splat(kLazy);
                    }
                }
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    f2 vv[C / 2];
                    sload_row<C>(vv, a.v + krow[c] * a.vs);
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        const f2 pj = exp2_2(s[c][P] - m[P]);
                        l[P] += pj;
                        acc[2 * P] = pfma(pj, vv[2 * P], acc[2 * P]);
                        acc[2 * P + 1] = pfma(pj, vv[2 * P + 1], acc[2 * P + 1]);
                    }
                }
            }
        });
        if (act) {
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                const f2 inv = (f2){1.0f / l[P].x, 1.0f / l[P].y};
                acc[2 * P] *= inv;
                acc[2 * P + 1] *= inv;
                const f2 lse2 = m[P] + (f2){fast_log2(l[P].x), fast_log2(l[P].y)};
                *reinterpret_cast<float2*>(a.lse + ti.row * NH + 2 * P) = make_float2(lse2.x, lse2.y);
            }
            vstore_row<C>(a.out + ti.row * a.os, acc, 1.0f);
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
        f2 orow[C / 2], grow[C / 2], vrow[C / 2];
        vload_row<C>(orow, o + r * os);
        vload_row<C>(grow, dout + r * os);
        vload_row<C>(vrow, vv + r * vs);
#pragma unroll
        for (int P = 0; P < NP; ++P) {
            const f2 d = pfma(orow[2 * P], grow[2 * P], orow[2 * P + 1] * grow[2 * P + 1]);
            *reinterpret_cast<float2*>(delta + r * NH + 2 * P) = make_float2(d.x, d.y);
        }
#pragma unroll
        for (int i = 0; i < C / 2; ++i) {
            md = fmaxf(md, fmaxf(fabsf(grow[i].x), fabsf(grow[i].y)));
            mv = fmaxf(mv, fmaxf(fabsf(vrow[i].x), fabsf(vrow[i].y)));
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

template <int C, int WW>
__global__ __launch_bounds__(512, 2) void wattn_bwd_sk_kernel(WAArgs a, int nq, int nunits, const float* delta) {
    constexpr int NH = C / 2, NP = NH / 2;
    constexpr int DS = NH + 1;   // odd u64 stride of the table-gradient rows (spreads LDS banks)
    extern __shared__ __attribute__((aligned(16))) unsigned long long dtab_s[];   // [Tsz][DS]
    const WGeom& g = a.g;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    const f2 L2E = splat(kLog2e);
    const float sl2 = a.scale * kLog2e;
    for (int e = threadIdx.x; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0ull;
    const int fexp = fix_exponent(a.maxbits, 2);
    const float fs = exp2f((float)fexp);     // 2^S: ds * 2^S < 2^30 (wattn_common.h)
    const float ifs = exp2f((float)-fexp);
    __syncthreads();

    for (int u = blockIdx.x * wpb + wave; u < nunits; u += gridDim.x * wpb) {
        const int w = u / nq, qt = u - w * nq;
        const Win v = window_of(g, w);
        const int t = qt * 64 + lane;
        const bool act = t < g.N;
        const TokenInfo ti = token_info(g, w, act ? t : g.N - 1);

        // ================= pass A: lane = query row -> dq, dtable
        {
            f2 aq[C / 2], dOs[C / 2], nlse[NP], ndl[NP], dqa[C / 2];
            vload_row<C>(aq, a.q + ti.row * a.qs);
            vload_row<C>(dOs, a.dout + ti.row * a.os);
            vload_tab<NP>(nlse, a.lse + ti.row * NH);
            vload_tab<NP>(ndl, delta + ti.row * NH);
#pragma unroll
            for (int i = 0; i < C / 2; ++i) {
                aq[i] *= splat(sl2);
                dOs[i] *= splat(act ? fs : 0.f);
                dqa[i] = splat(0.f);
            }
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                nlse[P] = act ? -nlse[P] : splat(-INFINITY);
                ndl[P] *= splat(act ? -fs : 0.f);
            }
            const int cq = ti.code + g.off, rq = ti.rc;
            walk_rows(g, v, [&](int64_t rowb, int codeb, int rcb) {
#pragma unroll
                for (int kx = 0; kx < (WW ? WW : g.ww); ++kx) {
                    int64_t row;
                    int code, rc;
                    key_of(g, v, rowb, codeb, rcb, kx, row, code, rc);
                    f2 kk[C / 2], vk[C / 2], tb[NP];
                    sload_row<C>(kk, a.k + row * a.ks);
                    sload_row<C>(vk, a.v + row * a.vs);
                    const int tix = cq - code;
                    vload_tab<NP>(tb, a.table + tix * NH);
                    f2 base[NP];
                    if (v.masked) {
                        const float madd = rc == rq ? 0.f : kMask2;
#pragma unroll
                        for (int P = 0; P < NP; ++P) base[P] = pfma(tb[P], L2E, nlse[P] + splat(madd));
                    } else {
#pragma unroll
                        for (int P = 0; P < NP; ++P) base[P] = pfma(tb[P], L2E, nlse[P]);
                    }
                    long long fx[NH];
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        f2 sc = pfma(aq[2 * P], kk[2 * P], base[P]);
                        sc = pfma(aq[2 * P + 1], kk[2 * P + 1], sc);
                        const f2 pr = exp2_2(sc);
                        f2 tt = pfma(dOs[2 * P], vk[2 * P], ndl[P]);
                        tt = pfma(dOs[2 * P + 1], vk[2 * P + 1], tt);
                        const f2 dsv = pr * tt;
                        dqa[2 * P] = pfma(dsv, kk[2 * P], dqa[2 * P]);
                        dqa[2 * P + 1] = pfma(dsv, kk[2 * P + 1], dqa[2 * P + 1]);
                        fx[2 * P] = fix_round(dsv.x);
                        fx[2 * P + 1] = fix_round(dsv.y);
                    }
                    unsigned long long* dt = dtab_s + tix * DS;
#pragma unroll
                    for (int h = 0; h < NH; ++h) atomicAdd(&dt[h], (unsigned long long)fx[h]);
                }
            });
            if (act) vstore_row<C>(a.dq + ti.row * a.qs, dqa, a.scale * ifs);
        }

        // ================= pass B: lane = key row -> dk, dv
        {
            f2 kr[C / 2], vr[C / 2], dka[C / 2], dva[C / 2];
            vload_row<C>(kr, a.k + ti.row * a.ks);
            vload_row<C>(vr, a.v + ti.row * a.vs);
#pragma unroll
            for (int i = 0; i < C / 2; ++i) {
                kr[i] *= splat(sl2);
                dka[i] = splat(0.f);
                dva[i] = splat(0.f);
            }
            const int cko = g.off - ti.code, rk = ti.rc;
            walk_rows(g, v, [&](int64_t rowb, int codeb, int rcb) {
#pragma unroll
                for (int qx = 0; qx < (WW ? WW : g.ww); ++qx) {
                    int64_t row;
                    int code, rc;
                    key_of(g, v, rowb, codeb, rcb, qx, row, code, rc);
                    f2 qq[C / 2], gg[C / 2], ll[NP], dd[NP], tb[NP];
                    sload_row<C>(qq, a.q + row * a.qs);
                    sload_row<C>(gg, a.dout + row * a.os);
                    sload_pairs<NP>(ll, a.lse + row * NH);
                    sload_pairs<NP>(dd, delta + row * NH);
                    vload_tab<NP>(tb, a.table + (code + cko) * NH);
                    const float madd = (v.masked && rc != rk) ? kMask2 : 0.f;
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        f2 base = pfma(tb[P], L2E, -ll[P]);
                        if (v.masked) base += splat(madd);
                        f2 sc = pfma(qq[2 * P], kr[2 * P], base);
                        sc = pfma(qq[2 * P + 1], kr[2 * P + 1], sc);
                        const f2 pr = exp2_2(sc);
                        f2 tt = pfma(gg[2 * P], vr[2 * P], gg[2 * P + 1] * vr[2 * P + 1]);
                        const f2 dsv = pr * (tt - dd[P]);
                        dva[2 * P] = pfma(pr, gg[2 * P], dva[2 * P]);
                        dva[2 * P + 1] = pfma(pr, gg[2 * P + 1], dva[2 * P + 1]);
                        dka[2 * P] = pfma(dsv, qq[2 * P], dka[2 * P]);
                        dka[2 * P + 1] = pfma(dsv, qq[2 * P + 1], dka[2 * P + 1]);
                    }
                }
            });
            if (act) {
                vstore_row<C>(a.dk + ti.row * a.ks, dka, a.scale);
                vstore_row<C>(a.dv + ti.row * a.vs, dva, 1.0f);
            }
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < g.Tsz * NH; e += blockDim.x) {
        const unsigned long long x = dtab_s[(e / NH) * DS + e % NH];
        if (x != 0ull) atomicAdd(&a.dtab_fix[e], x);
    }
}

}  // namespace sk

// ------------------------------------------------------------------------------------
// host side (called from wattn.hip for layout 1)
// ------------------------------------------------------------------------------------
static int sk_units(const WGeom& g, int& nq) {
    nq = (g.N + 63) / 64;
    return g.nwin * nq;
}

int wattn_sk_fwd(const WAArgs& a, int C, hipStream_t stream) {
    int nq;
    const int units = sk_units(a.g, nq);
    const int wpb = 8;
    int grid = (units + wpb - 1) / wpb;
    if (grid > 5 * kNumCU / 2) grid = 5 * kNumCU / 2;   // 5 waves per SIMD at <= 96 VGPRs
    const bool w6 = a.g.ww == 6;
    if (C == 12) {
        if (w6) sk::wattn_fwd_sk_kernel<12, 3, 6><<<grid, 64 * wpb, 0, stream>>>(a, nq, units);
        else sk::wattn_fwd_sk_kernel<12, 3, 0><<<grid, 64 * wpb, 0, stream>>>(a, nq, units);
    } else if (C == 24) {
        if (w6) sk::wattn_fwd_sk_kernel<24, 3, 6><<<grid, 64 * wpb, 0, stream>>>(a, nq, units);
        else sk::wattn_fwd_sk_kernel<24, 3, 0><<<grid, 64 * wpb, 0, stream>>>(a, nq, units);
    } else {
        set_error("wattn (pair layout): C=%d unsupported (12 or 24)", C);
        return -2;
    }
    return launch_status("wattn_fwd_sk");
}

size_t wattn_sk_workspace(const WGeom& g, int heads) {
    return (size_t)g.Tsz * heads * 8 + 16 + (size_t)g.nwin * g.N * heads * 4;
}

int wattn_sk_bwd(const WAArgs& a0, int C, int heads, void* workspace, hipStream_t stream) {
    WAArgs a = a0;
    const WGeom& g = a.g;
    const int ntab = g.Tsz * heads;
    a.dtab_fix = reinterpret_cast<unsigned long long*>(workspace);
    a.maxbits = reinterpret_cast<unsigned int*>(a.dtab_fix + ntab);
    float* delta = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + (size_t)ntab * 8 + 16);
    hipError_t e = hipMemsetAsync(workspace, 0, (size_t)ntab * 8 + 16, stream);
    if (e != hipSuccess) { set_error("wattn_bwd memset: %s", hipGetErrorString(e)); return (int)e; }
    const int64_t T = (int64_t)g.nwin * g.N;
    int nq;
    const int units = sk_units(g, nq);
    const int wpb = 8;
    int grid = (units + wpb - 1) / wpb;
    if (grid > 2 * kNumCU) grid = 2 * kNumCU;
    const size_t lds = (size_t)g.Tsz * (heads + 1) * 8;
    if (lds > 80 * 1024) {
        set_error("wattn_bwd (pair layout): table-gradient LDS %zu B exceeds 80 KiB", lds);
        return -2;
    }
    void* kern = nullptr;
    if (C == 12) {
        sk::wattn_prep_sk_kernel<12><<<1024, 256, 0, stream>>>(a.o, a.dout, a.os, a.v, a.vs, T, delta, a.maxbits);
        kern = a.g.ww == 6 ? reinterpret_cast<void*>(&sk::wattn_bwd_sk_kernel<12, 6>)
                           : reinterpret_cast<void*>(&sk::wattn_bwd_sk_kernel<12, 0>);
    } else if (C == 24) {
        sk::wattn_prep_sk_kernel<24><<<1024, 256, 0, stream>>>(a.o, a.dout, a.os, a.v, a.vs, T, delta, a.maxbits);
        kern = a.g.ww == 6 ? reinterpret_cast<void*>(&sk::wattn_bwd_sk_kernel<24, 6>)
                           : reinterpret_cast<void*>(&sk::wattn_bwd_sk_kernel<24, 0>);
    } else {
        set_error("wattn (pair layout): C=%d unsupported (12 or 24)", C);
        return -2;
    }
    int rc = launch_status("wattn_prep_sk");
    if (rc) return rc;
    if (lds > 64 * 1024) {
        e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
        if (e != hipSuccess) { set_error("hipFuncSetAttribute: %s", hipGetErrorString(e)); return (int)e; }
    }
    int nq_ = nq, units_ = units;
    const float* delta_c = delta;
    void* args[] = {&a, &nq_, &units_, &delta_c};
    e = hipLaunchKernel(kern, dim3(grid), dim3(64 * wpb), args, lds, stream);
    if (e != hipSuccess) { set_error("wattn_bwd_sk launch: %s", hipGetErrorString(e)); return (int)e; }
    return 0;
}

}  // namespace mmni
