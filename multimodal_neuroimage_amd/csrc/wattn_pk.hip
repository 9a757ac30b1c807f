// Packed-fp32 window attention for head_dim 2 (SwinFusion: C = 12 / 6 heads, C = 24 / 12 heads).
//
// Same algorithm, LDS layout and persistent grid as the generic kernels in wattn.hip (see the
// design notes there); the difference is the register/LDS row layout, which lets every per-head
// operation of the inner loops run on v_pk_{fma,mul,add}_f32 (two heads per instruction).
//
// Why: at head_dim 2 the kernels are VALU-issue-bound, not HBM-bound.  The generic forward
// spends ~12 VALU issue slots per (query, key, head); half of them are the per-head scalar
// FMAs/adds of the dot product, the bias/mask add, the l and acc updates.  Pairing heads
// (h, h+1) into a float2 halves those; v_exp_f32 (8-cycle issue) stays scalar.
//
// Row layout ("pk"): channel (head h, dim c) of a C-wide row sits at
//   pkpos(h, c) = (h / 2) * 4 + c * 2 + (h % 2)
// so float2 element 2P + c of a row holds dim c of heads (2P, 2P + 1).  Q/K/V rows are
// permuted into it when staged, dq/dk/dv/out are permuted back before the store.
#include "wattn_common.h"

#include <type_traits>

// Kernel ablations for experiments only (scripts/build_variant.sh): bit 0 drops the table-gradient
// atomics, bit 1 the pass-B loop, bit 2 the pass-A loop.  Product builds use 0.
#ifndef MMNI_ABL
#define MMNI_ABL 0
#endif
#ifndef MMNI_PK2_PAIRQ
#define MMNI_PK2_PAIRQ 0   // two-row backward pass B: queries i and i + N/2 together (3 table reads per 4 pairs; measured slower)
#endif
#ifndef MMNI_PK2_OPAQUE
#define MMNI_PK2_OPAQUE 1   // two-row backward: row base opaque per window (no hoisted addresses)
#endif

namespace mmni {

typedef float f2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int pkpos(int h, int c) { return (h >> 1) * 4 + c * 2 + (h & 1); }

__device__ __forceinline__ f2 splat(float x) { return (f2){x, x}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 exp2_2(f2 x) { return (f2){fast_exp2(x.x), fast_exp2(x.y)}; }
__device__ __forceinline__ f2 max2(f2 a, f2 b) { return (f2){fmaxf(a.x, b.x), fmaxf(a.y, b.y)}; }
__device__ __forceinline__ f2 shfl2(f2 v, int o) { return (f2){__shfl_xor(v.x, o), __shfl_xor(v.y, o)}; }

// natural row (head-major) -> pk float2 array
template <int C>
__device__ __forceinline__ void pack_row(f2 (&d)[C / 2], const float (&s)[C]) {
#pragma unroll
    for (int P = 0; P < C / 4; ++P)
#pragma unroll
        for (int c = 0; c < 2; ++c) d[P * 2 + c] = (f2){s[(2 * P) * 2 + c], s[(2 * P + 1) * 2 + c]};
}

// pk float2 array -> natural row
template <int C>
__device__ __forceinline__ void unpack_row(float (&d)[C], const f2 (&s)[C / 2]) {
#pragma unroll
    for (int P = 0; P < C / 4; ++P)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            d[(2 * P) * 2 + c] = s[P * 2 + c].x;
            d[(2 * P + 1) * 2 + c] = s[P * 2 + c].y;
        }
}

template <int C>
__device__ __forceinline__ void store_pk(float* dst, const f2 (&s)[C / 2]) {
#pragma unroll
    for (int i = 0; i < C / 2; i += 2)
        *reinterpret_cast<float4*>(dst + 2 * i) = make_float4(s[i].x, s[i].y, s[i + 1].x, s[i + 1].y);
}

// natural row in global memory -> pk float2 array, straight from float4 loads: float4 P of a row
// holds (h 2P c0, h 2P c1, h 2P+1 c0, h 2P+1 c1), i.e. pk elements 2P = (x, z) and 2P+1 = (y, w).
// (Going through a float[C] array lets the compiler shuffle the pairs through scratch memory.)
template <int C>
__device__ __forceinline__ void load_pk(f2 (&d)[C / 2], const float* src) {
#pragma unroll
    for (int P = 0; P < C / 4; ++P) {
        const float4 t = *reinterpret_cast<const float4*>(src + 4 * P);
        d[2 * P] = (f2){t.x, t.z};
        d[2 * P + 1] = (f2){t.y, t.w};
    }
}

// pk float2 array -> natural row in global memory, scaled
template <int C>
__device__ __forceinline__ void store_nat(float* dst, const f2 (&s)[C / 2], float scale) {
#pragma unroll
    for (int P = 0; P < C / 4; ++P)
        *reinterpret_cast<float4*>(dst + 4 * P) = make_float4(s[2 * P].x * scale, s[2 * P + 1].x * scale,
                                                              s[2 * P].y * scale, s[2 * P + 1].y * scale);
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int C, int KIND, int MAXT>
__global__ __launch_bounds__(MAXT, C == 12 ? 4 : 1) void wattn_fwd_pk_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB;
    float* kv_s = smem;                                              // [WPB*NPAD][2C] pk k | pk v
    int2* meta_s = reinterpret_cast<int2*>(kv_s + (size_t)WPB * NPAD * 2 * C);  // [WPB*NPAD]
    float* tab_s = reinterpret_cast<float*>(meta_s + WPB * NPAD);     // [Tsz][NH]

    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / N, t = r - wl * N;
    const int wl_c = wl < WPB ? wl : WPB - 1;

    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) tab_s[e] = a.table[e] * kLog2e;

    f2 tau2[NP];
#pragma unroll
    for (int P = 0; P < NP; ++P)
        tau2[P] = (KIND == 1) ? (f2){a.tau[2 * P], a.tau[2 * P + 1]} * kLog2e : splat(a.scale * kLog2e);

    float vabs = 0.f;   // running max|v| of the rows this thread staged (for the backward's bound)
    for (int grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
        for (int e = tid; e < WPB * NPAD; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            const int w = grp * WPB + w2;
            float kr[C], vr[C];
            int2 mt;
            if (t2 < N && w < g.nwin) {
                const TokenInfo ti = token_info(g, w, t2);
                load_row<C>(kr, a.k + ti.row * a.ks);
                load_row<C>(vr, a.v + ti.row * a.vs);
#pragma unroll
                for (int c = 0; c < C; ++c) vabs = fmaxf(vabs, fabsf(vr[c]));
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kr, nrm); }
                mt = make_int2(ti.code | (ti.rc << 16), 0);
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) { kr[c] = 0.f; vr[c] = 0.f; }
                mt = make_int2(0, __float_as_int(-INFINITY));
            }
            f2 kp[C / 2], vp[C / 2];
            pack_row<C>(kp, kr);
            pack_row<C>(vp, vr);
            store_pk<C>(kv_s + (size_t)e * 2 * C, kp);
            store_pk<C>(kv_s + (size_t)e * 2 * C + C, vp);
            meta_s[e] = mt;
        }

        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        f2 q[C / 2];
        int cq = 0, rq = 0;
        int64_t row = 0;
        {
            float qr[C];
            if (active) {
                const TokenInfo ti = token_info(g, w, t);
                row = ti.row;
                cq = ti.code + g.off;
                rq = ti.rc;
                load_row<C>(qr, a.q + row * a.qs);
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(qr, nrm); }
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) qr[c] = 0.f;
            }
            pack_row<C>(q, qr);
#pragma unroll
            for (int P = 0; P < NP; ++P) { q[2 * P] *= tau2[P]; q[2 * P + 1] *= tau2[P]; }
        }
        __syncthreads();

        f2 m[NP], l[NP], acc[C / 2];
#pragma unroll
        for (int P = 0; P < NP; ++P) { m[P] = splat(-INFINITY); l[P] = splat(0.f); }
#pragma unroll
        for (int i = 0; i < C / 2; ++i) acc[i] = splat(0.f);

        const float* kvw = kv_s + (size_t)wl_c * NPAD * 2 * C;
        const int2* mw = meta_s + wl_c * NPAD;
        const int nk = NPAD / KS;
        for (int n = 0; n < nk; n += kPkChunk) {
            f2 s[kPkChunk][NP];
#pragma unroll
            for (int cc = 0; cc < kPkChunk; ++cc) {
                const int j = p + KS * (n + cc);
                const int2 mt = mw[j];
                const int code = mt.x & 0xffff, rcj = mt.x >> 16;
                const float madd = (rcj == rq ? 0.f : kMask2) + __int_as_float(mt.y);
                const f2* tb = reinterpret_cast<const f2*>(tab_s + (cq - code) * NH);
                const f2* kr = reinterpret_cast<const f2*>(kvw + (size_t)j * 2 * C);
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 d = tb[P] + splat(madd);
                    d = pfma(q[2 * P], kr[2 * P], d);
                    s[cc][P] = pfma(q[2 * P + 1], kr[2 * P + 1], d);
                }
            }
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                f2 cm = s[0][P];
#pragma unroll
                for (int cc = 1; cc < kPkChunk; ++cc) cm = max2(cm, s[cc][P]);
                const f2 mn = max2(m[P], cm);
                const f2 al = exp2_2(m[P] - mn);
                m[P] = mn;
                l[P] *= al;
                acc[2 * P] *= al;
                acc[2 * P + 1] *= al;
            }
#pragma unroll
            for (int cc = 0; cc < kPkChunk; ++cc) {
                const int j = p + KS * (n + cc);
                const f2* vr = reinterpret_cast<const f2*>(kvw + (size_t)j * 2 * C + C);
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    const f2 pj = exp2_2(s[cc][P] - m[P]);
                    l[P] += pj;
                    acc[2 * P] = pfma(pj, vr[2 * P], acc[2 * P]);
                    acc[2 * P + 1] = pfma(pj, vr[2 * P + 1], acc[2 * P + 1]);
                }
            }
        }
        for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                const f2 mo = shfl2(m[P], o), lo = shfl2(l[P], o);
                const f2 mn = max2(m[P], mo);
                const f2 fa = exp2_2(m[P] - mn), fb = exp2_2(mo - mn);
                l[P] = l[P] * fa + lo * fb;
#pragma unroll
                for (int c = 0; c < 2; ++c) acc[2 * P + c] = acc[2 * P + c] * fa + shfl2(acc[2 * P + c], o) * fb;
                m[P] = mn;
            }
        }
        if (active && p == 0) {
            f2 op[C / 2];
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                const f2 inv = (f2){1.0f / l[P].x, 1.0f / l[P].y};
                op[2 * P] = acc[2 * P] * inv;
                op[2 * P + 1] = acc[2 * P + 1] * inv;
                a.lse[row * NH + 2 * P] = (m[P].x + fast_log2(l[P].x)) * kLn2;
                a.lse[row * NH + 2 * P + 1] = (m[P].y + fast_log2(l[P].y)) * kLn2;
            }
            float o[C];
            unpack_row<C>(o, op);
            store_row<C>(a.out + row * a.os, o);
        }
        __syncthreads();
    }
    if (a.vmax != nullptr) {
        for (int o = 32; o > 0; o >>= 1) vabs = fmaxf(vabs, __shfl_xor(vabs, o));
        if ((tid & 63) == 0) atomicMax(a.vmax, __float_as_uint(vabs));
    }
}

// ------------------------------------------------------------------------------------
// forward, two queries per lane
// ------------------------------------------------------------------------------------
// The forward above is bound by LDS instructions, not VALU: per (query, key) a lane reads the key
// row (3 x b128), the value row (3 x b128), the bias-table row and the key metadata, and a
// broadcast ds_read_b128 costs the same LDS cycles as a scattered one.  Here each lane carries
// queries t and t + N/2 of its window against the same keys, so every K/V/metadata read serves
// two queries (LDS instructions per query-key pair 8.5 -> 5).  Lanes per window: N/2 x KS.
template <int C, int KIND, int MAXT, int QPL = 2>
__global__ __launch_bounds__(MAXT) void wattn_fwd_pk2_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2, CK = MMNI_PK2_CHUNK;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB, NHALF = N / QPL;   // QPL queries per lane: t, t + N/QPL, ...
    float* kv_s = smem;                                              // [WPB*NPAD][2C] pk k | pk v
    int2* meta_s = reinterpret_cast<int2*>(kv_s + (size_t)WPB * NPAD * 2 * C);  // [WPB*NPAD]
    float* tab_s = reinterpret_cast<float*>(meta_s + WPB * NPAD);     // [Tsz][NH]

    // head groups (a.hsplit > 1): as in wattn_bwd_pk2_kernel, the NHG blocks of a window group
    // sit 8 block indices apart (one XCD) and take heads [h0, h0 + NH) of NHT
    const int NHG = a.hsplit;
    const int xslot = blockIdx.x >> 3;
    const int hg = NHG > 1 ? xslot % NHG : 0;
    const int gfirst = NHG > 1 ? (xslot / NHG) * 8 + (blockIdx.x & 7) : blockIdx.x;
    const int h0 = hg * NH, NHT = NH * NHG, coff = h0 * HD;
    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / NHALF, t = r - wl * NHALF;
    const int wl_c = wl < WPB ? wl : WPB - 1;

    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) tab_s[e] = a.table[(e / NH) * NHT + h0 + e % NH] * kLog2e;

    f2 tau2[NP];
#pragma unroll
    for (int P = 0; P < NP; ++P)
        tau2[P] = (KIND == 1) ? (f2){a.tau[h0 + 2 * P], a.tau[h0 + 2 * P + 1]} * kLog2e : splat(a.scale * kLog2e);

    float vabs = 0.f;
    for (int grp = gfirst; grp < a.ngroups; grp += gridDim.x / NHG) {
        for (int e = tid; e < WPB * NPAD; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            const int w = grp * WPB + w2;
            float kr[C], vr[C];
            int2 mt;
            if (t2 < N && w < g.nwin) {
                const TokenInfo ti = token_info(g, w, t2);
                load_row<C>(kr, a.k + ti.row * a.ks + coff);
                load_row<C>(vr, a.v + ti.row * a.vs + coff);
#pragma unroll
                for (int c = 0; c < C; ++c) vabs = fmaxf(vabs, fabsf(vr[c]));
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kr, nrm); }
                mt = make_int2(ti.code | (ti.rc << 16), 0);
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) { kr[c] = 0.f; vr[c] = 0.f; }
                mt = make_int2(0, __float_as_int(-INFINITY));
            }
            f2 kp[C / 2], vp[C / 2];
            pack_row<C>(kp, kr);
            pack_row<C>(vp, vr);
            store_pk<C>(kv_s + (size_t)e * 2 * C, kp);
            store_pk<C>(kv_s + (size_t)e * 2 * C + C, vp);
            meta_s[e] = mt;
        }

        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        f2 q[QPL][C / 2];
        int cq[QPL] = {}, rq[QPL] = {};
        int64_t row[QPL] = {};
#pragma unroll
        for (int u = 0; u < QPL; ++u) {
            float qr[C];
            if (active) {
                const TokenInfo ti = token_info(g, w, t + u * NHALF);
                row[u] = ti.row;
                cq[u] = ti.code + g.off;
                rq[u] = ti.rc;
                load_row<C>(qr, a.q + ti.row * a.qs + coff);
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(qr, nrm); }
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) qr[c] = 0.f;
            }
            pack_row<C>(q[u], qr);
#pragma unroll
            for (int P = 0; P < NP; ++P) { q[u][2 * P] *= tau2[P]; q[u][2 * P + 1] *= tau2[P]; }
        }
        __syncthreads();

        f2 m[QPL][NP], l[QPL][NP], acc[QPL][C / 2];
#pragma unroll
        for (int u = 0; u < QPL; ++u) {
#pragma unroll
            for (int P = 0; P < NP; ++P) { m[u][P] = splat(-INFINITY); l[u][P] = splat(0.f); }
#pragma unroll
            for (int i = 0; i < C / 2; ++i) acc[u][i] = splat(0.f);
        }

        const float* kvw = kv_s + (size_t)wl_c * NPAD * 2 * C;
        const int2* mw = meta_s + wl_c * NPAD;
        const int nk = NPAD / KS;
        for (int n = 0; n < nk; n += CK) {
            f2 s[QPL][CK][NP];
#pragma unroll
            for (int cc = 0; cc < CK; ++cc) {
                const int j = p + KS * (n + cc);
                const int2 mt = mw[j];
                const int code = mt.x & 0xffff, rcj = mt.x >> 16;
                const f2* kr = reinterpret_cast<const f2*>(kvw + (size_t)j * 2 * C);
                f2 kk[C / 2];
#pragma unroll
                for (int i = 0; i < C / 2; ++i) kk[i] = kr[i];
#pragma unroll
                for (int u = 0; u < QPL; ++u) {
                    const float madd = (rcj == rq[u] ? 0.f : kMask2) + __int_as_float(mt.y);
                    const f2* tb = reinterpret_cast<const f2*>(tab_s + (cq[u] - code) * NH);
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        f2 d = tb[P] + splat(madd);
                        d = pfma(q[u][2 * P], kk[2 * P], d);
                        s[u][cc][P] = pfma(q[u][2 * P + 1], kk[2 * P + 1], d);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < QPL; ++u) {
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 cm = s[u][0][P];
#pragma unroll
                    for (int cc = 1; cc < CK; ++cc) cm = max2(cm, s[u][cc][P]);
                    const f2 mn = max2(m[u][P], cm);
                    const f2 al = exp2_2(m[u][P] - mn);
                    m[u][P] = mn;
                    l[u][P] *= al;
                    acc[u][2 * P] *= al;
                    acc[u][2 * P + 1] *= al;
                }
            }
#pragma unroll
            for (int cc = 0; cc < CK; ++cc) {
                const int j = p + KS * (n + cc);
                const f2* vr = reinterpret_cast<const f2*>(kvw + (size_t)j * 2 * C + C);
                f2 vv[C / 2];
#pragma unroll
                for (int i = 0; i < C / 2; ++i) vv[i] = vr[i];
#pragma unroll
                for (int u = 0; u < QPL; ++u) {
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        const f2 pj = exp2_2(s[u][cc][P] - m[u][P]);
                        l[u][P] += pj;
                        acc[u][2 * P] = pfma(pj, vv[2 * P], acc[u][2 * P]);
                        acc[u][2 * P + 1] = pfma(pj, vv[2 * P + 1], acc[u][2 * P + 1]);
                    }
                }
            }
        }
        for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
            for (int u = 0; u < QPL; ++u) {
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    const f2 mo = shfl2(m[u][P], o), lo = shfl2(l[u][P], o);
                    const f2 mn = max2(m[u][P], mo);
                    const f2 fa = exp2_2(m[u][P] - mn), fb = exp2_2(mo - mn);
                    l[u][P] = l[u][P] * fa + lo * fb;
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        acc[u][2 * P + c] = acc[u][2 * P + c] * fa + shfl2(acc[u][2 * P + c], o) * fb;
                    m[u][P] = mn;
                }
            }
        }
        if (active && p == 0) {
#pragma unroll
            for (int u = 0; u < QPL; ++u) {
                f2 op[C / 2];
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    const f2 inv = (f2){1.0f / l[u][P].x, 1.0f / l[u][P].y};
                    op[2 * P] = acc[u][2 * P] * inv;
                    op[2 * P + 1] = acc[u][2 * P + 1] * inv;
                    a.lse[row[u] * NHT + h0 + 2 * P] = (m[u][P].x + fast_log2(l[u][P].x)) * kLn2;
                    a.lse[row[u] * NHT + h0 + 2 * P + 1] = (m[u][P].y + fast_log2(l[u][P].y)) * kLn2;
                }
                float o[C];
                unpack_row<C>(o, op);
                store_row<C>(a.out + row[u] * a.os + coff, o);
            }
        }
        __syncthreads();
    }
    if (a.vmax != nullptr) {
        for (int o = 32; o > 0; o >>= 1) vabs = fmaxf(vabs, __shfl_xor(vabs, o));
        if ((tid & 63) == 0) atomicMax(a.vmax, __float_as_uint(vabs));
    }
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
// Same two-pass flash-style structure as wattn_bwd_kernel (pass A: lane = query row -> dq and
// the table / tau gradients; pass B: lane = key row -> dk, dv), rewritten for issue efficiency:
//  * Shift-mask and pad handling only in windows that need it: a window is mask-free unless it
//    is the last one along a shifted axis (shift_region), i.e. ~82% of the windows of a shifted
//    96^3 block and all windows of an unshifted one.  The mask-free loop has no region test.
//  * The fixed-point scale 2^S of the table gradient is folded into dO and delta, so ds comes out
//    pre-scaled; dq/dk/dv accumulate the scaled values and are multiplied by 2^-S (exact) once.
//  * dO.v - delta is one fma chain seeded with -delta; the fixed-point rounding is a single
//    v_cvt_rpi_i32_f32 (round half up).
//  * The metadata of the next key is prefetched, and the table-gradient atomics of a key are
//    issued one iteration late, after the next key's LDS reads: LDS operations complete in order,
//    so an atomic issued ahead of a read would make the read's wait include it.
__device__ __forceinline__ long long fix_round(float x) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return (long long)r;
}

// window of a group needs the region test (last window along a shifted axis) or pad keys
__device__ __forceinline__ bool group_masked(const WGeom& g, int grp, int WPB, int NPAD) {
    if (NPAD != g.N) return true;
    for (int w2 = 0; w2 < WPB; ++w2) {
        int w = grp * WPB + w2;
        if (w >= g.nwin) return true;
        const int wx = w % g.nWw; w /= g.nWw;
        const int wy = w % g.nWh; w /= g.nWh;
        const int wz = w % g.nWd;
        if ((g.sw && wx == g.nWw - 1) || (g.sh && wy == g.nWh - 1) || (g.sd && wz == g.nWd - 1)) return true;
    }
    return false;
}

template <int C>
__device__ __forceinline__ void lds_row(f2 (&d)[C / 2], const float* s) {
#pragma unroll
    for (int i = 0; i < C / 2; i += 2) {
        const float4 t = *reinterpret_cast<const float4*>(s + 2 * i);
        d[i] = (f2){t.x, t.y};
        d[i + 1] = (f2){t.z, t.w};
    }
}

// position of float h of table row `row` (NHP floats per row, float4 chunks optionally swizzled)
template <int NHP>
__device__ __forceinline__ int tab_pos(int row, int h) {
    if constexpr (NHP == 2) return row * 2 + h;   // two-head rows: one 8-B read, no swizzle
    constexpr int NCH = NHP / 4;   // float4 chunks per row; the swizzle needs a power of two
    const int c = h >> 2;
    const int cs = (kTabSwz && (NCH & (NCH - 1)) == 0) ? (c ^ ((row >> 3) & (NCH - 1))) : c;
    return row * NHP + cs * 4 + (h & 3);
}

// table row (NHP floats, NHP % 4 == 0) -> NP float2
template <int NP, int NHP>
__device__ __forceinline__ void lds_tab(f2 (&d)[NP], const float* tab, int row) {
    if constexpr (NHP == 2) {
        d[0] = *reinterpret_cast<const f2*>(tab + row * 2);
        return;
    }
    float t[NHP];
#pragma unroll
    for (int i = 0; i < NHP; i += 4) {
        const float4 x = *reinterpret_cast<const float4*>(tab + tab_pos<NHP>(row, i));
        t[i] = x.x; t[i + 1] = x.y; t[i + 2] = x.z; t[i + 3] = x.w;
    }
#pragma unroll
    for (int P = 0; P < NP; ++P) d[P] = (f2){t[2 * P], t[2 * P + 1]};
}

template <int C, int KIND, int MAXT>
__global__ __launch_bounds__(MAXT) void wattn_bwd_pk_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2;
    constexpr int NHP = (NH + 3) & ~3;   // table row stride (float4 reads)
    constexpr int DS = NH + kDtabPad;    // table-gradient row stride in words (odd: spreads LDS banks)
    // block-local table-gradient sums: 64-bit, or 32-bit with the fixed-point scale lowered by
    // fix_shift bits so that every block's sums fit (host: 2^fix_shift >= windows per block * N / 2)
    using dt_t = std::conditional_t<kDtab32, unsigned int, unsigned long long>;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB;
    const int T = WPB * NPAD;
    float* rowb = smem;                                   // [T][2C]: pass A pk k | pk v; pass B pk a2 | pk dOs
    float* rs_s = smem + (size_t)T * 2 * C;               // [T][2NH]: pass B lse2 | -delta*2^S (pk pairs)
    int2* meta_s = reinterpret_cast<int2*>(rs_s + (size_t)T * 2 * NH);
    float* tab_s = reinterpret_cast<float*>(meta_s + T);  // [Tsz][NHP], log2-domain bias
    dt_t* dtab_s = reinterpret_cast<dt_t*>(tab_s + (size_t)g.Tsz * NHP);
    float* dtau_s = reinterpret_cast<float*>(dtab_s + (size_t)g.Tsz * DS);

    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / N, t = r - wl * N;
    const int wl_c = wl < WPB ? wl : WPB - 1;
    const int lane = tid & 63;

    for (int e = tid; e < g.Tsz * NHP; e += blockDim.x) {
        const int row = e / NHP, h = e - row * NHP;
        tab_s[tab_pos<NHP>(row, h)] = h < NH ? a.table[row * NH + h] * kLog2e : 0.f;
    }
    for (int e = tid; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0;
    if (tid < NH) dtau_s[tid] = 0.f;
    const int fexp = fix_exponent(a.maxbits, HD) - a.fix_shift;
    const float fs = exp2f((float)fexp);       // 2^S
    const float ifs = exp2f((float)-fexp);     // 2^-S (exact)
    f2 dtr[NP];
#pragma unroll
    for (int P = 0; P < NP; ++P) dtr[P] = splat(0.f);
    const int nk = NPAD / KS;                  // keys (pass A) / queries (pass B) per lane, even

    for (int grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        const bool masked = group_masked(g, grp, WPB, NPAD);
        const int own = wl_c * NPAD + (active ? t : 0);
        f2 aq[C / 2], dO[C / 2], lse2[NP], ndl[NP];
        int64_t row = 0;
        int code = 0, rc = 0;
        if (active) {
            const TokenInfo ti = token_info(g, w, t);
            row = ti.row;
            code = ti.code;
            rc = ti.rc;
            if constexpr (KIND == 1) {
                float qr[C], nrm[NH];
                load_row<C>(qr, a.q + row * a.qs);
                normalize_heads<C, HD>(qr, nrm);
                pack_row<C>(aq, qr);
            } else {
                load_pk<C>(aq, a.q + row * a.qs);
            }
            f2 orow[C / 2];
            load_pk<C>(dO, a.dout + row * a.os);
            load_pk<C>(orow, a.o + row * a.os);
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                const f2 t2 = (KIND == 1) ? (f2){a.tau[2 * P], a.tau[2 * P + 1]} * kLog2e : splat(a.scale * kLog2e);
                aq[2 * P] *= t2;
                aq[2 * P + 1] *= t2;
                const f2 dd = pfma(orow[2 * P], dO[2 * P], orow[2 * P + 1] * dO[2 * P + 1]);
                ndl[P] = dd * splat(-fs);
                dO[2 * P] *= splat(fs);
                dO[2 * P + 1] *= splat(fs);
                lse2[P] = (f2){a.lse[row * NH + 2 * P], a.lse[row * NH + 2 * P + 1]} * kLog2e;
            }
        } else {
#pragma unroll
            for (int i = 0; i < C / 2; ++i) { aq[i] = splat(0.f); dO[i] = splat(0.f); }
#pragma unroll
            for (int P = 0; P < NP; ++P) { lse2[P] = splat(INFINITY); ndl[P] = splat(0.f); }
        }
        // ---- stage K/V + metadata (owners write their row; pad rows get neutral values)
        if (active && p == 0) {
            f2 kp[C / 2], vp[C / 2];
            if constexpr (KIND == 1) {
                float kr[C], nrm[NH];
                load_row<C>(kr, a.k + row * a.ks);
                normalize_heads<C, HD>(kr, nrm);
                pack_row<C>(kp, kr);
            } else {
                load_pk<C>(kp, a.k + row * a.ks);
            }
            load_pk<C>(vp, a.v + row * a.vs);
            store_pk<C>(rowb + (size_t)own * 2 * C, kp);
            store_pk<C>(rowb + (size_t)own * 2 * C + C, vp);
            meta_s[own] = make_int2(code | (rc << 16), 0);
        }
        if (masked) {
            for (int e = tid; e < T; e += blockDim.x) {
                const int w2 = e / NPAD, t2 = e - w2 * NPAD;
                if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                    float4* z = reinterpret_cast<float4*>(rowb + (size_t)e * 2 * C);
#pragma unroll
                    for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                    meta_s[e] = make_int2(0x7fff0000, __float_as_int(-INFINITY));
                }
            }
        }
        __syncthreads();
        const int2* mw = meta_s + wl_c * NPAD;

        // ================= pass A: lane = query row -> dq, dtable, dtau
        {
            const float* kvw = rowb + (size_t)wl_c * NPAD * 2 * C;
            f2 dqa[C / 2];
#pragma unroll
            for (int i = 0; i < C / 2; ++i) dqa[i] = splat(0.f);
            const int cq = code + g.off;
            // lane p walks its own contiguous slice of the keys (keys N/KS apart never share a
            // relative offset within a wave's consecutive queries: fewer same-address atomics)
            const int jb = p * nk;
            int2 mm = mw[jb];
            // deferred table-gradient atomics of the previous key (issued after this key's reads)
            dt_t* dtp = dtab_s;
            long long fx[NH];
#pragma unroll
            for (int h = 0; h < NH; ++h) fx[h] = 0;
            for (int n = 0; n < ((MMNI_ABL & 4) ? 0 : nk); ++n) {
                const int j = jb + n;
                const int2 mnext = mw[j + 1];   // prefetch (reads past the slice on the last key: unused)
                const int tix = cq - (mm.x & 0xffff);
                f2 tb[NP], kj[C / 2], vj[C / 2];
                lds_tab<NP, NHP>(tb, tab_s, tix);
                lds_row<C>(kj, kvw + (size_t)j * 2 * C);
                lds_row<C>(vj, kvw + (size_t)j * 2 * C + C);
#pragma unroll
                for (int h = 0; h < NH; ++h)
                    if (!(MMNI_ABL & 1)) atomicAdd(&dtp[h], (dt_t)fx[h]);
                dtp = dtab_s + tix * DS;
                f2 base[NP];
                if (masked) {
                    const float madd = ((mm.x >> 16) == rc ? 0.f : kMask2) + __int_as_float(mm.y);
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] + (splat(madd) - lse2[P]);
                } else {
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] - lse2[P];
                }
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 pr, dsv;
                    if constexpr (KIND == 1) {
                        f2 dot = aq[2 * P] * kj[2 * P];
                        dot = pfma(aq[2 * P + 1], kj[2 * P + 1], dot);
                        pr = exp2_2(dot + base[P]);
                        f2 tt = pfma(dO[2 * P], vj[2 * P], ndl[P]);
                        tt = pfma(dO[2 * P + 1], vj[2 * P + 1], tt);
                        dsv = pr * tt;
                        dtr[P] = pfma(dsv, dot, dtr[P]);
                    } else {
                        f2 sc = pfma(aq[2 * P], kj[2 * P], base[P]);
                        sc = pfma(aq[2 * P + 1], kj[2 * P + 1], sc);
                        pr = exp2_2(sc);
                        f2 tt = pfma(dO[2 * P], vj[2 * P], ndl[P]);
                        tt = pfma(dO[2 * P + 1], vj[2 * P + 1], tt);
                        dsv = pr * tt;
                    }
                    dqa[2 * P] = pfma(dsv, kj[2 * P], dqa[2 * P]);
                    dqa[2 * P + 1] = pfma(dsv, kj[2 * P + 1], dqa[2 * P + 1]);
                    fx[2 * P] = fix_round(dsv.x);
                    fx[2 * P + 1] = fix_round(dsv.y);
                }
                mm = mnext;
            }
#pragma unroll
            for (int h = 0; h < NH; ++h) atomicAdd(&dtp[h], (dt_t)fx[h]);
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) dqa[i] += shfl2(dqa[i], o);
            }
            if (active && p == 0) {
                if constexpr (KIND == 1) {
                    float dqn[C], dq[C];
                    unpack_row<C>(dqn, dqa);
                    float qr[C], nrm[NH];
                    load_row<C>(qr, a.q + row * a.qs);
                    normalize_heads<C, HD>(qr, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dqn[h * HD + c] * (a.tau[h] * ifs);
                        normalize_bwd<HD>(dq + h * HD, dy, qr + h * HD, nrm[h]);
                    }
                    store_row<C>(a.dq + row * a.qs, dq);
                } else {
                    store_nat<C>(a.dq + row * a.qs, dqa, a.scale * ifs);
                }
            }
        }
        __syncthreads();
        // ---- restage: pk a2 / pk dOs and lse2 / -delta*2^S rows for pass B
        if (active && p == 0) {
            store_pk<C>(rowb + (size_t)own * 2 * C, aq);
            store_pk<C>(rowb + (size_t)own * 2 * C + C, dO);
            f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)own * 2 * NH);
#pragma unroll
            for (int P = 0; P < NP; ++P) { rs[P] = lse2[P]; rs[NP + P] = ndl[P]; }
        }
        if (masked) {
            for (int e = tid; e < T; e += blockDim.x) {
                const int w2 = e / NPAD, t2 = e - w2 * NPAD;
                if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                    float4* z = reinterpret_cast<float4*>(rowb + (size_t)e * 2 * C);
#pragma unroll
                    for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                    f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)e * 2 * NH);
#pragma unroll
                    for (int P = 0; P < NP; ++P) { rs[P] = splat(INFINITY); rs[NP + P] = splat(0.f); }
                }
            }
        }
        __syncthreads();

        // ================= pass B: lane = key row -> dk, dv
        {
            const float* qdw = rowb + (size_t)wl_c * NPAD * 2 * C;
            const float* rsw = rs_s + (size_t)wl_c * NPAD * 2 * NH;
            f2 kr[C / 2], vr[C / 2], dka[C / 2], dva[C / 2];
            if (active) {
                if constexpr (KIND == 1) {
                    float kn[C], nrm[NH];
                    load_row<C>(kn, a.k + row * a.ks);
                    normalize_heads<C, HD>(kn, nrm);
                    pack_row<C>(kr, kn);
                } else {
                    load_pk<C>(kr, a.k + row * a.ks);
                }
                load_pk<C>(vr, a.v + row * a.vs);
            } else {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) { kr[i] = splat(0.f); vr[i] = splat(0.f); }
            }
#pragma unroll
            for (int i = 0; i < C / 2; ++i) { dka[i] = splat(0.f); dva[i] = splat(0.f); }
            const int cko = g.off - code;
            const int ib = p * nk;
            int2 mm = mw[ib];
            for (int n = 0; n < ((MMNI_ABL & 2) ? 0 : nk); ++n) {
                const int i = ib + n;
                const int2 mnext = mw[i + 1];
                f2 tb[NP], ai[C / 2], gi[C / 2];
                lds_tab<NP, NHP>(tb, tab_s, (mm.x & 0xffff) + cko);
                lds_row<C>(ai, qdw + (size_t)i * 2 * C);
                lds_row<C>(gi, qdw + (size_t)i * 2 * C + C);
                const f2* rsi = reinterpret_cast<const f2*>(rsw + (size_t)i * 2 * NH);
                f2 base[NP];
                if (masked) {
                    const float madd = ((mm.x >> 16) == rc ? 0.f : kMask2) + __int_as_float(mm.y);
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] + (splat(madd) - rsi[P]);
                } else {
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] - rsi[P];
                }
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 sc = pfma(ai[2 * P], kr[2 * P], base[P]);
                    sc = pfma(ai[2 * P + 1], kr[2 * P + 1], sc);
                    const f2 pr = exp2_2(sc);
                    f2 tt = pfma(gi[2 * P], vr[2 * P], rsi[NP + P]);
                    tt = pfma(gi[2 * P + 1], vr[2 * P + 1], tt);
                    const f2 dsv = pr * tt;
                    dva[2 * P] = pfma(pr, gi[2 * P], dva[2 * P]);
                    dva[2 * P + 1] = pfma(pr, gi[2 * P + 1], dva[2 * P + 1]);
                    dka[2 * P] = pfma(dsv, ai[2 * P], dka[2 * P]);
                    dka[2 * P + 1] = pfma(dsv, ai[2 * P + 1], dka[2 * P + 1]);
                }
                mm = mnext;
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) {
                    dka[i] += shfl2(dka[i], o);
                    dva[i] += shfl2(dva[i], o);
                }
            }
            if (active && p == 0) {
                store_nat<C>(a.dv + row * a.vs, dva, ifs);
                if constexpr (KIND == 1) {
                    float dkn[C], dk[C];
                    unpack_row<C>(dkn, dka);
                    float kraw[C], nrm[NH];
                    load_row<C>(kraw, a.k + row * a.ks);
                    normalize_heads<C, HD>(kraw, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dkn[h * HD + c] * (kLn2 * ifs);
                        normalize_bwd<HD>(dk + h * HD, dy, kraw + h * HD, nrm[h]);
                    }
                    store_row<C>(a.dk + row * a.ks, dk);
                } else {
                    store_nat<C>(a.dk + row * a.ks, dka, kLn2 * ifs);
                }
            }
        }
        __syncthreads();
    }

    if (KIND == 1) {
#pragma unroll
        for (int P = 0; P < NP; ++P) {
            f2 v = dtr[P];
            for (int o = 32; o > 0; o >>= 1) v += shfl2(v, o);
            if (lane == 0) {
                atomicAdd(&dtau_s[2 * P], v.x);
                atomicAdd(&dtau_s[2 * P + 1], v.y);
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        const dt_t v = dtab_s[(e / NH) * DS + e % NH];
        if (v != 0) atomicAdd(&a.dtab_fix[e], kDtab32 ? (unsigned long long)(long long)(int)v : (unsigned long long)v);
    }
    if (KIND == 1 && tid < NH) atomicAdd(&a.dtau[tid], dtau_s[tid] * ifs / (a.tau[tid] * kLog2e));
}

// ------------------------------------------------------------------------------------
// backward, two rows per lane
// ------------------------------------------------------------------------------------
// The passes of wattn_bwd_pk_kernel with every lane carrying two rows of its window (tokens r
// and r + N/2): pass A's K/V/metadata reads serve two queries and pass B's Q/dO/lse/delta reads
// serve two keys, so the LDS instructions per (query, key) pair drop from ~15 (A) / ~12 (B) to
// ~11.5 / ~7.  A window takes N/2 x KS(4) lanes: 448 threads at N = 216, one block per CU (the
// LDS holds the bias table and its 64-bit gradient), 7 waves with up to 256 VGPRs each.
// Kind 0 (scaled dot + table bias) only; WPB = 1.
template <int C, int MAXT>
__global__ __launch_bounds__(MAXT, C == 4 ? 4 : 1) void wattn_bwd_pk2_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2;
    constexpr int NHP = NH == 2 ? 2 : (NH + 3) & ~3;
    constexpr int DS = NH + kDtabPad;
    using dt_t = std::conditional_t<kDtab32, unsigned int, unsigned long long>;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, NHALF = N / 2;
    float* rowb = smem;                                   // [NPAD][2C]: pass A pk k | pk v; pass B pk a2 | pk dOs
    float* rs_s = smem + (size_t)NPAD * 2 * C;            // [NPAD][2NH]: pass B lse2 | -delta*2^S
    int2* meta_s = reinterpret_cast<int2*>(rs_s + (size_t)NPAD * 2 * NH);
    float* tab_s = reinterpret_cast<float*>(meta_s + NPAD);
    dt_t* dtab_s = reinterpret_cast<dt_t*>(tab_s + (size_t)g.Tsz * NHP);

    // head groups (a.hsplit > 1): block b serves heads [h0, h0 + NH) of the NHT = NH * hsplit
    // heads, for windows b / hsplit, b / hsplit + gridDim / hsplit, ...  Rows, lse and the table
    // are addressed with the full head count; coff offsets the channel columns.
    // The NHG blocks of a window sit 8 block indices apart: blocks are dealt round-robin over the
    // 8 XCDs, so they share one XCD's L2 (one HBM fetch of the window's rows, and their 16-B
    // column pieces of dq / dk / dv merge there).  The host makes the grid a multiple of 8 NHG.
    const int NHG = a.hsplit;
    const int xslot = blockIdx.x >> 3;
    const int hg = NHG > 1 ? (MMNI_HS_XCD ? xslot % NHG : blockIdx.x % NHG) : 0;
    const int wfirst = NHG > 1 ? (MMNI_HS_XCD ? (xslot / NHG) * 8 + (blockIdx.x & 7) : blockIdx.x / NHG) : blockIdx.x;
    const int h0 = hg * NH, NHT = NH * NHG;
    const int coff = h0 * HD;
    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const bool lane_ok = r < NHALF;
    const int rr0 = lane_ok ? r : 0;

    for (int e = tid; e < g.Tsz * NHP; e += blockDim.x) {
        const int row = e / NHP, h = e - row * NHP;
        tab_s[tab_pos<NHP>(row, h)] = h < NH ? a.table[row * NHT + h0 + h] * kLog2e : 0.f;
    }
    for (int e = tid; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0;
    const int fexp = fix_exponent(a.maxbits, HD) - a.fix_shift;
    const float fs = exp2f((float)fexp);
    const float ifs = exp2f((float)-fexp);
    const int nk = NPAD / KS;
    const f2 qscale = splat(a.scale * kLog2e);

    for (int grp = wfirst; grp < a.ngroups; grp += gridDim.x / NHG) {
        const int w = grp;
        // rr opaque per window (MMNI_PK2_OPAQUE): addresses derived from it are not hoisted out
        // of the window loop, where they would stay live across both passes
        int rr = rr0;
        if (MMNI_PK2_OPAQUE) asm volatile("" : "+v"(rr));
        const bool active = lane_ok && (w < g.nwin);
        const bool masked = group_masked(g, grp, 1, NPAD);
        f2 aq[2][C / 2], dO[2][C / 2], lse2[2][NP], ndl[2][NP];
        int64_t row[2] = {0, 0};
        int code[2] = {0, 0}, rc[2] = {0, 0};
        if (active) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const TokenInfo ti = token_info(g, w, rr + u * NHALF);
                row[u] = ti.row;
                code[u] = ti.code;
                rc[u] = ti.rc;
            }
        }
        // K/V staging split over the row pair's KS = 4 lanes: lane p moves float4 chunks p, p + 4,
        // p + 8 of [K row 0 | V row 0 | K row 1 | V row 1] (3 chunks each), loaded in the same
        // round as the Q/dO/O rows below.  A chunk keeps its offset in the pk row layout, with its
        // components reordered (x, z, y, w) as store_pk does.
        constexpr int KVCH = 4 * (C / 4);       // float4 chunks of the two K and V rows
        constexpr int KVPL = (KVCH + 3) / 4;    // per lane
        float4 kvc[KVPL];
        if (active) {
#pragma unroll
            for (int m = 0; m < KVPL; ++m) {
                const int c = p + 4 * m, u = c / (2 * (C / 4)), cc = c - u * 2 * (C / 4);
                const bool isv = cc >= C / 4;
                const float* src = (isv ? a.v + row[u] * a.vs : a.k + row[u] * a.ks) + coff;
                kvc[m] = c < KVCH ? *reinterpret_cast<const float4*>(src + 4 * (cc - (isv ? C / 4 : 0)))
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (active) {
                const int64_t rw = row[u];
                load_pk<C>(aq[u], a.q + rw * a.qs + coff);
                f2 orow[C / 2];
                load_pk<C>(dO[u], a.dout + rw * a.os + coff);
                load_pk<C>(orow, a.o + rw * a.os + coff);
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    aq[u][2 * P] *= qscale;
                    aq[u][2 * P + 1] *= qscale;
                    const f2 dd = pfma(orow[2 * P], dO[u][2 * P], orow[2 * P + 1] * dO[u][2 * P + 1]);
                    ndl[u][P] = dd * splat(-fs);
                    dO[u][2 * P] *= splat(fs);
                    dO[u][2 * P + 1] *= splat(fs);
                    lse2[u][P] = (f2){a.lse[rw * NHT + h0 + 2 * P], a.lse[rw * NHT + h0 + 2 * P + 1]} * kLog2e;
                }
            } else {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) { aq[u][i] = splat(0.f); dO[u][i] = splat(0.f); }
#pragma unroll
                for (int P = 0; P < NP; ++P) { lse2[u][P] = splat(INFINITY); ndl[u][P] = splat(0.f); }
            }
        }
        // ---- stage K/V + metadata (pad rows get neutral values)
        if (active) {
#pragma unroll
            for (int m = 0; m < KVPL; ++m) {
                const int c = p + 4 * m, u = c / (2 * (C / 4)), cc = c - u * 2 * (C / 4);
                if (c < KVCH) {
                    const float4 t = kvc[m];
                    *reinterpret_cast<float4*>(rowb + (size_t)(rr + u * NHALF) * 2 * C + 4 * cc) =
                        make_float4(t.x, t.z, t.y, t.w);
                }
            }
            if (p == 0) {
#pragma unroll
                for (int u = 0; u < 2; ++u) meta_s[rr + u * NHALF] = make_int2(code[u] | (rc[u] << 16), 0);
            }
        }
        if (masked) {
            for (int e = tid; e < NPAD; e += blockDim.x) {
                if (e >= N || w >= g.nwin) {
                    float4* z = reinterpret_cast<float4*>(rowb + (size_t)e * 2 * C);
#pragma unroll
                    for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                    meta_s[e] = make_int2(0x7fff0000, __float_as_int(-INFINITY));
                }
            }
        }
        __syncthreads();

        f2 kr[2][C / 2], vr[2][C / 2];   // pass B's own K/V rows, read from the pass A staging
        // ================= pass A: queries rr, rr + N/2 -> dq, dtable
        {
            f2 dqa[2][C / 2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int i = 0; i < C / 2; ++i) dqa[u][i] = splat(0.f);
            const int cq0 = code[0] + g.off, cq1 = code[1] + g.off;
            // one (query u, key) pair: probability, dS (scaled by 2^S) and the dq update
            auto pair = [&](int u, const f2 (&tb)[NP], const f2 (&kj)[C / 2], const f2 (&vj)[C / 2], int2 mk,
                            f2 (&dsv)[NP]) {
                f2 base[NP];
                if (masked) {
                    const float madd = ((mk.x >> 16) == rc[u] ? 0.f : kMask2) + __int_as_float(mk.y);
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] + (splat(madd) - lse2[u][P]);
                } else {
#pragma unroll
                    for (int P = 0; P < NP; ++P) base[P] = tb[P] - lse2[u][P];
                }
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 sc = pfma(aq[u][2 * P], kj[2 * P], base[P]);
                    sc = pfma(aq[u][2 * P + 1], kj[2 * P + 1], sc);
                    const f2 pr = exp2_2(sc);
                    f2 tt = pfma(dO[u][2 * P], vj[2 * P], ndl[u][P]);
                    tt = pfma(dO[u][2 * P + 1], vj[2 * P + 1], tt);
                    dsv[P] = pr * tt;
                    dqa[u][2 * P] = pfma(dsv[P], kj[2 * P], dqa[u][2 * P]);
                    dqa[u][2 * P + 1] = pfma(dsv[P], kj[2 * P + 1], dqa[u][2 * P + 1]);
                }
            };
            auto scatter = [&](int tix, const f2 (&dsv)[NP]) {
                if (MMNI_ABL & 1) return;
                dt_t* dtp = dtab_s + tix * DS;
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    atomicAdd(&dtp[2 * P], (dt_t)fix_round(dsv[P].x));
                    atomicAdd(&dtp[2 * P + 1], (dt_t)fix_round(dsv[P].y));
                }
            };
            // Paired keys: when the window's second half is a whole number of planes later than
            // its first (N/2 a multiple of wh*ww: code(t + N/2) = code(t) + const), query rr + N/2
            // and key j + N/2 have the same relative offset as query rr and key j.  The lane takes
            // keys j and j + N/2 together: 4 pairs on 3 table rows, the shared row's two dS summed
            // before one set of atomics (|sum| < 2^31, see fix_exponent): 18 atomics and 3 table
            // reads per 4 pairs instead of 24 and 4.
            const bool paired = MMNI_PK2_PAIRK && NPAD == N && NHALF % (g.wh * g.ww) == 0 && NHALF % KS == 0;
            if (paired) {
                const int nk2 = NHALF / KS, jb = p * nk2;
                for (int n = 0; n < ((MMNI_ABL & 4) ? 0 : nk2); ++n) {
                    const int j0 = jb + n, j1 = j0 + NHALF;
                    const int2 m0 = meta_s[j0], m1 = meta_s[j1];
                    const int tA = cq0 - (m0.x & 0xffff);   // (rr, j0) and (rr + N/2, j1)
                    const int tC = cq1 - (m0.x & 0xffff);   // (rr + N/2, j0)
                    const int tB = cq0 - (m1.x & 0xffff);   // (rr, j1)
                    f2 kj[C / 2], vj[C / 2], tbA[NP], tb2[NP], dsA[NP], ds[NP];
                    lds_row<C>(kj, rowb + (size_t)j0 * 2 * C);
                    lds_row<C>(vj, rowb + (size_t)j0 * 2 * C + C);
                    lds_tab<NP, NHP>(tbA, tab_s, tA);
                    lds_tab<NP, NHP>(tb2, tab_s, tC);
                    pair(0, tbA, kj, vj, m0, dsA);
                    pair(1, tb2, kj, vj, m0, ds);
                    scatter(tC, ds);
                    __builtin_amdgcn_sched_barrier(0);   // keep key j1's reads behind key j0's work
                    lds_row<C>(kj, rowb + (size_t)j1 * 2 * C);
                    lds_row<C>(vj, rowb + (size_t)j1 * 2 * C + C);
                    lds_tab<NP, NHP>(tb2, tab_s, tB);
                    pair(0, tb2, kj, vj, m1, ds);
                    scatter(tB, ds);
                    pair(1, tbA, kj, vj, m1, ds);
#pragma unroll
                    for (int P = 0; P < NP; ++P) ds[P] += dsA[P];
                    scatter(tA, ds);
                }
            } else {
                const int jb = p * nk;
                for (int n = 0; n < ((MMNI_ABL & 4) ? 0 : nk); ++n) {
                    const int j = jb + n;
                    const int2 mk = meta_s[j];
                    f2 kj[C / 2], vj[C / 2], tb[NP], ds[NP];
                    lds_row<C>(kj, rowb + (size_t)j * 2 * C);
                    lds_row<C>(vj, rowb + (size_t)j * 2 * C + C);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int tix = (u ? cq1 : cq0) - (mk.x & 0xffff);
                        lds_tab<NP, NHP>(tb, tab_s, tix);
                        pair(u, tb, kj, vj, mk, ds);
                        scatter(tix, ds);
                    }
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int i = 0; i < C / 2; ++i) dqa[u][i] += shfl2(dqa[u][i], o);
            }
            if (active && p == 0) {
#pragma unroll
                for (int u = 0; u < 2; ++u) store_nat<C>(a.dq + row[u] * a.qs + coff, dqa[u], a.scale * ifs);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (active && MMNI_PK2_KVLDS) {
                    lds_row<C>(kr[u], rowb + (size_t)(rr + u * NHALF) * 2 * C);
                    lds_row<C>(vr[u], rowb + (size_t)(rr + u * NHALF) * 2 * C + C);
                } else if (active) {
                    load_pk<C>(kr[u], a.k + row[u] * a.ks + coff);
                    load_pk<C>(vr[u], a.v + row[u] * a.vs + coff);
                } else {
#pragma unroll
                    for (int i = 0; i < C / 2; ++i) { kr[u][i] = splat(0.f); vr[u][i] = splat(0.f); }
                }
            }
        }
        __syncthreads();
        // ---- restage: pk a2 / pk dOs and lse2 / -delta*2^S rows for pass B
        if (active && p == 0) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int t = rr + u * NHALF;
                store_pk<C>(rowb + (size_t)t * 2 * C, aq[u]);
                store_pk<C>(rowb + (size_t)t * 2 * C + C, dO[u]);
                f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)t * 2 * NH);
#pragma unroll
                for (int P = 0; P < NP; ++P) { rs[P] = lse2[u][P]; rs[NP + P] = ndl[u][P]; }
            }
        }
        if (masked) {
            for (int e = tid; e < NPAD; e += blockDim.x) {
                if (e >= N || w >= g.nwin) {
                    float4* z = reinterpret_cast<float4*>(rowb + (size_t)e * 2 * C);
#pragma unroll
                    for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                    f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)e * 2 * NH);
#pragma unroll
                    for (int P = 0; P < NP; ++P) { rs[P] = splat(INFINITY); rs[NP + P] = splat(0.f); }
                }
            }
        }
        __syncthreads();

        // ================= pass B: keys rr, rr + N/2 -> dk, dv
        {
            f2 dka[2][C / 2], dva[2][C / 2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int i = 0; i < C / 2; ++i) { dka[u][i] = splat(0.f); dva[u][i] = splat(0.f); }
            const int ck0 = g.off - code[0], ck1 = g.off - code[1];
            // one query row i against the lane's two keys, with their table rows
            auto qrow = [&](int i, int2 mcur, const f2 (&tb0)[NP], const f2 (&tb1)[NP]) {
                const int ri = mcur.x >> 16;
                f2 ai[C / 2], gi[C / 2];
                lds_row<C>(ai, rowb + (size_t)i * 2 * C);
                lds_row<C>(gi, rowb + (size_t)i * 2 * C + C);
                f2 rsi[2 * NP];
                {
                    const float4* rq = reinterpret_cast<const float4*>(rs_s + (size_t)i * 2 * NH);
#pragma unroll
                    for (int c = 0; c < NP; ++c) {
                        const float4 x = rq[c];
                        rsi[2 * c] = (f2){x.x, x.y};
                        rsi[2 * c + 1] = (f2){x.z, x.w};
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f2(&tb)[NP] = u ? tb1 : tb0;
                    f2 base[NP];
                    if (masked) {
                        const float madd = (ri == rc[u] ? 0.f : kMask2) + __int_as_float(mcur.y);
#pragma unroll
                        for (int P = 0; P < NP; ++P) base[P] = tb[P] + (splat(madd) - rsi[P]);
                    } else {
#pragma unroll
                        for (int P = 0; P < NP; ++P) base[P] = tb[P] - rsi[P];
                    }
#pragma unroll
                    for (int P = 0; P < NP; ++P) {
                        f2 sc = pfma(ai[2 * P], kr[u][2 * P], base[P]);
                        sc = pfma(ai[2 * P + 1], kr[u][2 * P + 1], sc);
                        const f2 pr = exp2_2(sc);
                        f2 tt = pfma(gi[2 * P], vr[u][2 * P], rsi[NP + P]);
                        tt = pfma(gi[2 * P + 1], vr[u][2 * P + 1], tt);
                        const f2 dsv = pr * tt;
                        dva[u][2 * P] = pfma(pr, gi[2 * P], dva[u][2 * P]);
                        dva[u][2 * P + 1] = pfma(pr, gi[2 * P + 1], dva[u][2 * P + 1]);
                        dka[u][2 * P] = pfma(dsv, ai[2 * P], dka[u][2 * P]);
                        dka[u][2 * P + 1] = pfma(dsv, ai[2 * P + 1], dka[u][2 * P + 1]);
                    }
                }
            };
            // Paired queries (as pass A's paired keys): query i + N/2 against key rr + N/2 has the
            // table row of query i against key rr, so queries i and i + N/2 together take 3 table
            // reads for their 4 pairs instead of 4.
            const bool pairedB = MMNI_PK2_PAIRQ && NPAD == N && NHALF % (g.wh * g.ww) == 0 && NHALF % KS == 0;
            if (pairedB) {
                const int nk2 = NHALF / KS, ib2 = p * nk2;
                for (int n = 0; n < ((MMNI_ABL & 2) ? 0 : nk2); ++n) {
                    const int i0 = ib2 + n, i1 = i0 + NHALF;
                    const int2 m0 = meta_s[i0], m1 = meta_s[i1];
                    const int c0 = m0.x & 0xffff;
                    f2 tA[NP], tB[NP], tC[NP];
                    lds_tab<NP, NHP>(tA, tab_s, c0 + ck0);                 // (i0, rr), (i1, rr + N/2)
                    lds_tab<NP, NHP>(tB, tab_s, c0 + ck1);                 // (i0, rr + N/2)
                    lds_tab<NP, NHP>(tC, tab_s, (m1.x & 0xffff) + ck0);    // (i1, rr)
                    qrow(i0, m0, tA, tB);
                    qrow(i1, m1, tC, tA);
                }
            } else {
                const int ib = p * nk;
                for (int n = 0; n < ((MMNI_ABL & 2) ? 0 : nk); ++n) {
                    const int i = ib + n;
                    const int2 mcur = meta_s[i];
                    const int ci = mcur.x & 0xffff;
                    f2 tb0[NP], tb1[NP];
                    lds_tab<NP, NHP>(tb0, tab_s, ci + ck0);
                    lds_tab<NP, NHP>(tb1, tab_s, ci + ck1);
                    qrow(i, mcur, tb0, tb1);
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int i = 0; i < C / 2; ++i) {
                        dka[u][i] += shfl2(dka[u][i], o);
                        dva[u][i] += shfl2(dva[u][i], o);
                    }
            }
            if (active && p == 0) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    store_nat<C>(a.dv + row[u] * a.vs + coff, dva[u], ifs);
                    store_nat<C>(a.dk + row[u] * a.ks + coff, dka[u], kLn2 * ifs);
                }
            }
        }
        __syncthreads();
    }
    __syncthreads();
    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        const dt_t v = dtab_s[(e / NH) * DS + e % NH];
        if (v != 0)
            atomicAdd(&a.dtab_fix[(e / NH) * NHT + h0 + e % NH],
                      kDtab32 ? (unsigned long long)(long long)(int)v : (unsigned long long)v);
    }
}

// ------------------------------------------------------------------------------------
// backward, four rows per lane
// ------------------------------------------------------------------------------------
// wattn_bwd_pk2_kernel with each lane carrying a quad of its window: tokens t, t + D1, t + D2 and
// t + D1 + D2, where D1 moves by half the window's planes and D2 by half its rows (wd, wh even).
// The relative code is linear in (i, j, k), so member m = a + 2c of a query quad and member
// n = a' + 2c' of a key quad read table row  base + (a - a') d1 + (c - c') d2 :  16 pairs touch
// 9 rows.  Pass A (lane = query quad) reads one key quad (4 K/V rows) and 9 table rows per 16
// pairs and issues 9 table-gradient atomics per head (two-row kernel: 8 K/V rows, 12 table rows,
// 12 atomics); pass B (lane = key quad) reads 4 query rows and 9 table rows per 16 pairs (8 and
// 16).  N/4 quads x KS = 8 key slices: 432 threads at 6^3.  Kind 0, C = 4 (one head pair per
// block, head groups as in wattn_bwd_pk2_kernel), one window per block.
#ifndef MMNI_PK4_WAVES
#define MMNI_PK4_WAVES 4
#endif
#ifndef MMNI_PK4_TB9
#define MMNI_PK4_TB9 1   // pass B holds the 9 table rows of a quad pair (0: 4 reads per query row)
#endif
#ifndef MMNI_PK4_OPAQUE
#define MMNI_PK4_OPAQUE 1
#endif
#ifndef MMNI_PK4_SCHED
#define MMNI_PK4_SCHED 1
#endif
template <int C, int MAXT>
__global__ __launch_bounds__(MAXT, MMNI_PK4_WAVES) void wattn_bwd_pk4_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2;
    constexpr int NHP = NH == 2 ? 2 : (NH + 3) & ~3;
    constexpr int DS = NH + kDtabPad;
    using dt_t = unsigned long long;
    static_assert(C == 4 && NP == 1, "one head pair per block: a K, V, Q or dO row is one float4");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, KS = a.KS, NQ = N / 4;
    float* kv_s = smem;                                   // [N][2C]: pk k | pk v
    float* qg_s = smem + (size_t)N * 2 * C;               // [N][2C]: pk q*scale | pk dO*2^S
    float* rs_s = smem + (size_t)N * 4 * C;               // [N][2NH]: lse2 | -delta*2^S
    int2* meta_s = reinterpret_cast<int2*>(rs_s + (size_t)N * 2 * NH);
    float* tab_s = reinterpret_cast<float*>(meta_s + N);
    dt_t* dtab_s = reinterpret_cast<dt_t*>(tab_s + (size_t)g.Tsz * NHP);

    const int NHG = a.hsplit;
    const int xslot = blockIdx.x >> 3;
    const int hg = NHG > 1 ? xslot % NHG : 0;
    const int wfirst = NHG > 1 ? (xslot / NHG) * 8 + (blockIdx.x & 7) : blockIdx.x;
    const int h0 = hg * NH, NHT = NH * NHG;
    const int coff = h0 * HD;
    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const bool lane_ok = r < NQ;
    const int rr = lane_ok ? r : 0;
    // quad geometry (window-independent): base b -> token, member shifts in tokens and in codes
    const int hw2 = (g.wh >> 1) * g.ww, pl = g.wh * g.ww;
    const int D1 = (g.wd >> 1) * pl, D2 = hw2;
    const int d1 = (g.wd >> 1) * g.tw, d2 = (g.wh >> 1) * g.th;
    auto quad_tok = [&](int b) {
        const int z = b / hw2;
        return z * pl + (b - z * hw2);
    };
    auto member = [&](int t, int m) { return t + (m & 1) * D1 + (m >> 1) * D2; };
    auto tab_row = [&](int t0, int ti) { return t0 + (ti / 3 - 1) * d1 + (ti % 3 - 1) * d2; };

    for (int e = tid; e < g.Tsz * NHP; e += blockDim.x) {
        const int row = e / NHP, h = e - row * NHP;
        tab_s[tab_pos<NHP>(row, h)] = h < NH ? a.table[row * NHT + h0 + h] * kLog2e : 0.f;
    }
    for (int e = tid; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0;
    const int fexp = fix_exponent(a.maxbits, HD) - a.fix_shift;
    const float fs = exp2f((float)fexp);
    const float ifs = exp2f((float)-fexp);
    const float qsc = a.scale * kLog2e;
    const int t0i = quad_tok(rr);
    const int nb = (NQ - p + KS - 1) / KS;   // bases p, p + KS, ... < NQ of this lane's slice

    for (int w = wfirst; w < a.ngroups; w += gridDim.x / NHG) {
        // t0 is opaque per window: keeps the compiler from hoisting every LDS / row address
        // derived from it out of the window loop (they would stay live across both passes)
        int t0 = t0i;
        if (MMNI_PK4_OPAQUE) asm volatile("" : "+v"(t0));
        // the member this lane stages (p >> 1) and stores (p < 4: member p)
        const int ts = member(t0, p >> 1), tw = member(t0, p & 3);
        const bool masked = group_masked(g, w, 1, N);
        int cq0, rcq[4];
        {
            const TokenInfo ti = token_info(g, w, t0);
            cq0 = ti.code + g.off;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) rcq[u] = masked ? token_info(g, w, member(t0, u)).rc : 0;
        // ---- staging: lane p of a quad moves member p / 2's rows; even lanes K, V and Q,
        //      odd lanes dO, O and lse (-> dO*2^S, -delta*2^S, lse2)
        if (lane_ok) {
            const TokenInfo ti = token_info(g, w, ts);
            const int64_t rw = ti.row;
            if ((p & 1) == 0) {
                const float4 kk = *reinterpret_cast<const float4*>(a.k + rw * a.ks + coff);
                const float4 vv = *reinterpret_cast<const float4*>(a.v + rw * a.vs + coff);
                const float4 qq = *reinterpret_cast<const float4*>(a.q + rw * a.qs + coff);
                *reinterpret_cast<float4*>(kv_s + (size_t)ts * 2 * C) = make_float4(kk.x, kk.z, kk.y, kk.w);
                *reinterpret_cast<float4*>(kv_s + (size_t)ts * 2 * C + C) = make_float4(vv.x, vv.z, vv.y, vv.w);
                *reinterpret_cast<float4*>(qg_s + (size_t)ts * 2 * C) =
                    make_float4(qq.x * qsc, qq.z * qsc, qq.y * qsc, qq.w * qsc);
                meta_s[ts] = make_int2(ti.code | (ti.rc << 16), 0);
            } else {
                const float4 gg = *reinterpret_cast<const float4*>(a.dout + rw * a.os + coff);
                const float4 oo = *reinterpret_cast<const float4*>(a.o + rw * a.os + coff);
                const float2 ls = *reinterpret_cast<const float2*>(a.lse + rw * NHT + h0);
                *reinterpret_cast<float4*>(qg_s + (size_t)ts * 2 * C + C) =
                    make_float4(gg.x * fs, gg.z * fs, gg.y * fs, gg.w * fs);
                // natural row (h0 c0, h0 c1, h1 c0, h1 c1): delta per head
                const float dl0 = fmaf(oo.x, gg.x, oo.y * gg.y), dl1 = fmaf(oo.z, gg.z, oo.w * gg.w);
                *reinterpret_cast<float4*>(rs_s + (size_t)ts * 2 * NH) =
                    make_float4(ls.x * kLog2e, ls.y * kLog2e, -dl0 * fs, -dl1 * fs);
            }
        }
        __syncthreads();

        // ================= pass A: query quad -> dq, dtable
        {
            f2 aq[4][C / 2], dO[4][C / 2], lse2[4], ndl[4], dqa[4][C / 2];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = member(t0, u);
                lds_row<C>(aq[u], qg_s + (size_t)t * 2 * C);
                lds_row<C>(dO[u], qg_s + (size_t)t * 2 * C + C);
                const float4 x = *reinterpret_cast<const float4*>(rs_s + (size_t)t * 2 * NH);
                lse2[u] = (f2){x.x, x.y};
                ndl[u] = (f2){x.z, x.w};
#pragma unroll
                for (int i = 0; i < C / 2; ++i) dqa[u][i] = splat(0.f);
            }
#pragma unroll 1
            for (int n = 0; n < ((MMNI_ABL & 4) ? 0 : nb); ++n) {
                const int k0 = quad_tok(p + KS * n);
                int2 mk[4];
                mk[0] = meta_s[k0];
                if (masked) {
#pragma unroll
                    for (int m = 1; m < 4; ++m) mk[m] = meta_s[member(k0, m)];
                } else {
                    mk[1] = mk[2] = mk[3] = mk[0];
                }
                const int tix0 = cq0 - (mk[0].x & 0xffff);
                f2 tb[9], acc[10];
#pragma unroll
                for (int ti = 0; ti < 9; ++ti) {
                    lds_tab<1, NHP>(*reinterpret_cast<f2(*)[1]>(&tb[ti]), tab_s, tab_row(tix0, ti));
                    acc[ti] = splat(0.f);
                }
                acc[9] = splat(0.f);
#pragma unroll
                for (int kn = 0; kn < 4; ++kn) {
                    if (MMNI_PK4_SCHED) __builtin_amdgcn_sched_barrier(0);   // one key row in flight
                    const int kt = member(k0, kn);
                    f2 kj[C / 2], vj[C / 2];
                    lds_row<C>(kj, kv_s + (size_t)kt * 2 * C);
                    lds_row<C>(vj, kv_s + (size_t)kt * 2 * C + C);
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const int ti = ((m & 1) - (kn & 1) + 1) * 3 + ((m >> 1) - (kn >> 1) + 1);
                        const int ai = (ti == 4 && m >= 2) ? 9 : ti;
                        f2 base = tb[ti] - lse2[m];
                        if (masked) base += splat(((mk[kn].x >> 16) == rcq[m] ? 0.f : kMask2) + __int_as_float(mk[kn].y));
                        f2 sc = pfma(aq[m][0], kj[0], base);
                        sc = pfma(aq[m][1], kj[1], sc);
                        const f2 pr = exp2_2(sc);
                        f2 tt = pfma(dO[m][0], vj[0], ndl[m]);
                        tt = pfma(dO[m][1], vj[1], tt);
                        const f2 dsv = pr * tt;
                        acc[ai] += dsv;
                        dqa[m][0] = pfma(dsv, kj[0], dqa[m][0]);
                        dqa[m][1] = pfma(dsv, kj[1], dqa[m][1]);
                    }
                }
                // each accumulator holds at most two contributions (|sum| < 2^31 after scaling);
                // the centre row's four are rounded as two sums and added in 64 bits
                if (!(MMNI_ABL & 1) && lane_ok) {
#pragma unroll
                    for (int ti = 0; ti < 9; ++ti) {
                        dt_t* dtp = dtab_s + tab_row(tix0, ti) * DS;
                        long long vx = fix_round(acc[ti].x), vy = fix_round(acc[ti].y);
                        if (ti == 4) { vx += fix_round(acc[9].x); vy += fix_round(acc[9].y); }
                        atomicAdd(&dtp[0], (dt_t)vx);
                        atomicAdd(&dtp[1], (dt_t)vy);
                    }
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int i = 0; i < C / 2; ++i) dqa[u][i] += shfl2(dqa[u][i], o);
            }
            // every slice lane holds the sums: lane p < 4 stores member p
            if (lane_ok && p < 4) {
                f2 d[C / 2] = {dqa[0][0], dqa[0][1]};
#pragma unroll
                for (int u = 1; u < 4; ++u)
                    if (p == u) { d[0] = dqa[u][0]; d[1] = dqa[u][1]; }
                store_nat<C>(a.dq + token_info(g, w, tw).row * a.qs + coff, d, a.scale * ifs);
            }
        }

        // ================= pass B: key quad -> dk, dv (rows staged above; no restage)
        {
            f2 kr[4][C / 2], vr[4][C / 2], dka[4][C / 2], dva[4][C / 2];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = member(t0, u);
                lds_row<C>(kr[u], kv_s + (size_t)t * 2 * C);
                lds_row<C>(vr[u], kv_s + (size_t)t * 2 * C + C);
#pragma unroll
                for (int i = 0; i < C / 2; ++i) { dka[u][i] = splat(0.f); dva[u][i] = splat(0.f); }
            }
            const int ckoff = 2 * g.off - cq0;   // off - code(own member 0)
#pragma unroll 1
            for (int n = 0; n < ((MMNI_ABL & 2) ? 0 : nb); ++n) {
                const int q0 = quad_tok(p + KS * n);
                int2 mq[4];
                mq[0] = meta_s[q0];
                if (masked) {
#pragma unroll
                    for (int m = 1; m < 4; ++m) mq[m] = meta_s[member(q0, m)];
                } else {
                    mq[1] = mq[2] = mq[3] = mq[0];
                }
                const int tix0 = (mq[0].x & 0xffff) + ckoff;
                f2 tb[9];
                if (MMNI_PK4_TB9) {
#pragma unroll
                    for (int ti = 0; ti < 9; ++ti)
                        lds_tab<1, NHP>(*reinterpret_cast<f2(*)[1]>(&tb[ti]), tab_s, tab_row(tix0, ti));
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    if (MMNI_PK4_SCHED) __builtin_amdgcn_sched_barrier(0);   // one query row in flight
                    const int qt = member(q0, m);
                    f2 ai[C / 2], gi[C / 2];
                    lds_row<C>(ai, qg_s + (size_t)qt * 2 * C);
                    lds_row<C>(gi, qg_s + (size_t)qt * 2 * C + C);
                    const float4 x = *reinterpret_cast<const float4*>(rs_s + (size_t)qt * 2 * NH);
                    const f2 ls = (f2){x.x, x.y}, nd = (f2){x.z, x.w};
                    if (!MMNI_PK4_TB9) {
#pragma unroll
                        for (int kn = 0; kn < 4; ++kn) {
                            const int ti = ((m & 1) - (kn & 1) + 1) * 3 + ((m >> 1) - (kn >> 1) + 1);
                            lds_tab<1, NHP>(*reinterpret_cast<f2(*)[1]>(&tb[ti]), tab_s, tab_row(tix0, ti));
                        }
                    }
#pragma unroll
                    for (int kn = 0; kn < 4; ++kn) {
                        const int ti = ((m & 1) - (kn & 1) + 1) * 3 + ((m >> 1) - (kn >> 1) + 1);
                        f2 base = tb[ti] - ls;
                        if (masked) base += splat(((mq[m].x >> 16) == rcq[kn] ? 0.f : kMask2) + __int_as_float(mq[m].y));
                        f2 sc = pfma(ai[0], kr[kn][0], base);
                        sc = pfma(ai[1], kr[kn][1], sc);
                        const f2 pr = exp2_2(sc);
                        f2 tt = pfma(gi[0], vr[kn][0], nd);
                        tt = pfma(gi[1], vr[kn][1], tt);
                        const f2 dsv = pr * tt;
                        dva[kn][0] = pfma(pr, gi[0], dva[kn][0]);
                        dva[kn][1] = pfma(pr, gi[1], dva[kn][1]);
                        dka[kn][0] = pfma(dsv, ai[0], dka[kn][0]);
                        dka[kn][1] = pfma(dsv, ai[1], dka[kn][1]);
                    }
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int i = 0; i < C / 2; ++i) {
                        dka[u][i] += shfl2(dka[u][i], o);
                        dva[u][i] += shfl2(dva[u][i], o);
                    }
            }
            if (lane_ok && p < 4) {
                f2 dk[C / 2] = {dka[0][0], dka[0][1]}, dv[C / 2] = {dva[0][0], dva[0][1]};
#pragma unroll
                for (int u = 1; u < 4; ++u)
                    if (p == u) { dk[0] = dka[u][0]; dk[1] = dka[u][1]; dv[0] = dva[u][0]; dv[1] = dva[u][1]; }
                const int64_t rw = token_info(g, w, tw).row;
                store_nat<C>(a.dv + rw * a.vs + coff, dv, ifs);
                store_nat<C>(a.dk + rw * a.ks + coff, dk, kLn2 * ifs);
            }
        }
        __syncthreads();
    }
    __syncthreads();
    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        const dt_t v = dtab_s[(e / NH) * DS + e % NH];
        if (v != 0) atomicAdd(&a.dtab_fix[(e / NH) * NHT + h0 + e % NH], v);
    }
}

template <int C, int MAXT>
static void* pk_fwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_fwd_pk_kernel<C, 1, MAXT>)
                : reinterpret_cast<void*>(&wattn_fwd_pk_kernel<C, 0, MAXT>);
}
template <int C, int MAXT>
static void* pk_bwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_bwd_pk_kernel<C, 1, MAXT>)
                : reinterpret_cast<void*>(&wattn_bwd_pk_kernel<C, 0, MAXT>);
}

template <int C, int MAXT, int QPL = 2>
static void* pk2_fwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_fwd_pk2_kernel<C, 1, MAXT, QPL>)
                : reinterpret_cast<void*>(&wattn_fwd_pk2_kernel<C, 0, MAXT, QPL>);
}

// Forward blocks of <= 512 threads (KS = 2 at N = 216): two blocks share a CU, so one block's
// K/V gather overlaps the other's compute.  The backward's LDS (bias table + its 64-bit
// gradient) allows one block per CU; it keeps 1024 threads (KS = 4) for occupancy.
// qpl_f / qpl_b: rows per lane of the forward / backward (2: the pk2 kernels, windows of even N;
// the two-row backward needs one window per block, N > 128).
int wattn_pk_kernels(int C, int kind, int N, bool quad, void*& kf, void*& kb, int& maxt_f, int& maxt_b, int& qpl_f,
                     int& qpl_b, int& hs_b, int& hs_f) {
    const bool two = MMNI_FWD_QPL >= 2 && N % 2 == 0 && N >= 64;
    // four queries per lane: head-pair blocks only (the C = 12 state of four rows does not fit)
    const bool four = MMNI_FWD_QPL == 4 && MMNI_FWD_HSPLIT == 3 && N % 4 == 0 && N >= 64;
    const bool two_b = MMNI_BWD_QPL >= 2 && kind == 0 && N % 2 == 0 && N > 128;
    const bool four_b = two_b && MMNI_BWD_QPL == 4 && MMNI_BWD_HSPLIT == 3 && quad;
    qpl_f = two ? 2 : 1;
    qpl_b = 1;
    hs_b = 1;
    hs_f = 1;
    if (C == 12) {
        // MMNI_FWD_HSPLIT 3: the two-query forward per (window group, head pair)
        kf = four ? pk2_fwd<4, 512, 4>(kind)
                  : two ? (MMNI_FWD_HSPLIT == 3 ? pk2_fwd<4, 512>(kind) : pk2_fwd<12, 512>(kind)) : pk_fwd<12, 512>(kind);
        if (two) hs_f = MMNI_FWD_HSPLIT == 3 ? 3 : 1;
        if (four) qpl_f = 4;
        maxt_f = 512;
        if (four_b) {
            // four rows per lane, one block per (window, head pair)
            kb = reinterpret_cast<void*>(&wattn_bwd_pk4_kernel<4, 512>);
            hs_b = 3;
            maxt_b = 512;
            qpl_b = 4;
        } else if (two_b) {
            // MMNI_BWD_HSPLIT 3: one block per (window, head pair), 4 channels each
            kb = MMNI_BWD_HSPLIT == 3 ? reinterpret_cast<void*>(&wattn_bwd_pk2_kernel<4, 512>)
                                      : reinterpret_cast<void*>(&wattn_bwd_pk2_kernel<12, 512>);
            hs_b = MMNI_BWD_HSPLIT == 3 ? 3 : 1;
            maxt_b = 512;
            qpl_b = 2;
        } else {
            kb = pk_bwd<12, 1024>(kind);
            maxt_b = 1024;
        }
        return 1;
    }
    if (C == 24) { kf = pk_fwd<24, 512>(kind); kb = pk_bwd<24, 512>(kind); maxt_f = 512; maxt_b = 512; qpl_f = 1; return 1; }
    return 0;
}

}  // namespace mmni
