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
    constexpr int HD = 2, NH = C / HD, NP = NH / 2, CK = kPk2Chunk;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB, NHALF = N / QPL;   // QPL queries per lane: t, t + N/QPL, ...
    float* kv_s = smem;                                              // [WPB*NPAD][2C] pk k | pk v
    int2* meta_s = reinterpret_cast<int2*>(kv_s + (size_t)WPB * NPAD * 2 * C);  // [WPB*NPAD]
    float* tab_s = reinterpret_cast<float*>(meta_s + WPB * NPAD);     // [Tsz][NH]

    // head groups (a.hsplit > 1; the host launches 1): the NHG blocks of a window group
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
    using dt_t = unsigned long long;
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
    float* dtau_s = reinterpret_cast<float*>(dtab_s + (size_t)g.Tsz * DS);   // [kMaxWaves][NH]

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
            for (int n = 0; n < nk; ++n) {
                const int j = jb + n;
                const int2 mnext = mw[j + 1];   // prefetch (reads past the slice on the last key: unused)
                const int tix = cq - (mm.x & 0xffff);
                f2 tb[NP], kj[C / 2], vj[C / 2];
                lds_tab<NP, NHP>(tb, tab_s, tix);
                lds_row<C>(kj, kvw + (size_t)j * 2 * C);
                lds_row<C>(vj, kvw + (size_t)j * 2 * C + C);
#pragma unroll
                for (int h = 0; h < NH; ++h)
                    atomicAdd(&dtp[h], (dt_t)fx[h]);
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
            for (int n = 0; n < nk; ++n) {
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
                dtau_s[(tid >> 6) * NH + 2 * P] = v.x;
                dtau_s[(tid >> 6) * NH + 2 * P + 1] = v.y;
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        const dt_t v = dtab_s[(e / NH) * DS + e % NH];
        if (v != 0) atomicAdd(&a.dtab_fix[e], v);
    }
    if (KIND == 1 && tid < NH) {   // this block's partial row, waves summed in a fixed order
        float v = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v += dtau_s[w * NH + tid];
        a.dtau_part[(size_t)blockIdx.x * NH + tid] = v * ifs / (a.tau[tid] * kLog2e);
    }
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
static void* pk_fwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_fwd_pk_kernel<C, 1, MAXT>)
                : reinterpret_cast<void*>(&wattn_fwd_pk_kernel<C, 0, MAXT>);
}
template <int C, int MAXT>
static void* pk_bwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_bwd_pk_kernel<C, 1, MAXT>)
                : reinterpret_cast<void*>(&wattn_bwd_pk_kernel<C, 0, MAXT>);
}

template <int C, int MAXT>
static void* pk2_fwd(int kind) {
    return kind ? reinterpret_cast<void*>(&wattn_fwd_pk2_kernel<C, 1, MAXT>)
                : reinterpret_cast<void*>(&wattn_fwd_pk2_kernel<C, 0, MAXT>);
}

// Forward blocks of <= 512 threads: two blocks share a CU, so one block's K/V gather overlaps
// the other's compute.  qpl_f: queries per lane of the forward (2: the two-query kernel, windows
// of even N >= 64).  The backward here is the one-row kernel; kind 0 at 6^3 windows takes the
// row-broadcast backward (wattn_bc.hip) before this dispatch.
int wattn_pk_kernels(int C, int kind, int N, void*& kf, void*& kb, int& maxt_f, int& maxt_b, int& qpl_f) {
    const bool two = N % 2 == 0 && N >= 64;
    qpl_f = two ? 2 : 1;
    if (C == 12) {
        kf = two ? pk2_fwd<12, 512>(kind) : pk_fwd<12, 512>(kind);
        maxt_f = 512;
        kb = pk_bwd<12, 1024>(kind);
        maxt_b = 1024;
        return 1;
    }
    if (C == 24) { kf = pk_fwd<24, 512>(kind); kb = pk_bwd<24, 512>(kind); maxt_f = 512; maxt_b = 512; qpl_f = 1; return 1; }
    return 0;
}

}  // namespace mmni
