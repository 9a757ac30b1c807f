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
}

// ------------------------------------------------------------------------------------
// backward (same two-pass structure and LDS regions as wattn_bwd_kernel)
// ------------------------------------------------------------------------------------
template <int C, int KIND, int MAXT>
__global__ __launch_bounds__(MAXT) void wattn_bwd_pk_kernel(WAArgs a) {
    constexpr int HD = 2, NH = C / HD, NP = NH / 2;
    static_assert(NH % 2 == 0, "head pairs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB;
    const int T = WPB * NPAD;
    float* R = smem;
    float* kv_s = R;                                      // pass A: [T][2C] pk k (k-hat), pk v
    float* qd_s = R;                                      // pass B: [T][2C] pk a2, pk dO
    float* rs_s = R + (size_t)T * 2 * C;                  // pass B: [T][2NH] lse2, delta (head order)
    int2* meta_s = reinterpret_cast<int2*>(R + (size_t)T * (2 * C + 2 * NH));
    float* tab_s = reinterpret_cast<float*>(meta_s + T);
    // table gradient rows padded to an odd stride DS = NH + 1 (u64 words): with stride 6 the
    // 64-bit atomics of queries 16 entries apart hit the same LDS banks
    constexpr int DS = NH + 1;
    unsigned long long* dtab_s = reinterpret_cast<unsigned long long*>(tab_s + ((g.Tsz * NH + 1) & ~1));
    float* dtau_s = reinterpret_cast<float*>(dtab_s + g.Tsz * DS);

    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / N, t = r - wl * N;
    const int wl_c = wl < WPB ? wl : WPB - 1;
    const int lane = tid & 63;

    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) tab_s[e] = a.table[e] * kLog2e;
    for (int e = tid; e < g.Tsz * DS; e += blockDim.x) dtab_s[e] = 0ull;
    if (tid < NH) dtau_s[tid] = 0.f;
    const f2 fscale = splat(exp2f((float)fix_exponent(a.maxbits, HD)));
    f2 dtr[NP];
#pragma unroll
    for (int P = 0; P < NP; ++P) dtr[P] = splat(0.f);

    for (int grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        const int own = wl_c * NPAD + (active ? t : 0);
        f2 aq[C / 2], dO[C / 2], lse2[NP], dl[NP];
        int64_t row = 0;
        int code = 0, rc = 0;
        if (active) {
            const TokenInfo ti = token_info(g, w, t);
            row = ti.row;
            code = ti.code;
            rc = ti.rc;
            float qr[C], gr[C], orow[C], dd[NH];
            load_row<C>(qr, a.q + row * a.qs);
            if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(qr, nrm); }
            load_row<C>(gr, a.dout + row * a.os);
            load_row<C>(orow, a.o + row * a.os);
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const float t2 = (KIND == 1) ? a.tau[h] * kLog2e : a.scale * kLog2e;
                qr[2 * h] *= t2;
                qr[2 * h + 1] *= t2;
                dd[h] = fmaf(orow[2 * h], gr[2 * h], orow[2 * h + 1] * gr[2 * h + 1]);
            }
            pack_row<C>(aq, qr);
            pack_row<C>(dO, gr);
#pragma unroll
            for (int P = 0; P < NP; ++P) {
                lse2[P] = (f2){a.lse[row * NH + 2 * P], a.lse[row * NH + 2 * P + 1]} * kLog2e;
                dl[P] = (f2){dd[2 * P], dd[2 * P + 1]};
            }
        } else {
#pragma unroll
            for (int i = 0; i < C / 2; ++i) { aq[i] = splat(0.f); dO[i] = splat(0.f); }
#pragma unroll
            for (int P = 0; P < NP; ++P) { lse2[P] = splat(INFINITY); dl[P] = splat(0.f); }
        }
        // ---- stage K/V + metadata (owners write their row; pad rows get neutral values)
        if (active && p == 0) {
            float kr[C], vr[C];
            load_row<C>(kr, a.k + row * a.ks);
            if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kr, nrm); }
            load_row<C>(vr, a.v + row * a.vs);
            f2 kp[C / 2], vp[C / 2];
            pack_row<C>(kp, kr);
            pack_row<C>(vp, vr);
            store_pk<C>(kv_s + (size_t)own * 2 * C, kp);
            store_pk<C>(kv_s + (size_t)own * 2 * C + C, vp);
            meta_s[own] = make_int2(code | (rc << 16), 0);
        }
        for (int e = tid; e < T; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                float4* z = reinterpret_cast<float4*>(kv_s + (size_t)e * 2 * C);
#pragma unroll
                for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                meta_s[e] = make_int2(0, __float_as_int(-INFINITY));
            }
        }
        __syncthreads();
        const int2* mw = meta_s + wl_c * NPAD;
        const int nk = NPAD / KS;

        // ================= pass A: lane = query row -> dq, dtable, dtau
        {
            const float* kvw = kv_s + (size_t)wl_c * NPAD * 2 * C;
            f2 dqa[C / 2];
#pragma unroll
            for (int i = 0; i < C / 2; ++i) dqa[i] = splat(0.f);
            const int cq = code + g.off;
            // key schedule: lane p walks its own contiguous quarter of the keys.  With the
            // interleaved order (p + KS*n) the 16 queries x 4 keys of a wave-instruction repeat
            // the same relative offset, i.e. the same table-gradient address, ~3 times: the
            // 64-bit LDS atomics then serialise.  Keys N/KS apart never share an offset within a
            // wave's 16 consecutive queries.
            for (int n = 0; n < nk; ++n) {
                const int j = p * nk + n;
                const int2 mt = mw[j];
                const int kcode = mt.x & 0xffff, rcj = mt.x >> 16;
                const float madd = (rcj == rc ? 0.f : kMask2) + __int_as_float(mt.y);
                const int tix = (cq - kcode) * NH;
                const int dix = (cq - kcode) * DS;
                const f2* tb = reinterpret_cast<const f2*>(tab_s + tix);
                const f2* kj = reinterpret_cast<const f2*>(kvw + (size_t)j * 2 * C);
                const f2* vj = kj + C / 2;
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 pr;
                    if constexpr (KIND == 1) {
                        f2 dot = aq[2 * P] * kj[2 * P];
                        dot = pfma(aq[2 * P + 1], kj[2 * P + 1], dot);
                        pr = exp2_2(dot + (tb[P] + (splat(madd) - lse2[P])));
                        f2 dp = dO[2 * P] * vj[2 * P];
                        dp = pfma(dO[2 * P + 1], vj[2 * P + 1], dp);
                        const f2 ds = pr * (dp - dl[P]);
                        dtr[P] = pfma(ds, dot, dtr[P]);
                        dqa[2 * P] = pfma(ds, kj[2 * P], dqa[2 * P]);
                        dqa[2 * P + 1] = pfma(ds, kj[2 * P + 1], dqa[2 * P + 1]);
                        const f2 fx = ds * fscale;
                        atomicAdd(&dtab_s[dix + 2 * P], (unsigned long long)(long long)__float2int_rn(fx.x));
                        atomicAdd(&dtab_s[dix + 2 * P + 1], (unsigned long long)(long long)__float2int_rn(fx.y));
                    } else {
                        f2 sc = tb[P] + (splat(madd) - lse2[P]);
                        sc = pfma(aq[2 * P], kj[2 * P], sc);
                        sc = pfma(aq[2 * P + 1], kj[2 * P + 1], sc);
                        pr = exp2_2(sc);
                        f2 dp = dO[2 * P] * vj[2 * P];
                        dp = pfma(dO[2 * P + 1], vj[2 * P + 1], dp);
                        const f2 ds = pr * (dp - dl[P]);
                        dqa[2 * P] = pfma(ds, kj[2 * P], dqa[2 * P]);
                        dqa[2 * P + 1] = pfma(ds, kj[2 * P + 1], dqa[2 * P + 1]);
                        const f2 fx = ds * fscale;
                        atomicAdd(&dtab_s[dix + 2 * P], (unsigned long long)(long long)__float2int_rn(fx.x));
                        atomicAdd(&dtab_s[dix + 2 * P + 1], (unsigned long long)(long long)__float2int_rn(fx.y));
                    }
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) dqa[i] += shfl2(dqa[i], o);
            }
            if (active && p == 0) {
                float dqn[C], dq[C];
                unpack_row<C>(dqn, dqa);
                if (KIND == 1) {
                    float qr[C], nrm[NH];
                    load_row<C>(qr, a.q + row * a.qs);
                    normalize_heads<C, HD>(qr, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dqn[h * HD + c] * a.tau[h];
                        normalize_bwd<HD>(dq + h * HD, dy, qr + h * HD, nrm[h]);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c) dq[c] = dqn[c] * a.scale;
                }
                store_row<C>(a.dq + row * a.qs, dq);
            }
        }
        __syncthreads();
        // ---- restage: pk a2 / pk dO and lse2 / delta rows for pass B
        if (active && p == 0) {
            store_pk<C>(qd_s + (size_t)own * 2 * C, aq);
            store_pk<C>(qd_s + (size_t)own * 2 * C + C, dO);
            f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)own * 2 * NH);
#pragma unroll
            for (int P = 0; P < NP; ++P) { rs[P] = lse2[P]; rs[NP + P] = dl[P]; }
        }
        for (int e = tid; e < T; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                float4* z = reinterpret_cast<float4*>(qd_s + (size_t)e * 2 * C);
#pragma unroll
                for (int c = 0; c < C / 2; ++c) z[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                f2* rs = reinterpret_cast<f2*>(rs_s + (size_t)e * 2 * NH);
#pragma unroll
                for (int P = 0; P < NP; ++P) { rs[P] = splat(INFINITY); rs[NP + P] = splat(0.f); }
            }
        }
        __syncthreads();

        // ================= pass B: lane = key row -> dk, dv
        {
            const float* qdw = qd_s + (size_t)wl_c * NPAD * 2 * C;
            const float* rsw = rs_s + (size_t)wl_c * NPAD * 2 * NH;
            f2 kr[C / 2], vr[C / 2], dka[C / 2], dva[C / 2];
            if (active) {
                float kn[C], vn[C];
                load_row<C>(kn, a.k + row * a.ks);
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kn, nrm); }
                load_row<C>(vn, a.v + row * a.vs);
                pack_row<C>(kr, kn);
                pack_row<C>(vr, vn);
            } else {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) { kr[i] = splat(0.f); vr[i] = splat(0.f); }
            }
#pragma unroll
            for (int i = 0; i < C / 2; ++i) { dka[i] = splat(0.f); dva[i] = splat(0.f); }
            for (int n = 0; n < nk; ++n) {
                const int i = p + KS * n;
                const int2 mt = mw[i];
                const int qcode = mt.x & 0xffff, rci = mt.x >> 16;
                const float madd = (rci == rc ? 0.f : kMask2) + __int_as_float(mt.y);
                const f2* tb = reinterpret_cast<const f2*>(tab_s + (qcode - code + g.off) * NH);
                const f2* ai = reinterpret_cast<const f2*>(qdw + (size_t)i * 2 * C);
                const f2* gi = ai + C / 2;
                const f2* rsi = reinterpret_cast<const f2*>(rsw + (size_t)i * 2 * NH);
#pragma unroll
                for (int P = 0; P < NP; ++P) {
                    f2 sc = tb[P] + (splat(madd) - rsi[P]);
                    sc = pfma(ai[2 * P], kr[2 * P], sc);
                    sc = pfma(ai[2 * P + 1], kr[2 * P + 1], sc);
                    const f2 pr = exp2_2(sc);
                    f2 dp = gi[2 * P] * vr[2 * P];
                    dp = pfma(gi[2 * P + 1], vr[2 * P + 1], dp);
                    const f2 ds = pr * (dp - rsi[NP + P]);
                    dva[2 * P] = pfma(pr, gi[2 * P], dva[2 * P]);
                    dva[2 * P + 1] = pfma(pr, gi[2 * P + 1], dva[2 * P + 1]);
                    dka[2 * P] = pfma(ds, ai[2 * P], dka[2 * P]);
                    dka[2 * P + 1] = pfma(ds, ai[2 * P + 1], dka[2 * P + 1]);
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int i = 0; i < C / 2; ++i) {
                    dka[i] += shfl2(dka[i], o);
                    dva[i] += shfl2(dva[i], o);
                }
            }
            if (active && p == 0) {
                float dkn[C], dk[C], dv[C];
                unpack_row<C>(dkn, dka);
                unpack_row<C>(dv, dva);
                if (KIND == 1) {
                    float kraw[C], nrm[NH];
                    load_row<C>(kraw, a.k + row * a.ks);
                    normalize_heads<C, HD>(kraw, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dkn[h * HD + c] * kLn2;
                        normalize_bwd<HD>(dk + h * HD, dy, kraw + h * HD, nrm[h]);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c) dk[c] = dkn[c] * kLn2;
                }
                store_row<C>(a.dk + row * a.ks, dk);
                store_row<C>(a.dv + row * a.vs, dv);
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
        const unsigned long long v = dtab_s[(e / NH) * DS + e % NH];
        if (v != 0ull) atomicAdd(&a.dtab_fix[e], v);
    }
    if (KIND == 1 && tid < NH) atomicAdd(&a.dtau[tid], dtau_s[tid] / (a.tau[tid] * kLog2e));
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

// Forward blocks of <= 512 threads (KS = 2 at N = 216): two blocks share a CU, so one block's
// K/V gather overlaps the other's compute.  The backward's LDS (bias table + its 64-bit
// gradient) allows one block per CU; it keeps 1024 threads (KS = 4) for occupancy.
int wattn_pk_kernels(int C, int kind, void*& kf, void*& kb, int& maxt_f, int& maxt_b) {
    if (C == 12) { kf = pk_fwd<12, 512>(kind); kb = pk_bwd<12, 1024>(kind); maxt_f = 512; maxt_b = 1024; return 1; }
    if (C == 24) { kf = pk_fwd<24, 512>(kind); kb = pk_bwd<24, 512>(kind); maxt_f = 512; maxt_b = 512; return 1; }
    return 0;
}

}  // namespace mmni
