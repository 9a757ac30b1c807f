// Shifted-window attention for gfx950.
//
// Replaces, on the device:
//   torch.roll + window_partition            modules/swin_v2_module.py:35-46,277-284
//                                            modules/swinfusion_module.py:33-45,350-357
//   WindowAttention_fusion.forward           modules/swinfusion_module.py:114-145
//   Cross_WindowAttention.forward            modules/swinfusion_module.py:213-246
//   WindowAttention.forward (cosine, Swin-V2) modules/swin_v2_module.py:138-178
//   window_reverse + reverse roll            modules/swinfusion_module.py:366-373
// between the qkv projection and the output projection (both stay GEMMs).
//
// Design (MI355X-first):
//  * head_dim is 2 (SwinFusion) or 4 (Swin-V2): the QK^T and AV contractions have K = 2..4,
//    far below any MFMA K-tile, so the kernels run the contractions on the fp32 VALU and
//    account for that honestly in the roofline.
//  * One workgroup owns WPB whole windows at a time (grid-stride over window groups, so the
//    bias table is staged into LDS once per workgroup).  K/V of the window are gathered from
//    the un-partitioned channels-last tensor straight into LDS: the roll/partition copies of
//    the reference never exist in HBM.
//  * Each query row is owned by KS adjacent lanes that split the keys; every lane keeps all
//    heads of its row in registers so the relative index, shift-mask test and K/V broadcast
//    reads are shared by all heads.  Partial softmax states merge with __shfl_xor.
//  * Softmax runs in the log2 domain (q, bias and mask pre-scaled by log2 e) with an online
//    max over chunks of CH keys: one v_exp_f32 per (row, key, head) + one per chunk.
//  * The shift mask (-100 between regions) is the analytic region-equivalence rule, the
//    relative-position index is code(query) - code(key) + offset — no N x N tensors in HBM.
//  * Backward recomputes P from the saved log-sum-exp: pass A (lane = query row) produces
//    dq and the bias-table gradient (LDS atomics, flushed once per workgroup), pass B
//    (lane = key row) produces dk and dv.  dq/dk/dv need no cross-window reduction.
#include "wattn_common.h"

namespace mmni {

// max|dout| and max|v| for the fixed-point bound (non-negative float bits order as uints).
// dout == nullptr: v only; v == nullptr: dout only.  Rows in a grid-stride loop (no 64-bit
// division per element), the block's maximum through LDS, ONE atomic per block and word (per-wave
// atomics on one word serialise at the L2: 4,096 of them cost ~48 us).
__global__ __launch_bounds__(256) void wattn_absmax_kernel(const float* dout, long long os, const float* v,
                                                           long long vs, long long T, int C,
                                                           unsigned int* maxbits) {
    __shared__ float red[2][4];
    float md = 0.f, mv = 0.f;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // a wave covers rpw whole rows per step (C <= 64: lane = sub-row * C + c) or one row in 64-lane
    // pieces (C > 64)
    const int rpw = C <= 64 ? 64 / C : 1;
    const int sub = C <= 64 ? lane / C : 0, c0 = C <= 64 ? lane - sub * C : lane, cstep = C <= 64 ? C : 64;
    if (sub < rpw) {
        const long long nw = (long long)gridDim.x * 4 * rpw;
#pragma unroll 4
        for (long long r = ((long long)blockIdx.x * 4 + wave) * rpw + sub; r < T; r += nw) {
            for (int c = c0; c < C; c += cstep) {
                if (dout) md = fmaxf(md, fabsf(dout[r * os + c]));
                if (v) mv = fmaxf(mv, fabsf(v[r * vs + c]));
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        md = fmaxf(md, __shfl_xor(md, o));
        mv = fmaxf(mv, __shfl_xor(mv, o));
    }
    if (lane == 0) { red[0][wave] = md; red[1][wave] = mv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        md = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
        mv = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
        if (dout) atomicMax(&maxbits[0], __float_as_uint(md));
        if (v) atomicMax(&maxbits[1], __float_as_uint(mv));
    }
}

// blocks of the generic scan: ~16 elements per lane, at most 2,048 blocks (one atomic each)
static unsigned absmax_blocks(long long T, int C) {
    long long b = (T * C + 4095) / 4096;
    return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

// max|dout| over a contiguous, 16-byte aligned array of n4 float4 (the common case: dout rows of
// C % 4 == 0 floats, stride C), and max|v| taken from the forward's running maximum (vmax).
// (One same-address atomic per block: per-wave atomics on one word serialise at the L2 and
// cost ~60 us at 8k waves.)
__global__ __launch_bounds__(1024) void wattn_absmax_dout4_kernel(const float4* dout, long long n4,
                                                                  const unsigned int* vmax, unsigned int* maxbits) {
    __shared__ float red[16];
    float md = 0.f;
    // four independent 16-B loads in flight per lane (one per lane leaves HBM latency exposed)
    const long long stride = (long long)gridDim.x * 1024;
    long long i = blockIdx.x * 1024ll + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        float4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = dout[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            md = fmaxf(md, fmaxf(fmaxf(fabsf(x[u].x), fabsf(x[u].y)), fmaxf(fabsf(x[u].z), fabsf(x[u].w))));
    }
    for (; i < n4; i += stride) {
        const float4 x = dout[i];
        md = fmaxf(md, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
    }
    for (int o = 32; o > 0; o >>= 1) md = fmaxf(md, __shfl_xor(md, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = md;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) md = fmaxf(md, red[w]);
        atomicMax(&maxbits[0], __float_as_uint(md));
        if (blockIdx.x == 0) atomicMax(&maxbits[1], *vmax);
    }
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int C, int HD, int KIND, int MAXT>
__global__ __launch_bounds__(MAXT) void wattn_fwd_kernel(WAArgs a) {
    constexpr int NH = C / HD;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB;
    float* kv_s = smem;                                              // [WPB*NPAD][2C]
    int2* meta_s = reinterpret_cast<int2*>(kv_s + (size_t)WPB * NPAD * 2 * C);  // [WPB*NPAD]
    float* tab_s = reinterpret_cast<float*>(meta_s + WPB * NPAD);     // [Tsz][NH]

    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / N, t = r - wl * N;
    const int wl_c = wl < WPB ? wl : WPB - 1;
    // head group blockIdx.y of a.hsplit: this block's heads h0 .. h0 + NH - 1 of NHT
    const int NHT = NH * a.hsplit, h0 = blockIdx.y * NH;
    a.q += h0 * HD; a.k += h0 * HD; a.v += h0 * HD; a.out += h0 * HD; a.tau += h0;

    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) tab_s[e] = a.table[(e / NH) * NHT + h0 + e % NH] * kLog2e;

    float tau2[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) tau2[h] = (KIND == 1) ? a.tau[h] * kLog2e : a.scale * kLog2e;

    for (int grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
        // ---- stage K/V of WPB windows (gathered through the shift) into LDS
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
            store_row<C>(kv_s + (size_t)e * 2 * C, kr);
            store_row<C>(kv_s + (size_t)e * 2 * C + C, vr);
            meta_s[e] = mt;
        }

        // ---- own query row (prescaled into the log2 domain)
        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        float q[C];
        int cq = 0, rq = 0;
        int64_t row = 0;
        if (active) {
            const TokenInfo ti = token_info(g, w, t);
            row = ti.row;
            cq = ti.code + g.off;
            rq = ti.rc;
            load_row<C>(q, a.q + row * a.qs);
            if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(q, nrm); }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) q[c] = 0.f;
        }
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int c = 0; c < HD; ++c) q[h * HD + c] *= tau2[h];
        __syncthreads();

        float m[NH], l[NH], acc[C];
#pragma unroll
        for (int h = 0; h < NH; ++h) { m[h] = -INFINITY; l[h] = 0.f; }
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;

        const float* kvw = kv_s + (size_t)wl_c * NPAD * 2 * C;
        const int2* mw = meta_s + wl_c * NPAD;
        const int nk = NPAD / KS;
        for (int n = 0; n < nk; n += CH) {
            float s[CH][NH];
#pragma unroll
            for (int cc = 0; cc < CH; ++cc) {
                const int j = p + KS * (n + cc);
                const int2 mt = mw[j];
                const int code = mt.x & 0xffff, rcj = mt.x >> 16;
                const float madd = (rcj == rq ? 0.f : kMask2) + __int_as_float(mt.y);
                const float* tb = tab_s + (cq - code) * NH;
                float kr[C];
                load_row<C>(kr, kvw + (size_t)j * 2 * C);
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    float d = tb[h] + madd;
#pragma unroll
                    for (int c = 0; c < HD; ++c) d = fmaf(q[h * HD + c], kr[h * HD + c], d);
                    s[cc][h] = d;
                }
            }
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                float cm = s[0][h];
#pragma unroll
                for (int cc = 1; cc < CH; ++cc) cm = fmaxf(cm, s[cc][h]);
                const float mn = fmaxf(m[h], cm);
                const float alpha = fast_exp2(m[h] - mn);
                m[h] = mn;
                l[h] *= alpha;
#pragma unroll
                for (int c = 0; c < HD; ++c) acc[h * HD + c] *= alpha;
            }
#pragma unroll
            for (int cc = 0; cc < CH; ++cc) {
                const int j = p + KS * (n + cc);
                float vr[C];
                load_row<C>(vr, kvw + (size_t)j * 2 * C + C);
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const float pj = fast_exp2(s[cc][h] - m[h]);
                    l[h] += pj;
#pragma unroll
                    for (int c = 0; c < HD; ++c) acc[h * HD + c] = fmaf(pj, vr[h * HD + c], acc[h * HD + c]);
                }
            }
        }
        // ---- merge the KS partial states of this row (adjacent lanes)
        for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const float mo = __shfl_xor(m[h], o);
                const float lo = __shfl_xor(l[h], o);
                const float mn = fmaxf(m[h], mo);
                const float fa = fast_exp2(m[h] - mn), fb = fast_exp2(mo - mn);
                l[h] = l[h] * fa + lo * fb;
#pragma unroll
                for (int c = 0; c < HD; ++c) {
                    const float ao = __shfl_xor(acc[h * HD + c], o);
                    acc[h * HD + c] = acc[h * HD + c] * fa + ao * fb;
                }
                m[h] = mn;
            }
        }
        if (active && p == 0) {
            float o[C];
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const float inv = 1.0f / l[h];
#pragma unroll
                for (int c = 0; c < HD; ++c) o[h * HD + c] = acc[h * HD + c] * inv;
                a.lse[row * NHT + h0 + h] = (m[h] + fast_log2(l[h])) * kLn2;
            }
            store_row<C>(a.out + row * a.os, o);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
template <int C, int HD, int KIND, int MAXT>
__global__ __launch_bounds__(MAXT) void wattn_bwd_kernel(WAArgs a) {
    // LDS: one region R reused by both passes (K/V rows for pass A, then a2/dO + lse/delta rows
    // for pass B), plus key metadata, the bias table and the fixed-point table gradient.
    constexpr int NH = C / HD;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int N = g.N, NPAD = a.NPAD, KS = a.KS, WPB = a.WPB;
    const int T = WPB * NPAD;
    float* R = smem;                                      // max(T*2C, T*(2C + 2NH)) floats
    float* kv_s = R;                                      // pass A: [T][2C] k (k-hat), v
    float* qd_s = R;                                      // pass B: [T][2C] a2, dO
    float* rs_s = R + (size_t)T * 2 * C;                  // pass B: [T][2NH] lse2, delta
    int2* meta_s = reinterpret_cast<int2*>(R + (size_t)T * (2 * C + 2 * NH));   // [T]
    float* tab_s = reinterpret_cast<float*>(meta_s + T); // [Tsz][NH] (log2 domain)
    unsigned long long* dtab_s =                          // [Tsz][NH] grad, 64-bit fixed point
        reinterpret_cast<unsigned long long*>(tab_s + ((g.Tsz * NH + 1) & ~1));
    float* dtau_s = reinterpret_cast<float*>(dtab_s + g.Tsz * NH);   // [kMaxWaves][NH]

    const int tid = threadIdx.x;
    const int r = tid / KS, p = tid - r * KS;
    const int wl = r / N, t = r - wl * N;
    const int wl_c = wl < WPB ? wl : WPB - 1;
    const int lane = tid & 63;
    // head group blockIdx.y of a.hsplit: this block's heads h0 .. h0 + NH - 1 of NHT
    const int NHT = NH * a.hsplit, h0 = blockIdx.y * NH;
    a.q += h0 * HD; a.k += h0 * HD; a.v += h0 * HD; a.o += h0 * HD; a.dout += h0 * HD;
    a.dq += h0 * HD; a.dk += h0 * HD; a.dv += h0 * HD; a.tau += h0;

    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        tab_s[e] = a.table[(e / NH) * NHT + h0 + e % NH] * kLog2e;
        dtab_s[e] = 0ull;
    }
    const float ymul = exp2f((float)fix_exponent(a.maxbits, HD));
    float dtr[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) dtr[h] = 0.f;

    for (int grp = blockIdx.x; grp < a.ngroups; grp += gridDim.x) {
        const int w = grp * WPB + wl;
        const bool active = (wl < WPB) && (w < g.nwin);
        const int own = wl_c * NPAD + (active ? t : 0);
        // ---- own row into registers: a2 (prescaled q), dO, lse2, delta
        float aq[C], dO[C], lse2[NH], dl[NH];
        int64_t row = 0;
        int code = 0, rc = 0;
        if (active) {
            const TokenInfo ti = token_info(g, w, t);
            row = ti.row;
            code = ti.code;
            rc = ti.rc;
            load_row<C>(aq, a.q + row * a.qs);
            if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(aq, nrm); }
            float o[C];
            load_row<C>(dO, a.dout + row * a.os);
            load_row<C>(o, a.o + row * a.os);
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const float t2 = (KIND == 1) ? a.tau[h] * kLog2e : a.scale * kLog2e;
                float dd = 0.f;
#pragma unroll
                for (int c = 0; c < HD; ++c) {
                    aq[h * HD + c] *= t2;
                    dd = fmaf(o[h * HD + c], dO[h * HD + c], dd);
                }
                lse2[h] = a.lse[row * NHT + h0 + h] * kLog2e;
                dl[h] = dd;
            }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) { aq[c] = 0.f; dO[c] = 0.f; }
#pragma unroll
            for (int h = 0; h < NH; ++h) { lse2[h] = INFINITY; dl[h] = 0.f; }
        }
        // ---- stage K/V + metadata (owners write their row; pad rows get neutral values)
        if (active && p == 0) {
            float kr[C], vr[C];
            load_row<C>(kr, a.k + row * a.ks);
            if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kr, nrm); }
            load_row<C>(vr, a.v + row * a.vs);
            store_row<C>(kv_s + (size_t)own * 2 * C, kr);
            store_row<C>(kv_s + (size_t)own * 2 * C + C, vr);
            meta_s[own] = make_int2(code | (rc << 16), 0);
        }
        for (int e = tid; e < T; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                float z[C];
#pragma unroll
                for (int c = 0; c < C; ++c) z[c] = 0.f;
                store_row<C>(kv_s + (size_t)e * 2 * C, z);
                store_row<C>(kv_s + (size_t)e * 2 * C + C, z);
                meta_s[e] = make_int2(0, __float_as_int(-INFINITY));
            }
        }
        __syncthreads();
        const int2* mw = meta_s + wl_c * NPAD;
        const int nk = NPAD / KS;

        // ================= pass A: lane = query row -> dq, dtable, dtau
        {
            const float* kvw = kv_s + (size_t)wl_c * NPAD * 2 * C;
            float dqa[C];
#pragma unroll
            for (int c = 0; c < C; ++c) dqa[c] = 0.f;
            const int cq = code + g.off;
            for (int n = 0; n < nk; ++n) {
                const int j = p * nk + n;   // contiguous key quarters: see wattn_pk.hip pass A
                const int2 mt = mw[j];
                const int kcode = mt.x & 0xffff, rcj = mt.x >> 16;
                const float madd = (rcj == rc ? 0.f : kMask2) + __int_as_float(mt.y);
                const int tix = (cq - kcode) * NH;
                float kj[C], vj[C];
                load_row<C>(kj, kvw + (size_t)j * 2 * C);
                load_row<C>(vj, kvw + (size_t)j * 2 * C + C);
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    float dot = 0.f, dp = 0.f;
#pragma unroll
                    for (int c = 0; c < HD; ++c) {
                        dot = fmaf(aq[h * HD + c], kj[h * HD + c], dot);
                        dp = fmaf(dO[h * HD + c], vj[h * HD + c], dp);
                    }
                    const float pr = fast_exp2(dot + tab_s[tix + h] + madd - lse2[h]);
                    const float ds = pr * (dp - dl[h]);
#pragma unroll
                    for (int c = 0; c < HD; ++c) dqa[h * HD + c] = fmaf(ds, kj[h * HD + c], dqa[h * HD + c]);
                    atomicAdd(&dtab_s[tix + h], to_fixed(ds, ymul));
                    if constexpr (KIND == 1) dtr[h] = fmaf(ds, dot, dtr[h]);
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int c = 0; c < C; ++c) dqa[c] += __shfl_xor(dqa[c], o);
            }
            if (active && p == 0) {
                float dq[C];
                if (KIND == 1) {
                    float qr[C], nrm[NH];
                    load_row<C>(qr, a.q + row * a.qs);
                    normalize_heads<C, HD>(qr, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dqa[h * HD + c] * a.tau[h];
                        normalize_bwd<HD>(dq + h * HD, dy, qr + h * HD, nrm[h]);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c) dq[c] = dqa[c] * a.scale;
                }
                store_row<C>(a.dq + row * a.qs, dq);
            }
        }
        __syncthreads();
        // ---- restage: a2/dO and lse2/delta rows for pass B (owners from registers)
        if (active && p == 0) {
            store_row<C>(qd_s + (size_t)own * 2 * C, aq);
            store_row<C>(qd_s + (size_t)own * 2 * C + C, dO);
            float* rs = rs_s + (size_t)own * 2 * NH;
#pragma unroll
            for (int h = 0; h < NH; ++h) { rs[h] = lse2[h]; rs[NH + h] = dl[h]; }
        }
        for (int e = tid; e < T; e += blockDim.x) {
            const int w2 = e / NPAD, t2 = e - w2 * NPAD;
            if (t2 >= N || grp * WPB + w2 >= g.nwin) {
                float z[C];
#pragma unroll
                for (int c = 0; c < C; ++c) z[c] = 0.f;
                store_row<C>(qd_s + (size_t)e * 2 * C, z);
                store_row<C>(qd_s + (size_t)e * 2 * C + C, z);
                float* rs = rs_s + (size_t)e * 2 * NH;
#pragma unroll
                for (int h = 0; h < NH; ++h) { rs[h] = INFINITY; rs[NH + h] = 0.f; }
            }
        }
        __syncthreads();

        // ================= pass B: lane = key row -> dk, dv
        {
            const float* qdw = qd_s + (size_t)wl_c * NPAD * 2 * C;
            const float* rsw = rs_s + (size_t)wl_c * NPAD * 2 * NH;
            float kr[C], vr[C], dka[C], dva[C];
            if (active) {
                load_row<C>(kr, a.k + row * a.ks);
                if (KIND == 1) { float nrm[NH]; normalize_heads<C, HD>(kr, nrm); }
                load_row<C>(vr, a.v + row * a.vs);
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) { kr[c] = 0.f; vr[c] = 0.f; }
            }
#pragma unroll
            for (int c = 0; c < C; ++c) { dka[c] = 0.f; dva[c] = 0.f; }
            for (int n = 0; n < nk; ++n) {
                const int i = p + KS * n;
                const int2 mt = mw[i];
                const int qcode = mt.x & 0xffff, rci = mt.x >> 16;
                const float madd = (rci == rc ? 0.f : kMask2) + __int_as_float(mt.y);
                const int tix = (qcode - code + g.off) * NH;
                float ai[C], gi[C];
                load_row<C>(ai, qdw + (size_t)i * 2 * C);
                load_row<C>(gi, qdw + (size_t)i * 2 * C + C);
                const float* rsi = rsw + (size_t)i * 2 * NH;
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    float dot = 0.f, dp = 0.f;
#pragma unroll
                    for (int c = 0; c < HD; ++c) {
                        dot = fmaf(ai[h * HD + c], kr[h * HD + c], dot);
                        dp = fmaf(gi[h * HD + c], vr[h * HD + c], dp);
                    }
                    const float pr = fast_exp2(dot + tab_s[tix + h] + madd - rsi[h]);
                    const float ds = pr * (dp - rsi[NH + h]);
#pragma unroll
                    for (int c = 0; c < HD; ++c) {
                        dva[h * HD + c] = fmaf(pr, gi[h * HD + c], dva[h * HD + c]);
                        dka[h * HD + c] = fmaf(ds, ai[h * HD + c], dka[h * HD + c]);
                    }
                }
            }
            for (int o = 1; o < KS; o <<= 1) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    dka[c] += __shfl_xor(dka[c], o);
                    dva[c] += __shfl_xor(dva[c], o);
                }
            }
            if (active && p == 0) {
                float dk[C];
                if (KIND == 1) {
                    float kraw[C], nrm[NH];
                    load_row<C>(kraw, a.k + row * a.ks);
                    normalize_heads<C, HD>(kraw, nrm);
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        float dy[HD];
#pragma unroll
                        for (int c = 0; c < HD; ++c) dy[c] = dka[h * HD + c] * kLn2;
                        normalize_bwd<HD>(dk + h * HD, dy, kraw + h * HD, nrm[h]);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c) dk[c] = dka[c] * kLn2;
                }
                store_row<C>(a.dk + row * a.ks, dk);
                store_row<C>(a.dv + row * a.vs, dva);
            }
        }
        __syncthreads();
    }

    // ---- dtau: fixed butterfly per wave into its LDS slot, waves summed in order into this
    // block's partial row; flush the (exact, order-free) fixed-point table-gradient sums
    if (KIND == 1) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            float v = dtr[h];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) dtau_s[(tid >> 6) * NH + h] = v;
        }
    }
    __syncthreads();
    for (int e = tid; e < g.Tsz * NH; e += blockDim.x) {
        const unsigned long long v = dtab_s[e];
        if (v != 0ull) atomicAdd(&a.dtab_fix[(e / NH) * NHT + h0 + e % NH], v);
    }
    if (KIND == 1 && tid < NH) {
        // dtau = sum ds * (q-hat . k-hat);  dot was taken against tau*log2e*q-hat
        float v = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v += dtau_s[w * NH + tid];
        a.dtau_part[(size_t)blockIdx.x * NHT + h0 + tid] = v / (a.tau[tid] * kLog2e);
    }
}

__global__ void wattn_dtable_convert_kernel(const unsigned long long* fix, const unsigned int* maxbits, int hd,
                                            int shift, float* dtable, int n) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) dtable[e] += (float)ldexp((double)(long long)fix[e], -(fix_exponent(maxbits, hd) - shift));
}

// ------------------------------------------------------------------------------------
// integer maps (exported for parity tests)
// ------------------------------------------------------------------------------------
__global__ void window_rows_kernel(WGeom g, int32_t* rows) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)g.nwin * g.N) return;
    const int w = (int)(e / g.N), t = (int)(e % g.N);
    rows[e] = (int32_t)token_info(g, w, t).row;
}

__global__ void window_mask_kernel(WGeom g, int nWs, float* mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t NN = (int64_t)g.N * g.N;
    if (e >= (int64_t)nWs * NN) return;
    const int w = (int)(e / NN);
    const int ij = (int)(e % NN);
    const int i = ij / g.N, j = ij % g.N;
    const int ri = token_info(g, w, i).rc, rj = token_info(g, w, j).rc;
    mask[e] = (ri == rj) ? 0.f : -100.f;
}

__global__ void relative_index_kernel(WGeom g, int32_t* idx) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= g.N * g.N) return;
    const int i = e / g.N, j = e % g.N;
    idx[e] = token_info(g, 0, i).code - token_info(g, 0, j).code + g.off;
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
static int make_geom(const mmni_wattn_desc* d, WGeom& g) {
    MMNI_ARG_CHECK(d != nullptr, "wattn: null descriptor");
    MMNI_ARG_CHECK(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0, "wattn: bad extents B=%d D=%d H=%d W=%d",
                   d->B, d->D, d->H, d->W);
    MMNI_ARG_CHECK(d->wd > 0 && d->wh > 0 && d->ww > 0, "wattn: bad window");
    MMNI_ARG_CHECK(d->D % d->wd == 0 && d->H % d->wh == 0 && d->W % d->ww == 0,
                   "wattn: extents (%d,%d,%d) not multiples of window (%d,%d,%d)", d->D, d->H, d->W,
                   d->wd, d->wh, d->ww);
    MMNI_ARG_CHECK(d->sd >= 0 && d->sd < d->wd && d->sh >= 0 && d->sh < d->wh && d->sw >= 0 && d->sw < d->ww,
                   "wattn: shift must satisfy 0 <= shift < window");
    g.B = d->B; g.D = d->D; g.H = d->H; g.W = d->W;
    g.wd = d->wd; g.wh = d->wh; g.ww = d->ww;
    g.sd = d->sd; g.sh = d->sh; g.sw = d->sw;
    g.nWd = d->D / d->wd; g.nWh = d->H / d->wh; g.nWw = d->W / d->ww;
    const int64_t nwin = (int64_t)d->B * g.nWd * g.nWh * g.nWw;
    MMNI_ARG_CHECK(nwin < (1ll << 31), "wattn: too many windows");
    MMNI_ARG_CHECK((int64_t)d->B * d->D * d->H * d->W < (1ll << 31), "wattn: too many tokens");
    g.nwin = (int)nwin;
    g.N = d->wd * d->wh * d->ww;
    g.th = 2 * d->ww - 1;
    g.tw = (2 * d->wh - 1) * g.th;
    g.off = (d->wd - 1) * g.tw + (d->wh - 1) * g.th + (d->ww - 1);
    g.Tsz = (2 * d->wd - 1) * g.tw;
    MMNI_ARG_CHECK(g.Tsz <= 0xffff, "wattn: relative table too large (%d)", g.Tsz);
    return 0;
}

template <int C, int HD, int MAXT>
struct WAKernels {
    static void* fwd(int kind) {
        return kind ? reinterpret_cast<void*>(&wattn_fwd_kernel<C, HD, 1, MAXT>)
                    : reinterpret_cast<void*>(&wattn_fwd_kernel<C, HD, 0, MAXT>);
    }
    static void* bwd(int kind) {
        return kind ? reinterpret_cast<void*>(&wattn_bwd_kernel<C, HD, 1, MAXT>)
                    : reinterpret_cast<void*>(&wattn_bwd_kernel<C, HD, 0, MAXT>);
    }
};

struct WAConfig {
    int KS, WPB, NPAD, threads, ngroups, grid;
    int cap;   // block cap of the launch (resident blocks; x4 for the forward)
    size_t lds;
};

// Generic backward: table rows of NH floats, table-gradient rows of NH u64.  Packed backward
// (wattn_pk.hip): table rows padded to a multiple of 4 floats (float4 reads), table-gradient rows
// of NH + 1 u64 (odd stride).
static size_t wattn_lds_bytes(bool bwd, bool packed, int C, int NH, int WPB, int NPAD, int Tsz) {
    const size_t T = (size_t)WPB * NPAD;
    if (!bwd) return T * 2 * C * 4 + T * 8 + (size_t)Tsz * NH * 4;
    if (packed)
        return T * (2 * C + 2 * NH) * 4 + T * 8 + (size_t)Tsz * (NH == 2 ? 2 : (NH + 3) & ~3) * 4 +
               (size_t)Tsz * (NH + kDtabPad) * 8 +
               (size_t)kMaxWaves * NH * 4;
    const size_t tab = (size_t)((Tsz * NH + 1) & ~1) * 4;
    return T * (2 * C + 2 * NH) * 4 + T * 8 + tab + (size_t)Tsz * NH * 8 + (size_t)kMaxWaves * NH * 4;
}

// qpl: queries per lane (2 for wattn_fwd_pk2_kernel, forward only): a window occupies N / qpl x KS lanes.
// hs: head groups (blocks per window group, grid.y).  Small launches (few windows, e.g. the 3^3
// and 6^3 Swin-V2 stages of C2: 4 windows) spread over the CUs: 4 key slices per row and fewer
// windows per block, so windows x head groups make the blocks.
static int plan(const WGeom& g, int C, int NH, int maxt, bool bwd, bool packed, WAConfig& cfg, int qpl = 1,
                int hs = 1) {
    const int chunk = packed ? (qpl >= 2 ? kPk2Chunk : kPkChunk) : CH;
    const int N = g.N, R = N / qpl;
    const bool small = !packed && (int64_t)g.nwin * hs < kNumCU;
    int KS = qpl >= 2 ? kPk2Ks : (N >= 128 || small ? 4 : (N >= 32 ? 2 : 1));
    auto r64 = [](int x) { return (x + 63) / 64 * 64; };
    while (KS > 1 && r64(R * KS) > maxt) KS >>= 1;
    MMNI_ARG_CHECK(r64(R) <= maxt, "wattn: window of %d tokens exceeds %d threads", N, maxt);
    const int target = maxt < 512 ? maxt : 512;
    int WPB = target / (R * KS);
    if (qpl == 2 && !bwd && WPB > kPk2FwdWpb) WPB = kPk2FwdWpb;
    if (small) WPB = 1;
    if (WPB < 1) WPB = 1;
    const int NPAD = (N + KS * chunk - 1) / (KS * chunk) * (KS * chunk);
    while (WPB > 1 && wattn_lds_bytes(bwd, packed, C, NH, WPB, NPAD, g.Tsz) > 160 * 1024) --WPB;
    const size_t lds = wattn_lds_bytes(bwd, packed, C, NH, WPB, NPAD, g.Tsz);
    MMNI_ARG_CHECK(lds <= 160 * 1024, "wattn: LDS footprint %zu B exceeds 160 KiB", lds);
    cfg.KS = KS;
    cfg.WPB = WPB;
    cfg.NPAD = NPAD;
    cfg.threads = r64(WPB * R * KS);
    cfg.ngroups = (g.nwin + WPB - 1) / WPB;
    int per_cu = (int)((160 * 1024) / lds);
    const int by_threads = 2048 / cfg.threads;
    if (by_threads < per_cu) per_cu = by_threads;
    if (per_cu > 8) per_cu = 8;
    if (per_cu < 1) per_cu = 1;
    const int resident = kNumCU * per_cu;
    // forward: a few groups per block amortise the table staging; backward: one flush
    // of the table gradient per block, so stay at one resident wave of blocks.
    const int cap = bwd ? resident : resident * 4;
    cfg.cap = cap;
    cfg.grid = cfg.ngroups < cap ? cfg.ngroups : cap;
    cfg.lds = lds;
    return 0;
}

// C: the channels one block attends over (d->C, or d->C / head groups for the head-split launches)
static int dispatch(const mmni_wattn_desc* d, int C, int HD, bool bwd, void*& kf, void*& kb, int& maxt, bool& packed,
                    int& qpl) {
    packed = false;
    qpl = 1;
    int mf = 0, mb = 0, qf = 1;
    if (HD == 2 && wattn_pk_kernels(C, d->kind, d->wd * d->wh * d->ww, kf, kb, mf, mb, qf)) {
        maxt = bwd ? mb : mf;
        qpl = bwd ? 1 : qf;
        packed = true;
        return 0;
    }
#define MMNI_WA_CASE(CC, HH, MT)                         \
    if (C == CC && HD == HH) {                           \
        kf = WAKernels<CC, HH, MT>::fwd(d->kind);        \
        kb = WAKernels<CC, HH, MT>::bwd(d->kind);        \
        maxt = MT;                                       \
        return 0;                                        \
    }
    MMNI_WA_CASE(12, 2, 1024)
    MMNI_WA_CASE(4, 4, 1024)
    MMNI_WA_CASE(12, 4, 1024)
    MMNI_WA_CASE(24, 2, 512)
    MMNI_WA_CASE(24, 4, 512)
    MMNI_WA_CASE(48, 4, 256)
    MMNI_WA_CASE(6, 2, 1024)
#undef MMNI_WA_CASE
    set_error("wattn: unsupported (C=%d, head_dim=%d); supported: (12,2) (4,4) (12,4) (24,2) (24,4) (48,4) (6,2)", C, HD);
    return -2;
}

// Head groups for small launches of the generic head_dim-4 kernels (Swin-V2): each block takes
// C / hs channels (an instantiated width), so few windows still fill the chip.  The smallest split
// that reaches kNumCU blocks, else the largest available.
static int head_split(const WGeom& g, int C, int heads, int HD) {
    if (HD != 4 || (int64_t)g.nwin >= kNumCU) return 1;
    int best = 1;
    for (int hs = 2; hs <= heads; ++hs) {
        if (heads % hs) continue;
        const int cs = C / hs;
        if (cs != 4 && cs != 12 && cs != 24) continue;
        best = hs;
        if ((int64_t)g.nwin * hs >= kNumCU) break;
    }
    return best;
}

static int fill_args(const mmni_wattn_desc* d, WAArgs& a, int& HD) {
    int rc = make_geom(d, a.g);
    if (rc) return rc;
    MMNI_ARG_CHECK(d->heads > 0 && d->C % d->heads == 0, "wattn: C=%d not divisible by heads=%d", d->C, d->heads);
    MMNI_ARG_CHECK(d->kind == 0 || d->kind == 1, "wattn: kind must be 0 or 1");
    MMNI_ARG_CHECK(d->q_stride >= d->C && d->k_stride >= d->C && d->v_stride >= d->C && d->o_stride >= d->C,
                   "wattn: token strides must be >= C");
    HD = d->C / d->heads;
    a.kind = d->kind;
    a.scale = d->scale;
    a.qs = d->q_stride; a.ks = d->k_stride; a.vs = d->v_stride; a.os = d->o_stride;
    return 0;
}

// Dynamic LDS above 64 KiB: raise the per-function limit once (host-side attribute, no sync).
// Set once per kernel (a host-side attribute, no stream work: safe inside hipGraph capture).
static int ensure_lds_attr(void* fn, size_t bytes) {
    if (bytes <= 64 * 1024) return 0;
    static void* done[64];
    static int ndone = 0;
    for (int i = 0; i < ndone; ++i)
        if (done[i] == fn) return 0;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) { set_error("hipFuncSetAttribute: %s", hipGetErrorString(e)); return (int)e; }
    if (ndone < 64) done[ndone++] = fn;
    return 0;
}

// float4 row access needs 16-byte aligned rows when C % 4 == 0; scalar access otherwise.
static bool row_aligned(const void* p, int64_t stride, int C) {
    if (C % 4 != 0) return reinterpret_cast<uintptr_t>(p) % 4 == 0;
    return (reinterpret_cast<uintptr_t>(p) % 16 == 0) && (stride % 4 == 0);
}

}  // namespace mmni

using namespace mmni;

extern "C" int mmni_wattn_fwd(const mmni_wattn_desc* d, const float* q, const float* k, const float* v,
                              const float* table, const float* tau, float* out, float* lse, unsigned int* vmax,
                              void* stream) {
    WAArgs a{};
    int HD = 0;
    int rc = fill_args(d, a, HD);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && table && out && lse, "wattn_fwd: null pointer");
    MMNI_ARG_CHECK(d->kind == 0 || tau != nullptr, "wattn_fwd: kind 1 needs tau");
    MMNI_ARG_CHECK(row_aligned(q, d->q_stride, d->C) && row_aligned(k, d->k_stride, d->C) &&
                       row_aligned(v, d->v_stride, d->C) && row_aligned(out, d->o_stride, d->C),
                   "wattn_fwd: q/k/v/out must be 16-byte aligned with strides multiple of 4");
    if (wattn_bc_supported(a.g, d->C, d->heads, d->kind)) {   // 6^3 kind 0 head pairs: row-broadcast kernel
        a.q = q; a.k = k; a.v = v; a.table = table; a.tau = table; a.out = out; a.lse = lse; a.vmax = vmax;
        return wattn_bc_forward(a, d->heads, (hipStream_t)stream);
    }
    void *kf, *kb;
    int maxt;
    bool packed = false;
    int qpl = 1;
    const int hs = head_split(a.g, d->C, d->heads, HD);
    rc = dispatch(d, d->C / hs, HD, false, kf, kb, maxt, packed, qpl);
    if (rc) return rc;
    WAConfig cfg;
    rc = plan(a.g, d->C / hs, d->heads / hs, maxt, false, packed, cfg, qpl, hs);
    if (rc) return rc;
    a.KS = cfg.KS; a.WPB = cfg.WPB; a.NPAD = cfg.NPAD; a.ngroups = cfg.ngroups;
    a.q = q; a.k = k; a.v = v; a.table = table; a.tau = tau ? tau : table; a.out = out; a.lse = lse;
    a.vmax = packed ? vmax : nullptr;   // the packed kernels fold max|v| into their K/V staging
    a.hsplit = hs;
    rc = ensure_lds_attr(kf, cfg.lds);
    if (rc) return rc;
    void* args[] = {&a};
    hipError_t e = hipLaunchKernel(kf, dim3(cfg.grid, hs), dim3(cfg.threads), args, cfg.lds, (hipStream_t)stream);
    if (e != hipSuccess) { set_error("wattn_fwd launch: %s", hipGetErrorString(e)); return (int)e; }
    if (vmax && !packed) {   // generic kernels: a separate pass over v (vmax is maxbits[1]-shaped: pass vmax - 1)
        const long long T = (long long)a.g.nwin * a.g.N;
        wattn_absmax_kernel<<<absmax_blocks(T, d->C), 256, 0, (hipStream_t)stream>>>(nullptr, 0, v, d->v_stride, T, d->C,
                                                                               vmax - 1);
        return launch_status("wattn_absmax_v");
    }
    return 0;
}

extern "C" size_t mmni_wattn_bwd_workspace_bytes(const mmni_wattn_desc* d) {
    WGeom g;
    if (make_geom(d, g)) return 0;
    // fixed-point table gradient + the two absmax words + the dtau partial rows (kind 1)
    const size_t fixed = (size_t)g.Tsz * d->heads * sizeof(unsigned long long) + 16 +
                         (size_t)kMaxBwdBlocks * d->heads * sizeof(float);
    if (d->heads > 0 && wattn_bc_supported(g, d->C, d->heads, d->kind)) {
        const size_t b = wattn_bc_workspace_bytes(g, d->heads);
        return b > fixed ? b : fixed;
    }
    return fixed;
}

extern "C" int mmni_wattn_bwd(const mmni_wattn_desc* d, const float* q, const float* k, const float* v,
                              const float* table, const float* tau, const float* out, const float* dout,
                              const float* lse, float* dq, float* dk, float* dv, float* dtable, float* dtau,
                              void* workspace, const unsigned int* vmax, void* stream) {
    WAArgs a{};
    int HD = 0;
    int rc = fill_args(d, a, HD);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && table && out && dout && lse && dq && dk && dv && dtable && workspace,
                   "wattn_bwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(workspace) % 8 == 0, "wattn_bwd: workspace must be 8-byte aligned");
    MMNI_ARG_CHECK(d->kind == 0 || (tau != nullptr && dtau != nullptr), "wattn_bwd: kind 1 needs tau and dtau");
    MMNI_ARG_CHECK(row_aligned(q, d->q_stride, d->C) && row_aligned(k, d->k_stride, d->C) &&
                       row_aligned(v, d->v_stride, d->C) && row_aligned(out, d->o_stride, d->C) &&
                       row_aligned(dout, d->o_stride, d->C) && row_aligned(dq, d->q_stride, d->C) &&
                       row_aligned(dk, d->k_stride, d->C) && row_aligned(dv, d->v_stride, d->C),
                   "wattn_bwd: tensors must be 16-byte aligned with strides multiple of 4");
    if (wattn_bc_supported(a.g, d->C, d->heads, d->kind)) {   // 64-bit row addressing: any token count
        a.q = q; a.k = k; a.v = v; a.table = table; a.tau = table; a.lse = const_cast<float*>(lse);
        a.o = out; a.dout = dout; a.dq = dq; a.dk = dk; a.dv = dv; a.dtable = dtable; a.dtau = dtable;
        return wattn_bc_backward(a, d->heads, dtable, workspace, (hipStream_t)stream);
    }
    void *kf, *kb;
    int maxt;
    bool packed = false;
    int qpl = 1;
    const int hs = head_split(a.g, d->C, d->heads, HD);
    rc = dispatch(d, d->C / hs, HD, true, kf, kb, maxt, packed, qpl);
    if (rc) return rc;
    WAConfig cfg;
    rc = plan(a.g, d->C / hs, d->heads / hs, maxt, true, packed, cfg, qpl, hs);
    if (rc) return rc;
    a.hsplit = hs;
    a.KS = cfg.KS; a.WPB = cfg.WPB; a.NPAD = cfg.NPAD; a.ngroups = cfg.ngroups;
    a.q = q; a.k = k; a.v = v; a.table = table; a.tau = tau ? tau : table; a.lse = const_cast<float*>(lse);
    a.o = out; a.dout = dout; a.dq = dq; a.dk = dk; a.dv = dv; a.dtable = dtable; a.dtau = dtau ? dtau : dtable;
    a.dtab_fix = reinterpret_cast<unsigned long long*>(workspace);
    a.fix_shift = 0;
    rc = ensure_lds_attr(kb, cfg.lds);
    if (rc) return rc;
    const int ntab = a.g.Tsz * d->heads;
    a.maxbits = reinterpret_cast<unsigned int*>(a.dtab_fix + ntab);
    a.dtau_part = reinterpret_cast<float*>(a.maxbits + 4);
    MMNI_ARG_CHECK(cfg.grid <= kMaxBwdBlocks, "wattn_bwd: grid %d exceeds the dtau partial rows", cfg.grid);
    hipError_t e = hipMemsetAsync(workspace, 0, (size_t)ntab * 8 + 16, (hipStream_t)stream);
    if (e != hipSuccess) { set_error("wattn_bwd memset: %s", hipGetErrorString(e)); return (int)e; }
    const long long T = (long long)a.g.nwin * a.g.N;   // tokens
    if (vmax && d->o_stride == d->C && d->C % 4 == 0 && reinterpret_cast<uintptr_t>(dout) % 16 == 0) {
        const long long n4 = T * d->C / 4;
        long long blocks = (n4 + 1023) / 1024;
        if (blocks > 512) blocks = 512;
        wattn_absmax_dout4_kernel<<<(unsigned)blocks, 1024, 0, (hipStream_t)stream>>>(
            reinterpret_cast<const float4*>(dout), n4, vmax, a.maxbits);
    } else {
        wattn_absmax_kernel<<<absmax_blocks(T, d->C), 256, 0, (hipStream_t)stream>>>(dout, d->o_stride, v, d->v_stride, T,
                                                                               d->C, a.maxbits);
    }
    rc = launch_status("wattn_absmax");
    if (rc) return rc;
    void* args[] = {&a};
    e = hipLaunchKernel(kb, dim3(cfg.grid, hs), dim3(cfg.threads), args, cfg.lds, (hipStream_t)stream);
    if (e != hipSuccess) { set_error("wattn_bwd launch: %s", hipGetErrorString(e)); return (int)e; }
    wattn_dtable_convert_kernel<<<(ntab + 255) / 256, 256, 0, (hipStream_t)stream>>>(a.dtab_fix, a.maxbits, HD,
                                                                                     a.fix_shift, dtable, ntab);
    rc = launch_status("wattn_dtable_convert");
    if (rc || d->kind != 1) return rc;
    ColSegs segs{};   // dtau += the fixed-order column sums of the blocks' partial rows
    segs.n = 1;
    segs.end[0] = d->heads;
    segs.dst[0] = dtau;
    segs.accumulate = 1;
    column_sum_segs(a.dtau_part, cfg.grid, d->heads, segs, (hipStream_t)stream);
    return launch_status("wattn_dtau_sum");
}

extern "C" int mmni_window_rows(const mmni_wattn_desc* d, int32_t* rows, void* stream) {
    WGeom g;
    int rc = make_geom(d, g);
    if (rc) return rc;
    MMNI_ARG_CHECK(rows != nullptr, "window_rows: null pointer");
    const int64_t n = (int64_t)g.nwin * g.N;
    window_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(g, rows);
    return launch_status("window_rows");
}

extern "C" int mmni_window_mask(const mmni_wattn_desc* d, float* mask, void* stream) {
    WGeom g;
    int rc = make_geom(d, g);
    if (rc) return rc;
    MMNI_ARG_CHECK(mask != nullptr, "window_mask: null pointer");
    const int nWs = g.nWd * g.nWh * g.nWw;
    const int64_t n = (int64_t)nWs * g.N * g.N;
    window_mask_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(g, nWs, mask);
    return launch_status("window_mask");
}

extern "C" int mmni_relative_index(const mmni_wattn_desc* d, int32_t* idx, void* stream) {
    WGeom g;
    int rc = make_geom(d, g);
    if (rc) return rc;
    MMNI_ARG_CHECK(idx != nullptr, "relative_index: null pointer");
    relative_index_kernel<<<(g.N * g.N + 255) / 256, 256, 0, (hipStream_t)stream>>>(g, idx);
    return launch_status("relative_index");
}
