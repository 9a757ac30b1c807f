// Crossmodal multi-head attention core for gfx950.
//
// Replaces the bmm -> (+causal mask) -> fp32 softmax -> bmm section of
//   MultiheadAttention.forward   modules/multihead_attention.py:95-130
// with buffered_future_mask      modules/crossmodal_transformer.py:179-186
// (mask = -inf where key - query >= causal_diag = 1 + |Tk - Tq|).
// The in_proj / out_proj GEMMs stay on hipBLASLt through torch.
//
// Layout: time-major (T, B, E) exactly as the reference passes it, read in place —
// element (t, b, head, c) at ptr[(t*B + b)*stride + head*hd + c] — so the reference's
// .view(T, B*h, d).transpose(0,1) copies (multihead_attention.py:92-96) never happen.
//
// Structure (this round): flash-style, fp32 on the VALU.  KS adjacent lanes own one query
// row and split every K/V tile's keys; K/V tiles of KT keys are staged in LDS; the online
// softmax runs in the log2 domain over chunks of 4 keys; causal tiles past the diagonal are
// skipped.  Backward: a delta = rowsum(dO*O) kernel, a dq kernel (lane = query row) and a
// dk/dv kernel (lane = key row) — no atomics, deterministic.
#include "mmni_common.h"

namespace mmni {

struct MhaArgs {
    int Tq, Tk, B, H, causal;   // causal: diag (<=0 none)
    float scale2;               // scale * log2(e)
    float scale;
    int64_t qs, ks, vs, os;
    const float* q;
    const float* k;
    const float* v;
    float* out;
    float* lse;                 // (B, H, Tq) natural log
    const float* o;
    const float* dout;
    float* dq;
    float* dk;
    float* dv;
    float* delta;               // (B, H, Tq)
    float* probs;               // (B, Tq, Tk)
};

constexpr int MHA_KT = 64;      // keys per LDS tile
constexpr int MHA_KS = 4;       // lanes per query row
constexpr int MHA_ROWS = 64;    // query rows per block (threads = ROWS*KS = 256)
constexpr int MHA_CH = 4;

template <int HD>
__device__ __forceinline__ void ld(float (&d)[HD], const float* s) {
#pragma unroll
    for (int c = 0; c < HD; ++c) d[c] = s[c];
}

// key limit (exclusive) for query row i under the causal mask
__device__ __forceinline__ int key_end(const MhaArgs& a, int i) {
    if (a.causal <= 0) return a.Tk;
    const int e = i + a.causal;
    return e < a.Tk ? e : a.Tk;
}

template <int HD>
__global__ __launch_bounds__(256) void mha_fwd_kernel(MhaArgs a) {
    __shared__ __attribute__((aligned(16))) float ks_[MHA_KT * HD];
    __shared__ __attribute__((aligned(16))) float vs_[MHA_KT * HD];
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, r = tid / MHA_KS, p = tid % MHA_KS;
    const int i = blockIdx.x * MHA_ROWS + r;
    const bool active = i < a.Tq;
    float q[HD];
    if (active) ld<HD>(q, a.q + ((int64_t)i * a.B + b) * a.qs + h * HD);
    else for (int c = 0; c < HD; ++c) q[c] = 0.f;
#pragma unroll
    for (int c = 0; c < HD; ++c) q[c] *= a.scale2;
    const int kend_row = active ? key_end(a, i) : 0;
    const int i_last = min(a.Tq - 1, (int)blockIdx.x * MHA_ROWS + MHA_ROWS - 1);
    const int kend_blk = key_end(a, i_last);

    float m = -INFINITY, l = 0.f, acc[HD];
#pragma unroll
    for (int c = 0; c < HD; ++c) acc[c] = 0.f;

    for (int k0 = 0; k0 < kend_blk; k0 += MHA_KT) {
        __syncthreads();
        for (int e = tid; e < MHA_KT * HD; e += blockDim.x) {
            const int j = k0 + e / HD, c = e % HD;
            float kv = 0.f, vv = 0.f;
            if (j < a.Tk) {
                kv = a.k[((int64_t)j * a.B + b) * a.ks + h * HD + c];
                vv = a.v[((int64_t)j * a.B + b) * a.vs + h * HD + c];
            }
            ks_[e] = kv;
            vs_[e] = vv;
        }
        __syncthreads();
        for (int n = 0; n < MHA_KT / MHA_KS; n += MHA_CH) {
            float s[MHA_CH];
#pragma unroll
            for (int cc = 0; cc < MHA_CH; ++cc) {
                const int jl = p + MHA_KS * (n + cc);
                float d = 0.f;
#pragma unroll
                for (int c = 0; c < HD; ++c) d = fmaf(q[c], ks_[jl * HD + c], d);
                s[cc] = (k0 + jl < kend_row) ? d : -INFINITY;
            }
            float cm = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
            const float mn = fmaxf(m, cm);
            if (mn == -INFINITY) continue;   // nothing visible yet for this lane
            const float alpha = fast_exp2(m - mn);
            m = mn;
            l *= alpha;
#pragma unroll
            for (int c = 0; c < HD; ++c) acc[c] *= alpha;
#pragma unroll
            for (int cc = 0; cc < MHA_CH; ++cc) {
                const int jl = p + MHA_KS * (n + cc);
                const float pj = fast_exp2(s[cc] - m);
                l += pj;
#pragma unroll
                for (int c = 0; c < HD; ++c) acc[c] = fmaf(pj, vs_[jl * HD + c], acc[c]);
            }
        }
    }
#pragma unroll
    for (int o = 1; o < MHA_KS; o <<= 1) {
        const float mo = __shfl_xor(m, o), lo = __shfl_xor(l, o);
        const float mn = fmaxf(m, mo);
        const float fa = (m == -INFINITY) ? 0.f : fast_exp2(m - mn);
        const float fb = (mo == -INFINITY) ? 0.f : fast_exp2(mo - mn);
        l = l * fa + lo * fb;
#pragma unroll
        for (int c = 0; c < HD; ++c) acc[c] = acc[c] * fa + __shfl_xor(acc[c], o) * fb;
        m = mn;
    }
    if (active && p == 0) {
        const float inv = 1.0f / l;
        float* o = a.out + ((int64_t)i * a.B + b) * a.os + h * HD;
#pragma unroll
        for (int c = 0; c < HD; ++c) o[c] = acc[c] * inv;
        a.lse[((int64_t)b * a.H + h) * a.Tq + i] = (m + fast_log2(l)) * kLn2;
    }
}

template <int HD>
__global__ __launch_bounds__(256) void mha_delta_kernel(MhaArgs a) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (i, b, h)
    if (e >= (int64_t)a.Tq * a.B * a.H) return;
    const int h = (int)(e % a.H);
    const int64_t ib = e / a.H;
    const int b = (int)(ib % a.B), i = (int)(ib / a.B);
    const float* o = a.o + ib * a.os + h * HD;
    const float* g = a.dout + ib * a.os + h * HD;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < HD; ++c) d = fmaf(o[c], g[c], d);
    a.delta[((int64_t)b * a.H + h) * a.Tq + i] = d;
}

// dq: lane group = query row, loops over key tiles.
template <int HD>
__global__ __launch_bounds__(256) void mha_bwd_dq_kernel(MhaArgs a) {
    __shared__ __attribute__((aligned(16))) float ks_[MHA_KT * HD];
    __shared__ __attribute__((aligned(16))) float vs_[MHA_KT * HD];
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, r = tid / MHA_KS, p = tid % MHA_KS;
    const int i = blockIdx.x * MHA_ROWS + r;
    const bool active = i < a.Tq;
    float q[HD], g[HD], dqa[HD];
    float lse2 = INFINITY, dl = 0.f;
    if (active) {
        const int64_t ib = (int64_t)i * a.B + b;
        ld<HD>(q, a.q + ib * a.qs + h * HD);
        ld<HD>(g, a.dout + ib * a.os + h * HD);
        lse2 = a.lse[((int64_t)b * a.H + h) * a.Tq + i] * kLog2e;
        dl = a.delta[((int64_t)b * a.H + h) * a.Tq + i];
    } else {
        for (int c = 0; c < HD; ++c) { q[c] = 0.f; g[c] = 0.f; }
    }
#pragma unroll
    for (int c = 0; c < HD; ++c) { q[c] *= a.scale2; dqa[c] = 0.f; }
    const int kend_row = active ? key_end(a, i) : 0;
    const int i_last = min(a.Tq - 1, (int)blockIdx.x * MHA_ROWS + MHA_ROWS - 1);
    const int kend_blk = key_end(a, i_last);
    for (int k0 = 0; k0 < kend_blk; k0 += MHA_KT) {
        __syncthreads();
        for (int e = tid; e < MHA_KT * HD; e += blockDim.x) {
            const int j = k0 + e / HD, c = e % HD;
            float kv = 0.f, vv = 0.f;
            if (j < a.Tk) {
                kv = a.k[((int64_t)j * a.B + b) * a.ks + h * HD + c];
                vv = a.v[((int64_t)j * a.B + b) * a.vs + h * HD + c];
            }
            ks_[e] = kv;
            vs_[e] = vv;
        }
        __syncthreads();
        for (int n = 0; n < MHA_KT / MHA_KS; ++n) {
            const int jl = p + MHA_KS * n;
            float s = 0.f, dp = 0.f;
#pragma unroll
            for (int c = 0; c < HD; ++c) {
                s = fmaf(q[c], ks_[jl * HD + c], s);
                dp = fmaf(g[c], vs_[jl * HD + c], dp);
            }
            const float pr = (k0 + jl < kend_row) ? fast_exp2(s - lse2) : 0.f;
            const float ds = pr * (dp - dl);
#pragma unroll
            for (int c = 0; c < HD; ++c) dqa[c] = fmaf(ds, ks_[jl * HD + c], dqa[c]);
        }
    }
#pragma unroll
    for (int o = 1; o < MHA_KS; o <<= 1)
#pragma unroll
        for (int c = 0; c < HD; ++c) dqa[c] += __shfl_xor(dqa[c], o);
    if (active && p == 0) {
        float* d = a.dq + ((int64_t)i * a.B + b) * a.qs + h * HD;
#pragma unroll
        for (int c = 0; c < HD; ++c) d[c] = dqa[c] * a.scale;
    }
}

// dk, dv: lane group = key row, loops over query tiles.
template <int HD>
__global__ __launch_bounds__(256) void mha_bwd_dkv_kernel(MhaArgs a) {
    __shared__ __attribute__((aligned(16))) float qs_[MHA_KT * HD];
    __shared__ __attribute__((aligned(16))) float gs_[MHA_KT * HD];
    __shared__ float ls_[MHA_KT];
    __shared__ float ds_[MHA_KT];
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, r = tid / MHA_KS, p = tid % MHA_KS;
    const int j = blockIdx.x * MHA_ROWS + r;
    const bool active = j < a.Tk;
    float kr[HD], vr[HD], dka[HD], dva[HD];
    if (active) {
        ld<HD>(kr, a.k + ((int64_t)j * a.B + b) * a.ks + h * HD);
        ld<HD>(vr, a.v + ((int64_t)j * a.B + b) * a.vs + h * HD);
    } else {
        for (int c = 0; c < HD; ++c) { kr[c] = 0.f; vr[c] = 0.f; }
    }
#pragma unroll
    for (int c = 0; c < HD; ++c) { dka[c] = 0.f; dva[c] = 0.f; }
    // first query that can see key j: j - i < diag  <=>  i > j - diag
    const int j_first = (int)blockIdx.x * MHA_ROWS;
    int q_begin = 0;
    if (a.causal > 0) q_begin = max(0, j_first - a.causal + 1);
    q_begin = q_begin / MHA_KT * MHA_KT;
    for (int i0 = q_begin; i0 < a.Tq; i0 += MHA_KT) {
        __syncthreads();
        for (int e = tid; e < MHA_KT * HD; e += blockDim.x) {
            const int i = i0 + e / HD, c = e % HD;
            float qv = 0.f, gv = 0.f;
            if (i < a.Tq) {
                qv = a.q[((int64_t)i * a.B + b) * a.qs + h * HD + c] * a.scale2;
                gv = a.dout[((int64_t)i * a.B + b) * a.os + h * HD + c];
            }
            qs_[e] = qv;
            gs_[e] = gv;
        }
        for (int e = tid; e < MHA_KT; e += blockDim.x) {
            const int i = i0 + e;
            ls_[e] = (i < a.Tq) ? a.lse[((int64_t)b * a.H + h) * a.Tq + i] * kLog2e : INFINITY;
            ds_[e] = (i < a.Tq) ? a.delta[((int64_t)b * a.H + h) * a.Tq + i] : 0.f;
        }
        __syncthreads();
        for (int n = 0; n < MHA_KT / MHA_KS; ++n) {
            const int il = p + MHA_KS * n;
            const int i = i0 + il;
            float s = 0.f, dp = 0.f;
#pragma unroll
            for (int c = 0; c < HD; ++c) {
                s = fmaf(qs_[il * HD + c], kr[c], s);
                dp = fmaf(gs_[il * HD + c], vr[c], dp);
            }
            const bool vis = active && (a.causal <= 0 || j - i < a.causal);
            const float pr = vis ? fast_exp2(s - ls_[il]) : 0.f;
            const float dsv = pr * (dp - ds_[il]);
#pragma unroll
            for (int c = 0; c < HD; ++c) {
                dva[c] = fmaf(pr, gs_[il * HD + c], dva[c]);
                dka[c] = fmaf(dsv, qs_[il * HD + c], dka[c]);
            }
        }
    }
#pragma unroll
    for (int o = 1; o < MHA_KS; o <<= 1)
#pragma unroll
        for (int c = 0; c < HD; ++c) {
            dka[c] += __shfl_xor(dka[c], o);
            dva[c] += __shfl_xor(dva[c], o);
        }
    if (active && p == 0) {
        float* dk = a.dk + ((int64_t)j * a.B + b) * a.ks + h * HD;
        float* dv = a.dv + ((int64_t)j * a.B + b) * a.vs + h * HD;
        // qs_ held q * scale * log2e: ds/dk = scale*q  ->  multiply by ln2
#pragma unroll
        for (int c = 0; c < HD; ++c) { dk[c] = dka[c] * kLn2; dv[c] = dva[c]; }
    }
}

// head-averaged probabilities: probs[b, i, j] = mean_h softmax_j(...)
template <int HD>
__global__ __launch_bounds__(256) void mha_probs_kernel(MhaArgs a) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (b, i, j)
    if (e >= (int64_t)a.B * a.Tq * a.Tk) return;
    const int j = (int)(e % a.Tk);
    const int64_t bi = e / a.Tk;
    const int i = (int)(bi % a.Tq), b = (int)(bi / a.Tq);
    float sum = 0.f;
    const bool vis = a.causal <= 0 || j - i < a.causal;
    if (vis) {
        for (int h = 0; h < a.H; ++h) {
            const float* q = a.q + ((int64_t)i * a.B + b) * a.qs + h * HD;
            const float* k = a.k + ((int64_t)j * a.B + b) * a.ks + h * HD;
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < HD; ++c) s = fmaf(q[c], k[c], s);
            sum += fast_exp2(s * a.scale2 - a.lse[((int64_t)b * a.H + h) * a.Tq + i] * kLog2e);
        }
    }
    a.probs[e] = sum / (float)a.H;
}

static int mha_fill(const mmni_mha_desc* d, MhaArgs& a) {
    MMNI_ARG_CHECK(d != nullptr, "mha: null descriptor");
    MMNI_ARG_CHECK(d->Tq > 0 && d->Tk > 0 && d->B > 0 && d->heads > 0 && d->head_dim > 0, "mha: bad sizes");
    const int E = d->heads * d->head_dim;
    MMNI_ARG_CHECK(d->q_stride >= E && d->k_stride >= E && d->v_stride >= E && d->o_stride >= E,
                   "mha: strides must be >= heads*head_dim");
    MMNI_ARG_CHECK((int64_t)d->B * d->heads <= 65535, "mha: B*heads exceeds the grid y limit");
    a.Tq = d->Tq; a.Tk = d->Tk; a.B = d->B; a.H = d->heads; a.causal = d->causal_diag;
    a.scale = d->scale;
    a.scale2 = d->scale * kLog2e;
    a.qs = d->q_stride; a.ks = d->k_stride; a.vs = d->v_stride; a.os = d->o_stride;
    return 0;
}

template <int HD>
static int mha_fwd_launch(MhaArgs& a, hipStream_t s) {
    dim3 grid((a.Tq + MHA_ROWS - 1) / MHA_ROWS, a.B * a.H);
    mha_fwd_kernel<HD><<<grid, MHA_ROWS * MHA_KS, 0, s>>>(a);
    return launch_status("mha_fwd");
}

template <int HD>
static int mha_bwd_launch(MhaArgs& a, hipStream_t s) {
    const int64_t n = (int64_t)a.Tq * a.B * a.H;
    mha_delta_kernel<HD><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
    int rc = launch_status("mha_delta");
    if (rc) return rc;
    dim3 gq((a.Tq + MHA_ROWS - 1) / MHA_ROWS, a.B * a.H);
    mha_bwd_dq_kernel<HD><<<gq, MHA_ROWS * MHA_KS, 0, s>>>(a);
    rc = launch_status("mha_bwd_dq");
    if (rc) return rc;
    dim3 gk((a.Tk + MHA_ROWS - 1) / MHA_ROWS, a.B * a.H);
    mha_bwd_dkv_kernel<HD><<<gk, MHA_ROWS * MHA_KS, 0, s>>>(a);
    return launch_status("mha_bwd_dkv");
}

template <int HD>
static int mha_probs_launch(MhaArgs& a, hipStream_t s) {
    const int64_t n = (int64_t)a.B * a.Tq * a.Tk;
    mha_probs_kernel<HD><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
    return launch_status("mha_probs");
}

#define MMNI_MHA_DISPATCH(FN, HDV)                                                        \
    switch (HDV) {                                                                        \
        case 2: return FN<2>(a, (hipStream_t)stream);                                     \
        case 4: return FN<4>(a, (hipStream_t)stream);                                     \
        case 7: return FN<7>(a, (hipStream_t)stream);                                     \
        case 8: return FN<8>(a, (hipStream_t)stream);                                     \
        case 14: return FN<14>(a, (hipStream_t)stream);                                   \
        case 16: return FN<16>(a, (hipStream_t)stream);                                   \
        default:                                                                          \
            set_error("mha: unsupported head_dim %d (supported 2,4,7,8,14,16)", HDV);      \
            return -2;                                                                    \
    }

}  // namespace mmni

using namespace mmni;

extern "C" int mmni_mha_fwd(const mmni_mha_desc* d, const float* q, const float* k, const float* v,
                            float* out, float* lse, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && out && lse, "mha_fwd: null pointer");
    a.q = q; a.k = k; a.v = v; a.out = out; a.lse = lse;
    MMNI_MHA_DISPATCH(mha_fwd_launch, d->head_dim)
}

extern "C" int mmni_mha_bwd(const mmni_mha_desc* d, const float* q, const float* k, const float* v,
                            const float* out, const float* dout, const float* lse, float* dq, float* dk,
                            float* dv, float* workspace, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && out && dout && lse && dq && dk && dv && workspace, "mha_bwd: null pointer");
    a.q = q; a.k = k; a.v = v; a.o = out; a.dout = dout; a.lse = const_cast<float*>(lse);
    a.dq = dq; a.dk = dk; a.dv = dv; a.delta = workspace;
    MMNI_MHA_DISPATCH(mha_bwd_launch, d->head_dim)
}

extern "C" int mmni_mha_mean_probs(const mmni_mha_desc* d, const float* q, const float* k, const float* lse,
                                   float* probs, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && lse && probs, "mha_mean_probs: null pointer");
    a.q = q; a.k = k; a.lse = const_cast<float*>(lse); a.probs = probs;
    MMNI_MHA_DISPATCH(mha_probs_launch, d->head_dim)
}
