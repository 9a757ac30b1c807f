// Crossmodal multi-head attention core for gfx950.
//
// Replaces the bmm -> (+causal mask) -> fp32 softmax -> dropout -> bmm section of
//   MultiheadAttention.forward   modules/multihead_attention.py:109-125
// with buffered_future_mask      modules/crossmodal_transformer.py:179-186
// (mask = -inf where key - query >= causal_diag = 1 + |Tk - Tq|).
// The in_proj / out_proj GEMMs stay on hipBLASLt through torch.
//
// Layout: time-major (T, B, E) exactly as the reference passes it, read in place — element
// (t, b, head, c) at ptr[(t*B + b)*stride + head*hd + c] — so the reference's
// .view(T, B*h, d).transpose(0,1) copies (multihead_attention.py:92-96) never happen.
//
// Contractions on the f32 matrix cores (v_mfma_f32_16x16x4_f32; exact fp32, the same 157 TF as
// the packed VALU, so the VALU stays free for the softmax).  head_dim d is padded to HDP = 4, 8
// or 16 (7 -> 8, 14 -> 16; padding lanes read zeros).  One wave owns 16 rows; K/V (or Q/dO) tiles
// of 64 rows are staged in LDS and consumed as 4 sub-tiles of 16.
//   forward   S^T(16 keys x 16 queries) = K Q^T        (HDP/4 MFMAs per sub-tile)
//             O^T(d x 16 queries)     += V^T P^T       (4 MFMAs per sub-tile; P^T is the S^T
//                                                      accumulator itself: C/D rows = keys = the
//                                                      B operand's k index, no data movement)
//   dq        S^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T
//   dk, dv    S = Q K^T, dP = dO V^T, dS, dV^T += dO^T P, dK^T += Q^T dS
// Online softmax in the log2 domain: each lane holds 4 keys of one query per sub-tile; the row
// max is two cross-lane shuffles per 64 keys, the row sum stays a per-lane partial until the end.
// Causal tiles past a wave's diagonal are skipped.  No atomics: deterministic.
//
// Attention dropout (multihead_attention.py:123, F.dropout on the probabilities, reference default
// --attn_dropout 0.1, main.py:176): counter-based, keep(b*h, i, j) = hash(seed, (b*h)*Tq + i, j)
// < (1 - p) * 2^32, regenerated identically in the backward and by mmni_mha_dropout_mask.
#include "mmni_common.h"

namespace mmni {

typedef float mf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ mf4 mfma4(float a, float b, mf4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct MhaArgs {
    int Tq, Tk, B, H, hd, causal;   // causal: diag (<=0 none)
    float scale;
    float scale2;                   // scale * log2(e)
    int64_t qs, ks, vs, os;
    const float* q;
    const float* k;
    const float* v;
    float* out;
    float* lse;                     // (B, H, Tq) natural log
    const float* o;
    const float* dout;
    float* dq;
    float* dk;
    float* dv;
    float* delta;                   // (B, H, Tq)
    float* probs;                   // (B, Tq, Tk)
    float inv_keep;                 // 1 / (1 - p)
    uint32_t thresh;                // keep iff hash < thresh
    uint32_t seed;
};

constexpr int MT = 64;      // rows per LDS tile and per workgroup (4 waves x 16)
constexpr int VST = 20;     // row stride of the tiles read as [row 4g+i][col lane&15] (conflict-free halves)

// ---- dropout hash (lowbias32 mixer, two rounds keyed by row then column)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t drop_row(uint32_t seed, int bh, int Tq, int i) {
    return mix32(seed ^ mix32((uint32_t)(bh * Tq + i) * 0x9e3779b9U + 0x632be5abU));
}
__device__ __forceinline__ bool drop_keep(uint32_t rowh, int j, uint32_t thresh) {
    return mix32(rowh + (uint32_t)j * 0x85ebca6bU) < thresh;
}

// key limit (exclusive) for query row i under the causal mask
__device__ __forceinline__ int key_end(const MhaArgs& a, int i) {
    if (a.causal <= 0) return a.Tk;
    const int e = i + a.causal;
    return e < a.Tk ? e : a.Tk;
}

__device__ __forceinline__ float load_pad(const float* base, int64_t rowoff, int c, int hd, bool ok) {
    return (ok && c < hd) ? base[rowoff + c] : 0.f;
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int HDP, bool DROP>
__global__ __launch_bounds__(256) void mha_fwd_mfma_kernel(MhaArgs a) {
    constexpr int KST = HDP + 1;   // K tile row stride (read as [lane&15][4dc + lane>>4])
    __shared__ float ks_[MT * KST + 16];
    __shared__ float vs_[MT * VST + 16];
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int q0 = blockIdx.x * MT + wave * 16;
    const int qi = q0 + ln;
    const bool qok = qi < a.Tq;
    float qb[HDP / 4];
#pragma unroll
    for (int dc = 0; dc < HDP / 4; ++dc)
        qb[dc] = load_pad(a.q, ((int64_t)qi * a.B + b) * a.qs + h * a.hd, 4 * dc + lg, a.hd, qok) * a.scale2;
    const uint32_t rowh = DROP ? drop_row(a.seed, bh, a.Tq, qi) : 0u;
    mf4 o = {0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    const int kend_blk = key_end(a, min(a.Tq - 1, (int)blockIdx.x * MT + MT - 1));
    const int kend_w = q0 < a.Tq ? key_end(a, min(a.Tq - 1, q0 + 15)) : 0;
    for (int k0 = 0; k0 < kend_blk; k0 += MT) {
        __syncthreads();
        for (int e = tid; e < MT * HDP; e += 256) {
            const int r = e / HDP, c = e - r * HDP, j = k0 + r;
            const bool ok = j < a.Tk;
            ks_[r * KST + c] = load_pad(a.k, ((int64_t)j * a.B + b) * a.ks + h * a.hd, c, a.hd, ok);
            vs_[r * VST + c] = load_pad(a.v, ((int64_t)j * a.B + b) * a.vs + h * a.hd, c, a.hd, ok);
        }
        __syncthreads();
        if (k0 >= kend_w) continue;   // wave-uniform: every key of the tile is masked for this wave
        mf4 s[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            s[st] = (mf4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dc = 0; dc < HDP / 4; ++dc) s[st] = mfma4(ks_[(16 * st + ln) * KST + 4 * dc + lg], qb[dc], s[st]);
        }
        // lane: s[st][i] = S^T[key k0 + 16 st + 4 lg + i][query qi] (log2 domain)
        const bool edge = (k0 + MT > a.Tk) || (a.causal > 0 && k0 + MT > q0 + a.causal);
        if (edge) {
#pragma unroll
            for (int st = 0; st < 4; ++st)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int j = k0 + 16 * st + 4 * lg + i;
                    if (j >= a.Tk || (a.causal > 0 && j - qi >= a.causal)) s[st][i] = -INFINITY;
                }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[st][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mn = fmaxf(m, mx);
        const float ms = mn == -INFINITY ? 0.f : mn;   // no visible key yet: every p below is 0
        const float alpha = fast_exp2(m - ms);
        m = mn;
        lsum *= alpha;
        o *= alpha;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = fast_exp2(s[st][i] - ms);
                lsum += p;
                float pv = p;
                if (DROP) pv = drop_keep(rowh, k0 + 16 * st + 4 * lg + i, a.thresh) ? p * a.inv_keep : 0.f;
                s[st][i] = pv;
            }
        }
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) o = mfma4(vs_[(16 * st + 4 * lg + i) * VST + ln], s[st][i], o);
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    if (qok) {
        const float inv = 1.0f / lsum;
        float* orow = a.out + ((int64_t)qi * a.B + b) * a.os + h * a.hd;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = 4 * lg + i;
            if (d < a.hd) orow[d] = o[i] * inv;
        }
        if (lg == 0) a.lse[(int64_t)bh * a.Tq + qi] = (m + fast_log2(lsum)) * kLn2;
    }
}

// delta = rowsum(dO * O) per (b, h, i): with dropout O is the dropped output, which is exactly
// the p-weighted mean of the dropped-probability gradient the backward needs
__global__ __launch_bounds__(256) void mha_delta_kernel(MhaArgs a) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (i, b, h)
    if (e >= (int64_t)a.Tq * a.B * a.H) return;
    const int h = (int)(e % a.H);
    const int64_t ib = e / a.H;
    const int b = (int)(ib % a.B), i = (int)(ib / a.B);
    const float* o = a.o + ib * a.os + h * a.hd;
    const float* g = a.dout + ib * a.os + h * a.hd;
    float d = 0.f;
    for (int c = 0; c < a.hd; ++c) d = fmaf(o[c], g[c], d);
    a.delta[((int64_t)b * a.H + h) * a.Tq + i] = d;
}

// ------------------------------------------------------------------------------------
// dq: wave = 16 queries, loops over key tiles
// ------------------------------------------------------------------------------------
template <int HDP, bool DROP>
__global__ __launch_bounds__(256) void mha_dq_mfma_kernel(MhaArgs a) {
    constexpr int KST = HDP + 1;
    __shared__ float ks_[MT * KST + 16];   // read as A[key][d] (S^T) and as A[d = lane&15][key] (dQ^T)
    __shared__ float vs_[MT * KST + 16];   // read as A[key][d] (dP^T)
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int q0 = blockIdx.x * MT + wave * 16;
    const int qi = q0 + ln;
    const bool qok = qi < a.Tq;
    float qb[HDP / 4], gb[HDP / 4];
    const int64_t rq = ((int64_t)qi * a.B + b) * a.qs + h * a.hd, ro = ((int64_t)qi * a.B + b) * a.os + h * a.hd;
#pragma unroll
    for (int dc = 0; dc < HDP / 4; ++dc) {
        qb[dc] = load_pad(a.q, rq, 4 * dc + lg, a.hd, qok) * a.scale2;
        gb[dc] = load_pad(a.dout, ro, 4 * dc + lg, a.hd, qok);
    }
    const float lse2 = qok ? a.lse[(int64_t)bh * a.Tq + qi] * kLog2e : INFINITY;
    const float dl = qok ? a.delta[(int64_t)bh * a.Tq + qi] : 0.f;
    const uint32_t rowh = DROP ? drop_row(a.seed, bh, a.Tq, qi) : 0u;
    mf4 dq = {0.f, 0.f, 0.f, 0.f};
    const int kend_blk = key_end(a, min(a.Tq - 1, (int)blockIdx.x * MT + MT - 1));
    const int kend_w = q0 < a.Tq ? key_end(a, min(a.Tq - 1, q0 + 15)) : 0;
    for (int k0 = 0; k0 < kend_blk; k0 += MT) {
        __syncthreads();
        for (int e = tid; e < MT * HDP; e += 256) {
            const int r = e / HDP, c = e - r * HDP, j = k0 + r;
            const bool ok = j < a.Tk;
            ks_[r * KST + c] = load_pad(a.k, ((int64_t)j * a.B + b) * a.ks + h * a.hd, c, a.hd, ok);
            vs_[r * KST + c] = load_pad(a.v, ((int64_t)j * a.B + b) * a.vs + h * a.hd, c, a.hd, ok);
        }
        __syncthreads();
        if (k0 >= kend_w) continue;
        mf4 s[4], dp[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            s[st] = (mf4){0.f, 0.f, 0.f, 0.f};
            dp[st] = (mf4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dc = 0; dc < HDP / 4; ++dc) {
                s[st] = mfma4(ks_[(16 * st + ln) * KST + 4 * dc + lg], qb[dc], s[st]);
                dp[st] = mfma4(vs_[(16 * st + ln) * KST + 4 * dc + lg], gb[dc], dp[st]);
            }
        }
        const bool edge = (k0 + MT > a.Tk) || (a.causal > 0 && k0 + MT > q0 + a.causal);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = k0 + 16 * st + 4 * lg + i;
                float p = fast_exp2(s[st][i] - lse2);
                if (edge && (j >= a.Tk || (a.causal > 0 && j - qi >= a.causal))) p = 0.f;
                float g = dp[st][i];
                if (DROP) g = drop_keep(rowh, j, a.thresh) ? g * a.inv_keep : 0.f;
                s[st][i] = p * (g - dl);   // dS^T
            }
        }
        // dQ^T(d x queries) += K^T dS^T: A[m = d][k = key] = K[16 st + 4 lg + i][lane & 15]
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) dq = mfma4(ks_[(16 * st + 4 * lg + i) * KST + ln], s[st][i], dq);
    }
    if (qok) {
        float* drow = a.dq + rq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = 4 * lg + i;
            if (d < a.hd) drow[d] = dq[i] * a.scale;
        }
    }
}

// ------------------------------------------------------------------------------------
// dk, dv: wave = 16 keys, loops over query tiles
// ------------------------------------------------------------------------------------
template <int HDP, bool DROP>
__global__ __launch_bounds__(256) void mha_dkv_mfma_kernel(MhaArgs a) {
    constexpr int QST = 17;                // read as A[query][d] and as A[d = lane&15][query 4g+i]
    __shared__ float qs_[MT * QST + 16];   // q * scale * log2e
    __shared__ float gs_[MT * QST + 16];   // dO
    __shared__ float ls_[MT];              // lse2
    __shared__ float ds_[MT];              // delta
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int j0 = blockIdx.x * MT + wave * 16;
    const int kj = j0 + ln;
    const bool kok = kj < a.Tk;
    float kb[HDP / 4], vb[HDP / 4];
    const int64_t rk = ((int64_t)kj * a.B + b) * a.ks + h * a.hd, rv = ((int64_t)kj * a.B + b) * a.vs + h * a.hd;
#pragma unroll
    for (int dc = 0; dc < HDP / 4; ++dc) {
        kb[dc] = load_pad(a.k, rk, 4 * dc + lg, a.hd, kok);
        vb[dc] = load_pad(a.v, rv, 4 * dc + lg, a.hd, kok);
    }
    mf4 dk = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
    // first query that can see the block's first key: j - i < diag  <=>  i > j - diag
    int i_begin = 0;
    if (a.causal > 0) i_begin = max(0, (int)blockIdx.x * MT - a.causal + 1);
    i_begin = i_begin / MT * MT;
    const int ib_w = a.causal > 0 ? max(0, j0 - a.causal + 1) : 0;   // this wave's first visible query
    for (int i0 = i_begin; i0 < a.Tq; i0 += MT) {
        __syncthreads();
        for (int e = tid; e < MT * HDP; e += 256) {
            const int r = e / HDP, c = e - r * HDP, i = i0 + r;
            const bool ok = i < a.Tq;
            qs_[r * QST + c] = load_pad(a.q, ((int64_t)i * a.B + b) * a.qs + h * a.hd, c, a.hd, ok) * a.scale2;
            gs_[r * QST + c] = load_pad(a.dout, ((int64_t)i * a.B + b) * a.os + h * a.hd, c, a.hd, ok);
        }
        for (int e = tid; e < MT; e += 256) {
            const int i = i0 + e;
            ls_[e] = i < a.Tq ? a.lse[(int64_t)bh * a.Tq + i] * kLog2e : INFINITY;
            ds_[e] = i < a.Tq ? a.delta[(int64_t)bh * a.Tq + i] : 0.f;
        }
        __syncthreads();
        if (i0 + MT <= ib_w || j0 >= a.Tk) continue;   // wave-uniform: nothing visible
        mf4 s[4], dp[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            s[st] = (mf4){0.f, 0.f, 0.f, 0.f};
            dp[st] = (mf4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dc = 0; dc < HDP / 4; ++dc) {
                s[st] = mfma4(qs_[(16 * st + ln) * QST + 4 * dc + lg], kb[dc], s[st]);
                dp[st] = mfma4(gs_[(16 * st + ln) * QST + 4 * dc + lg], vb[dc], dp[st]);
            }
        }
        // lane: s[st][i] = S[query i0 + 16 st + 4 lg + i][key kj]
        const bool edge = (i0 + MT > a.Tq) || !kok || (a.causal > 0 && i0 < j0 + 16 - a.causal + 1);
        mf4 pd[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 16 * st + 4 * lg + i, qi = i0 + r;
                float p = fast_exp2(s[st][i] - ls_[r]);
                if (edge && (qi >= a.Tq || !kok || (a.causal > 0 && kj - qi >= a.causal))) p = 0.f;
                float g = dp[st][i], pv = p;
                if (DROP) {
                    const bool kp = drop_keep(drop_row(a.seed, bh, a.Tq, qi), kj, a.thresh);
                    g = kp ? g * a.inv_keep : 0.f;
                    pv = kp ? p * a.inv_keep : 0.f;
                }
                pd[st][i] = pv;
                s[st][i] = p * (g - ds_[r]);   // dS
            }
        }
        // dV^T(d x keys) += dO^T Pd, dK^T += Q2^T dS: A[m = d][k = query] = X[16 st + 4 lg + i][lane & 15]
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 16 * st + 4 * lg + i;
                dv = mfma4(gs_[r * QST + ln], pd[st][i], dv);
                dk = mfma4(qs_[r * QST + ln], s[st][i], dk);
            }
    }
    if (kok) {
        float* krow = a.dk + rk;
        float* vrow = a.dv + rv;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = 4 * lg + i;
            if (d < a.hd) {
                krow[d] = dk[i] * kLn2;   // staged q2 = q * scale * log2e
                vrow[d] = dv[i];
            }
        }
    }
}

// head-averaged (dropped) probabilities: probs[b, i, j] = mean_h keep * softmax_j(...) / (1 - p)
template <bool DROP>
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
            const float* q = a.q + ((int64_t)i * a.B + b) * a.qs + h * a.hd;
            const float* k = a.k + ((int64_t)j * a.B + b) * a.ks + h * a.hd;
            float s = 0.f;
            for (int c = 0; c < a.hd; ++c) s = fmaf(q[c], k[c], s);
            float p = fast_exp2(s * a.scale2 - a.lse[((int64_t)b * a.H + h) * a.Tq + i] * kLog2e);
            if (DROP) p = drop_keep(drop_row(a.seed, b * a.H + h, a.Tq, i), j, a.thresh) ? p * a.inv_keep : 0.f;
            sum += p;
        }
    }
    a.probs[e] = sum / (float)a.H;
}

// the dropout multipliers (0 or 1 / (1 - p)) of every (b, h, i, j), for tests
__global__ __launch_bounds__(256) void mha_dropout_mask_kernel(MhaArgs a, float* mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (bh, i, j)
    if (e >= (int64_t)a.B * a.H * a.Tq * a.Tk) return;
    const int j = (int)(e % a.Tk);
    const int64_t r = e / a.Tk;
    const int i = (int)(r % a.Tq), bh = (int)(r / a.Tq);
    mask[e] = drop_keep(drop_row(a.seed, bh, a.Tq, i), j, a.thresh) ? a.inv_keep : 0.f;
}

static int mha_fill(const mmni_mha_desc* d, MhaArgs& a) {
    MMNI_ARG_CHECK(d != nullptr, "mha: null descriptor");
    MMNI_ARG_CHECK(d->Tq > 0 && d->Tk > 0 && d->B > 0 && d->heads > 0 && d->head_dim > 0, "mha: bad sizes");
    if (d->head_dim > 16) {
        set_error("mha: unsupported head_dim %d (supported 1..16)", d->head_dim);
        return -2;
    }
    const int E = d->heads * d->head_dim;
    MMNI_ARG_CHECK(d->q_stride >= E && d->k_stride >= E && d->v_stride >= E && d->o_stride >= E,
                   "mha: strides must be >= heads*head_dim");
    MMNI_ARG_CHECK((int64_t)d->B * d->heads <= 65535, "mha: B*heads exceeds the grid y limit");
    MMNI_ARG_CHECK((int64_t)d->B * d->heads * d->Tq < (1ll << 31), "mha: too many rows");
    MMNI_ARG_CHECK(d->dropout >= 0.f && d->dropout < 1.f, "mha: dropout must be in [0, 1)");
    a.Tq = d->Tq; a.Tk = d->Tk; a.B = d->B; a.H = d->heads; a.hd = d->head_dim; a.causal = d->causal_diag;
    a.scale = d->scale;
    a.scale2 = d->scale * kLog2e;
    a.qs = d->q_stride; a.ks = d->k_stride; a.vs = d->v_stride; a.os = d->o_stride;
    const double keep = 1.0 - (double)d->dropout;
    a.inv_keep = (float)(1.0 / keep);
    const double t = keep * 4294967296.0;
    a.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
    a.seed = d->seed;
    return 0;
}

static int hd_pad(int hd) { return hd <= 4 ? 4 : (hd <= 8 ? 8 : 16); }

template <int HDP, bool DROP>
static int mha_fwd_launch(MhaArgs& a, hipStream_t s) {
    dim3 grid((a.Tq + MT - 1) / MT, a.B * a.H);
    mha_fwd_mfma_kernel<HDP, DROP><<<grid, 256, 0, s>>>(a);
    return launch_status("mha_fwd");
}

template <int HDP, bool DROP>
static int mha_bwd_launch(MhaArgs& a, hipStream_t s) {
    const int64_t n = (int64_t)a.Tq * a.B * a.H;
    mha_delta_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
    int rc = launch_status("mha_delta");
    if (rc) return rc;
    dim3 gq((a.Tq + MT - 1) / MT, a.B * a.H);
    mha_dq_mfma_kernel<HDP, DROP><<<gq, 256, 0, s>>>(a);
    rc = launch_status("mha_bwd_dq");
    if (rc) return rc;
    dim3 gk((a.Tk + MT - 1) / MT, a.B * a.H);
    mha_dkv_mfma_kernel<HDP, DROP><<<gk, 256, 0, s>>>(a);
    return launch_status("mha_bwd_dkv");
}

#define MMNI_MHA_DISPATCH(FN)                                                             \
    {                                                                                     \
        const bool drop = a.thresh != 0xffffffffu;                                        \
        hipStream_t st_ = (hipStream_t)stream;                                            \
        switch (hd_pad(a.hd)) {                                                           \
            case 4: return drop ? FN<4, true>(a, st_) : FN<4, false>(a, st_);             \
            case 8: return drop ? FN<8, true>(a, st_) : FN<8, false>(a, st_);             \
            default: return drop ? FN<16, true>(a, st_) : FN<16, false>(a, st_);          \
        }                                                                                 \
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
    MMNI_MHA_DISPATCH(mha_fwd_launch)
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
    MMNI_MHA_DISPATCH(mha_bwd_launch)
}

extern "C" int mmni_mha_mean_probs(const mmni_mha_desc* d, const float* q, const float* k, const float* lse,
                                   float* probs, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && lse && probs, "mha_mean_probs: null pointer");
    a.q = q; a.k = k; a.lse = const_cast<float*>(lse); a.probs = probs;
    const int64_t n = (int64_t)a.B * a.Tq * a.Tk;
    if (a.thresh != 0xffffffffu)
        mha_probs_kernel<true><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
    else
        mha_probs_kernel<false><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
    return launch_status("mha_probs");
}

extern "C" int mmni_mha_dropout_mask(const mmni_mha_desc* d, float* mask, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(mask != nullptr, "mha_dropout_mask: null pointer");
    const int64_t n = (int64_t)a.B * a.H * a.Tq * a.Tk;
    mha_dropout_mask_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a, mask);
    return launch_status("mha_dropout_mask");
}
