// Swin-V2 continuous position bias table (reference: WindowAttention.cpb_mlp and
// its use, swin_v2_module.py:88-91,158-162):
//   out[t][h] = 16 * sigmoid( sum_j w2[h][j] * relu( w1[j] . coords[t] + b1[j] ) )
// over the (2w-1)^k table entries t (1,331 at 6^3 windows), hidden = 512, heads <= 32, k = 2 / 3.
// The torch path ran it as two library GEMMs on a 1,331 x 512 activation plus ReLU / sigmoid / scale
// kernels, and the backward as four more GEMMs and their elementwise partners: ~12 launches of
// ~5-13 us per Swin-V2 block and step, all latency.  Here: one forward and one backward launch (+ the
// fixed-order column sum of the weight-gradient partials, deterministic).
#include "mmni_common.h"

namespace mmni {
namespace cpb {

constexpr int kMaxHeads = 32, kMaxHidden = 512, kMaxNd = 3;   // the reference's cpb_mlp is 512 wide
constexpr int kEpb = 16;         // table entries per forward block
constexpr int kBwdBlocks = 128;  // backward partial rows

struct Args {
    int64_t tsz;
    int nd, hidden, heads;
    const float* coords;   // (tsz, nd)
    const float* w1;       // (hidden, nd)
    const float* b1;       // (hidden)
    const float* w2;       // (heads, hidden)
    const float* out;      // (tsz, heads): the forward's 16 * sigmoid(z) (backward input)
    const float* dout;     // (tsz, heads)
    float* y;              // forward output
    float* part;           // backward: [block][heads * hidden | hidden * nd | hidden]
};

// hidden activations of kEpb entries and the W2 rows in LDS (rows padded to an odd stride: the
// reads below are conflict-free), then a thread per (entry, head) output sums its hidden units in
// order (fixed order; no cross-lane reduction — a 64-lane butterfly per output was a chain of
// ds_bpermute round trips)
constexpr int kHs = kMaxHidden + 1;   // LDS row stride
__global__ __launch_bounds__(256) void cpb_fwd_kernel(Args a) {
    extern __shared__ float fsm[];
    float* h = fsm;                       // [kEpb][kHs]
    float* w2s = fsm + kEpb * kHs;        // [heads][kHs]
    __shared__ float cs[kEpb][kMaxNd];
    const int64_t e0 = (int64_t)blockIdx.x * kEpb;
    const int ne = e0 + kEpb <= a.tsz ? kEpb : (int)(a.tsz - e0);
    if (threadIdx.x < kEpb * kMaxNd) {
        const int e = threadIdx.x / kMaxNd, d = threadIdx.x - e * kMaxNd;
        cs[e][d] = (e < ne && d < a.nd) ? a.coords[(e0 + e) * a.nd + d] : 0.f;
    }
    for (int i = threadIdx.x; i < a.heads * a.hidden; i += 256) {
        const int hd = i / a.hidden, j = i - hd * a.hidden;
        w2s[hd * kHs + j] = a.w2[i];
    }
    // a thread per hidden unit (up to 4 units): its W1 row and bias in registers
    constexpr int UH = kMaxHidden / 256;
    float w1r[UH][kMaxNd], b1r[UH];
#pragma unroll
    for (int u = 0; u < UH; ++u) {
        const int j = threadIdx.x + 256 * u;
        const bool ok = j < a.hidden;
#pragma unroll
        for (int d = 0; d < kMaxNd; ++d) w1r[u][d] = (ok && d < a.nd) ? a.w1[j * a.nd + d] : 0.f;
        b1r[u] = ok ? a.b1[j] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < UH; ++u) {
        const int j = threadIdx.x + 256 * u;
        if (j >= a.hidden) break;
        for (int e = 0; e < kEpb; ++e) {
            float z = b1r[u];
#pragma unroll
            for (int d = 0; d < kMaxNd; ++d) z = fmaf(w1r[u][d], cs[e][d], z);
            h[e * kHs + j] = fmaxf(z, 0.f);
        }
    }
    __syncthreads();
    for (int o = threadIdx.x; o < ne * a.heads; o += 256) {
        const int e = o / a.heads, hd = o - e * a.heads;
        const float* hr = h + e * kHs;
        const float* wr = w2s + hd * kHs;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;   // four fixed-order partial chains
        int j = 0;
        for (; j + 3 < a.hidden; j += 4) {
            s0 = fmaf(wr[j], hr[j], s0);
            s1 = fmaf(wr[j + 1], hr[j + 1], s1);
            s2 = fmaf(wr[j + 2], hr[j + 2], s2);
            s3 = fmaf(wr[j + 3], hr[j + 3], s3);
        }
        for (; j < a.hidden; ++j) s0 = fmaf(wr[j], hr[j], s0);
        const float sv = (s0 + s1) + (s2 + s3);
        a.y[(e0 + e) * a.heads + hd] = 16.f / (1.f + expf(-sv));
    }
}

size_t fwd_lds_bytes(int heads) { return (size_t)(kEpb + heads) * kHs * sizeof(float); }

// a thread per hidden unit (hidden / 256 units each), a contiguous range of entries per block:
// dz = dout * out * (1 - out / 16) (d(16 sigmoid)), dh_j = [h_j > 0] sum_h w2[h][j] dz_h, and the
// per-thread sums of dw2[h][j] (dz_h h_j), dw1[j][d] (dh_j c_d), db1[j] (dh_j): one partial row
// per block (no atomics)
constexpr int kChunk = 64;       // backward entries staged in LDS per round

template <int U>
__global__ __launch_bounds__(256) void cpb_bwd_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) float dz[kChunk][kMaxHeads];
    __shared__ float cs[kChunk][kMaxNd];
    float w2c[U][kMaxHeads], w1r[U][kMaxNd], b1r[U];
    float gw2[U][kMaxHeads], gw1[U][kMaxNd], gb1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = threadIdx.x + 256 * u;
        const bool ok = j < a.hidden;
#pragma unroll
        for (int h = 0; h < kMaxHeads; ++h) {
            w2c[u][h] = (ok && h < a.heads) ? a.w2[h * a.hidden + j] : 0.f;
            gw2[u][h] = 0.f;
        }
#pragma unroll
        for (int d = 0; d < kMaxNd; ++d) {
            w1r[u][d] = (ok && d < a.nd) ? a.w1[j * a.nd + d] : 0.f;
            gw1[u][d] = 0.f;
        }
        b1r[u] = ok ? a.b1[j] : 0.f;
        gb1[u] = 0.f;
    }
    // the block's contiguous entry range, staged kChunk entries at a time (dz and coordinates for
    // all of them in one round trip)
    const int64_t per = (a.tsz + gridDim.x - 1) / gridDim.x;
    const int64_t e_begin = (int64_t)blockIdx.x * per;
    const int64_t e_end = e_begin + per < a.tsz ? e_begin + per : a.tsz;
    for (int64_t c0 = e_begin; c0 < e_end; c0 += kChunk) {
        const int n = (int)(e_end - c0 < kChunk ? e_end - c0 : kChunk);
        __syncthreads();   // the previous chunk is consumed
        for (int i = threadIdx.x; i < n * kMaxHeads; i += 256) {
            const int e = i / kMaxHeads, h = i - e * kMaxHeads;
            float v = 0.f;   // heads past a.heads: zero pad (read by the float4 loads)
            if (h < a.heads) {
                const float o = a.out[(c0 + e) * a.heads + h];
                v = a.dout[(c0 + e) * a.heads + h] * o * (1.f - o * (1.f / 16.f));   // d(16 sigmoid)
            }
            dz[e][h] = v;
        }
        for (int i = threadIdx.x; i < n * a.nd; i += 256) cs[i / a.nd][i % a.nd] = a.coords[c0 * a.nd + i];
        __syncthreads();
        for (int e = 0; e < n; ++e) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float z = b1r[u];
#pragma unroll
                for (int d = 0; d < kMaxNd; ++d) z = fmaf(w1r[u][d], d < a.nd ? cs[e][d] : 0.f, z);
                const float hj = fmaxf(z, 0.f);
                float dh = 0.f;
#pragma unroll
                for (int h4 = 0; h4 < kMaxHeads; h4 += 4) {
                    if (h4 >= a.heads) break;   // uniform; heads past a.heads read the zeroed pad
                    const float4 g4 = *reinterpret_cast<const float4*>(&dz[e][h4]);
                    const float g[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        dh = fmaf(w2c[u][h4 + i], g[i], dh);
                        gw2[u][h4 + i] = fmaf(g[i], hj, gw2[u][h4 + i]);
                    }
                }
                dh = z > 0.f ? dh : 0.f;
#pragma unroll
                for (int d = 0; d < kMaxNd; ++d) gw1[u][d] = fmaf(dh, d < a.nd ? cs[e][d] : 0.f, gw1[u][d]);
                gb1[u] += dh;
            }
        }
    }
    const int64_t ncols = (int64_t)a.heads * a.hidden + (int64_t)a.hidden * a.nd + a.hidden;
    float* p = a.part + (int64_t)blockIdx.x * ncols;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = threadIdx.x + 256 * u;
        if (j >= a.hidden) continue;
#pragma unroll
        for (int h = 0; h < kMaxHeads; ++h)
            if (h < a.heads) p[h * a.hidden + j] = gw2[u][h];
#pragma unroll
        for (int d = 0; d < kMaxNd; ++d)
            if (d < a.nd) p[(int64_t)a.heads * a.hidden + j * a.nd + d] = gw1[u][d];
        p[(int64_t)a.heads * a.hidden + (int64_t)a.hidden * a.nd + j] = gb1[u];
    }
}

int bwd_blocks(int64_t tsz) { return (int)(tsz < kBwdBlocks ? tsz : kBwdBlocks); }

}  // namespace cpb
}  // namespace mmni

using namespace mmni;

#define MMNI_CPB_CHECK(what)                                                                                   \
    MMNI_ARG_CHECK(tsz > 0 && nd >= 1 && nd <= cpb::kMaxNd && hidden >= 1 && hidden <= cpb::kMaxHidden &&     \
                       heads >= 1 && heads <= cpb::kMaxHeads,                                                  \
                   what ": tsz=%lld nd=%d hidden=%d heads=%d outside the supported range (nd <= 3, hidden <= " \
                        "512, heads <= 32)",                                                                  \
                   (long long)tsz, nd, hidden, heads)

extern "C" int mmni_cpb_fwd(int64_t tsz, int nd, int hidden, int heads, const float* coords, const float* w1,
                            const float* b1, const float* w2, float* out, void* stream) {
    MMNI_CPB_CHECK("cpb_fwd");
    MMNI_ARG_CHECK(coords && w1 && b1 && w2 && out, "cpb_fwd: null pointer");
    cpb::Args a{};
    a.tsz = tsz; a.nd = nd; a.hidden = hidden; a.heads = heads;
    a.coords = coords; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.y = out;
    const unsigned blocks = (unsigned)((tsz + cpb::kEpb - 1) / cpb::kEpb);
    const size_t lds = cpb::fwd_lds_bytes(heads);   // <= 98.5 KB (32 heads x 512 hidden): raise the 64 KB cap
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cpb::cpb_fwd_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)cpb::fwd_lds_bytes(cpb::kMaxHeads));
        if (e != hipSuccess) { set_error("cpb_fwd attribute: %s", hipGetErrorString(e)); return (int)e; }
        attr_set = true;
    }
    cpb::cpb_fwd_kernel<<<blocks, 256, lds, (hipStream_t)stream>>>(a);
    return launch_status("cpb_fwd");
}

extern "C" size_t mmni_cpb_bwd_workspace_bytes(int64_t tsz, int nd, int hidden, int heads) {
    if (tsz <= 0) return 0;
    return (size_t)cpb::bwd_blocks(tsz) * ((size_t)heads * hidden + (size_t)hidden * nd + hidden) * sizeof(float);
}

extern "C" int mmni_cpb_bwd(int64_t tsz, int nd, int hidden, int heads, const float* coords, const float* w1,
                            const float* b1, const float* w2, const float* out, const float* dout, float* dw1,
                            float* db1, float* dw2, void* workspace, void* stream) {
    MMNI_CPB_CHECK("cpb_bwd");
    MMNI_ARG_CHECK(coords && w1 && b1 && w2 && out && dout && dw1 && db1 && dw2 && workspace,
                   "cpb_bwd: null pointer");
    cpb::Args a{};
    a.tsz = tsz; a.nd = nd; a.hidden = hidden; a.heads = heads;
    a.coords = coords; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.out = out; a.dout = dout;
    a.part = static_cast<float*>(workspace);
    const int blocks = cpb::bwd_blocks(tsz);
    hipStream_t s = (hipStream_t)stream;
    const int U = (hidden + 255) / 256;
    if (U == 1) cpb::cpb_bwd_kernel<1><<<blocks, 256, 0, s>>>(a);
    else cpb::cpb_bwd_kernel<2><<<blocks, 256, 0, s>>>(a);
    int rc = launch_status("cpb_bwd");
    if (rc) return rc;
    ColSegs segs{};
    segs.n = 3;
    segs.end[0] = heads * hidden;
    segs.end[1] = heads * hidden + hidden * nd;
    segs.end[2] = heads * hidden + hidden * nd + hidden;
    segs.dst[0] = dw2;
    segs.dst[1] = dw1;
    segs.dst[2] = db1;
    column_sum_segs(a.part, blocks, segs.end[2], segs, s);
    return launch_status("cpb_bwd_sum");
}
