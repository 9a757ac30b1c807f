// Split-K weight-gradient reductions of the crossmodal encoder's Linears (functional._SplitKLinear,
// the backward of crossmodal_transformer.py:189-194 Linear / multihead_attention.py in/out_proj).
// The row contraction dW = dY^T X runs as one batched library GEMM over S row chunks (S partial
// N x K products, bf16 under the C5 head's autocast); this file finishes it in two launches:
//   1. one grid with two block kinds: dW blocks sum the S partials (16 chunk slices per element quad,
//      then a fixed LDS tree; fp32) and db blocks take column sums of dY over row slabs of `rpb`
//      rows into a partial matrix;
//   2. the fixed-order column sum of the db partials (16 slab slices per column + an LDS tree).
// Both orders are fixed by the shape: bitwise deterministic.  Replaces torch's two reductions per
// Linear (bmm(...).sum(0) and dY.sum(0): 7 + 17 us per call at 32,768 rows in the C5 profile).
#include "mmni_common.h"

namespace mmni {
namespace splitk {

struct Args {
    const void* part;   // [S][NK] chunk partials of dW
    const void* dy;     // [rows][ldy] output gradient (db source)
    float* dw;          // [NK]
    float* dpart;       // [nbd][N] db partials
    int64_t NK, rows, ldy;
    int S, N, rpb, nbw;
};

template <typename T>
__device__ __forceinline__ float ld1(const T* p);
template <>
__device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld1<__bf16>(const __bf16* p) { return (float)*p; }

// four consecutive elements (one 8- or 16-byte load when VEC)
template <typename T, bool VEC>
__device__ __forceinline__ void ld4(const T* p, float v[4]) {
    if constexpr (VEC && sizeof(T) == 4) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else if constexpr (VEC) {
        const uint2 q = *reinterpret_cast<const uint2*>(p);
        v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
        v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ld1<T>(p + i);
    }
}

constexpr int kNT = 256;
constexpr int kQB = 16, kSL = 16;   // dW block: 16 element quads x 16 chunk slices

// dW: thread (q, sl) sums chunks sl, sl + 16, ... of element quad q (all loads in flight at S <= 64),
// then the 16 slices add by a fixed LDS tree
template <typename T, bool VEC>
__device__ __forceinline__ void dw_block(const Args& a, int bx, float4* red) {
    const T* part = static_cast<const T*>(a.part);
    const int q = threadIdx.x % kQB, sl = threadIdx.x / kQB;
    const int64_t e0 = ((int64_t)bx * kQB + q) * 4;
    const bool live = e0 < a.NK;
    // tail quads: clamp to the last full quad (VEC: NK % 4 == 0) or per element
    const int64_t eb = live ? e0 : 0;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = sl; c0 < a.S; c0 += 4 * kSL) {
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = c0 + u * kSL;
            const T* p = part + (int64_t)(c < a.S ? c : a.S - 1) * a.NK;
            if (VEC) {
                ld4<T, true>(p + eb, v[u]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[u][i] = ld1<T>(p + (eb + i < a.NK ? eb + i : a.NK - 1));
            }
            if (c >= a.S) v[u][0] = v[u][1] = v[u][2] = v[u][3] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) s[i] += v[u][i];
    }
    red[sl * kQB + q] = make_float4(s[0], s[1], s[2], s[3]);
    __syncthreads();
#pragma unroll
    for (int h = kSL / 2; h > 0; h >>= 1) {
        if (sl < h) {
            float4 x = red[sl * kQB + q];
            const float4 y = red[(sl + h) * kQB + q];
            x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
            red[sl * kQB + q] = x;
        }
        __syncthreads();
    }
    if (sl == 0 && live) {
        const float4 r = red[q];
        const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (e0 + i < a.NK) a.dw[e0 + i] = rv[i];
    }
}

// db partial of one slab of rows: thread (u, g) sums column quad u (VEC; else column u) over rows
// g, g + R, ... of the slab; the R row groups then add in LDS in group order
template <typename T, bool VEC>
__device__ __forceinline__ void db_block(const Args& a, int bx, float* red) {
    constexpr int W = VEC ? 4 : 1;   // columns per thread
    const T* dy = static_cast<const T*>(a.dy);
    const int64_t r0 = (int64_t)bx * a.rpb;
    const int64_t r1 = r0 + a.rpb < a.rows ? r0 + a.rpb : a.rows;
    const int NU = (a.N + W - 1) / W;
    const int NUb = NU < kNT ? NU : kNT;   // column units per pass
    const int R = kNT / NUb;               // row groups
    const int u = threadIdx.x % NUb, g = threadIdx.x / NUb;
    for (int c0 = 0; c0 < NU; c0 += NUb) {
        const int cu = c0 + u;
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        if (g < R && cu < NU) {
            const T* p = dy + (int64_t)cu * W;
            int64_t r = r0 + g;
            for (; r + 3 * R < r1; r += 4 * R) {   // 4 rows in flight
                float v[4][4] = {};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (VEC) ld4<T, true>(p + (r + j * R) * a.ldy, v[j]);
                    else v[j][0] = ld1<T>(p + (r + j * R) * a.ldy);
                }
#pragma unroll
                for (int i = 0; i < W; ++i) s[i] += (v[0][i] + v[1][i]) + (v[2][i] + v[3][i]);
            }
            for (; r < r1; r += R) {
                float v0[4] = {0.f, 0.f, 0.f, 0.f};
                if (VEC) ld4<T, true>(p + r * a.ldy, v0);
                else v0[0] = ld1<T>(p + r * a.ldy);
#pragma unroll
                for (int i = 0; i < W; ++i) s[i] += v0[i];
            }
        }
#pragma unroll
        for (int i = 0; i < W; ++i) red[i * kNT + threadIdx.x] = s[i];
        __syncthreads();
        if (threadIdx.x < NUb && cu < NU) {
#pragma unroll
            for (int i = 0; i < W; ++i) {
                float t = red[i * kNT + u];
                for (int k = 1; k < R; ++k) t += red[i * kNT + k * NUb + u];
                if (cu * W + i < a.N) a.dpart[(int64_t)bx * a.N + cu * W + i] = t;
            }
        }
        __syncthreads();
    }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kNT) void reduce_kernel(Args a) {
    __shared__ float4 red[kNT];
    const int bx = blockIdx.x;
    if (bx < a.nbw) dw_block<T, VEC>(a, bx, red);
    else db_block<T, VEC>(a, bx - a.nbw, reinterpret_cast<float*>(red));
}

// db[n] = sum_b dpart[b][n]: a block owns 16 columns x 16 slices (slice sl sums slabs sl, sl + 16,
// ... in order, 8 loads in flight), then the slices add by a fixed LDS tree
__global__ __launch_bounds__(kNT) void db_final_kernel(const float* __restrict__ dpart, int nbd, int N, float* db) {
    __shared__ float red[kSL][kQB];
    const int c = threadIdx.x % kQB, sl = threadIdx.x / kQB;
    const int n = blockIdx.x * kQB + c;
    const int nc = n < N ? n : N - 1;
    float s = 0.f;
    for (int b0 = sl; b0 < nbd; b0 += 8 * kSL) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int b = b0 + u * kSL;
            v[u] = dpart[(int64_t)(b < nbd ? b : nbd - 1) * N + nc];
            if (b >= nbd) v[u] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    red[sl][c] = s;
    __syncthreads();
#pragma unroll
    for (int h = kSL / 2; h > 0; h >>= 1) {
        if (sl < h) red[sl][c] += red[sl + h][c];
        __syncthreads();
    }
    if (sl == 0 && n < N) db[n] = red[0][c];
}

// rows per db slab: ~256 slabs (one per CU), at least 32 rows
int64_t slab_rows(int64_t rows) {
    int64_t r = (rows + 255) / 256;
    return r < 32 ? 32 : r;
}

}  // namespace splitk
}  // namespace mmni

namespace mmni {
namespace splitk {

// fp32 -> bf16 (round to nearest even) of up to kMaxSegs tensors in one launch: blockIdx.y picks the
// segment, blocks stride its elements 4 at a time
struct CastSegs {
    int n;
    const float* src[MMNI_CAST_MAX_SEGS];
    __bf16* dst[MMNI_CAST_MAX_SEGS];
    int64_t count[MMNI_CAST_MAX_SEGS];
};

__global__ __launch_bounds__(kNT) void cast_bf16_kernel(CastSegs c) {
    const int g = blockIdx.y;
    const float* __restrict__ src = c.src[g];
    __bf16* __restrict__ dst = c.dst[g];
    const int64_t n = c.count[g];
    for (int64_t e = ((int64_t)blockIdx.x * kNT + threadIdx.x) * 4; e < n; e += (int64_t)gridDim.x * kNT * 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (e + i < n) dst[e + i] = (__bf16)src[e + i];
    }
}

}  // namespace splitk
}  // namespace mmni

using namespace mmni;

extern "C" int mmni_cast_bf16_multi(int n, const float* const* src, void* const* dst, const int64_t* count,
                                    void* stream) {
    MMNI_ARG_CHECK(n >= 0 && n <= MMNI_CAST_MAX_SEGS && (n == 0 || (src && dst && count)),
                   "cast_bf16_multi: %d segments (1..%d)", n, MMNI_CAST_MAX_SEGS);
    if (n == 0) return 0;
    splitk::CastSegs c{};
    c.n = n;
    int64_t mx = 0;
    for (int i = 0; i < n; ++i) {
        MMNI_ARG_CHECK(src[i] && dst[i] && count[i] >= 0, "cast_bf16_multi: segment %d", i);
        c.src[i] = src[i];
        c.dst[i] = static_cast<__bf16*>(dst[i]);
        c.count[i] = count[i];
        if (count[i] > mx) mx = count[i];
    }
    if (mx == 0) return 0;
    int64_t bx = (mx + 4 * splitk::kNT - 1) / (4 * splitk::kNT);
    if (bx > 64) bx = 64;
    splitk::cast_bf16_kernel<<<dim3((unsigned)bx, (unsigned)n), splitk::kNT, 0, (hipStream_t)stream>>>(c);
    return launch_status("cast_bf16_multi");
}

extern "C" size_t mmni_splitk_reduce_workspace_bytes(int64_t rows, int N) {
    if (rows <= 0 || N <= 0) return 0;
    const int64_t rpb = splitk::slab_rows(rows);
    return (size_t)((rows + rpb - 1) / rpb) * N * sizeof(float);
}

extern "C" int mmni_splitk_reduce(int S, int64_t NK, const void* part, int64_t rows, int N, const void* dy,
                                  int64_t ldy, int dtype, float* dw, float* db, void* workspace, void* stream) {
    MMNI_ARG_CHECK(S > 0 && NK > 0 && part && dw, "splitk_reduce: bad dW operands S=%d NK=%lld", S, (long long)NK);
    MMNI_ARG_CHECK(dtype == 0 || dtype == 1, "splitk_reduce: dtype %d (0 fp32, 1 bf16)", dtype);
    MMNI_ARG_CHECK(db == nullptr || (dy && rows > 0 && N > 0 && ldy >= N && workspace),
                   "splitk_reduce: bad db operands rows=%lld N=%d ldy=%lld", (long long)rows, N, (long long)ldy);
    splitk::Args a{};
    a.part = part; a.dy = dy; a.dw = dw; a.dpart = static_cast<float*>(workspace);
    a.NK = NK; a.rows = rows; a.ldy = ldy; a.S = S; a.N = N;
    a.rpb = (int)splitk::slab_rows(rows > 0 ? rows : 1);
    a.nbw = (int)((NK + 4 * splitk::kQB - 1) / (4 * splitk::kQB));
    const int nbd = db != nullptr ? (int)((rows + a.rpb - 1) / a.rpb) : 0;
    // 8- / 16-byte quads when every row and chunk starts 4-element aligned
    const size_t esz = dtype == 1 ? 2 : 4;
    const auto al = [&](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % (4 * esz)) == 0; };
    const bool vec = NK % 4 == 0 && al(part) && (db == nullptr || (N % 4 == 0 && ldy % 4 == 0 && al(dy)));
    hipStream_t s = (hipStream_t)stream;
    const unsigned grid = (unsigned)(a.nbw + nbd);
    if (dtype == 1) {
        if (vec) splitk::reduce_kernel<__bf16, true><<<grid, splitk::kNT, 0, s>>>(a);
        else splitk::reduce_kernel<__bf16, false><<<grid, splitk::kNT, 0, s>>>(a);
    } else {
        if (vec) splitk::reduce_kernel<float, true><<<grid, splitk::kNT, 0, s>>>(a);
        else splitk::reduce_kernel<float, false><<<grid, splitk::kNT, 0, s>>>(a);
    }
    int rc = launch_status("splitk_reduce");
    if (rc != 0 || db == nullptr) return rc;
    splitk::db_final_kernel<<<(N + splitk::kQB - 1) / splitk::kQB, splitk::kNT, 0, s>>>(a.dpart, nbd, N, db);
    return launch_status("splitk_reduce_colsum");
}
