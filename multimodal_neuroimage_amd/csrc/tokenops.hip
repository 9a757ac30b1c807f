// Token-wise ops of the Swin blocks for gfx950 (SURVEY §8 row a3b / §8f.1 building blocks).
//
// At C = 12 every LayerNorm and every weight gradient of the block's Linear layers runs over
// ~3.5M token rows of 48 bytes.  Generic library kernels handle these shapes badly (rocprof r01:
// torch's LayerNorm fwd 2.9 ms, its gamma/beta backward 3.1 ms and hipBLASLt's K = 3.5M
// weight-gradient GEMMs 3.1 ms per call, ~1.8 s of a 3.9 s step).  These kernels stream the rows
// once:
//   layernorm_fwd   one lane per row, the row in registers, y + (mean, rstd) written
//                   (nn.LayerNorm semantics: biased variance, eps inside the sqrt)
//   layernorm_bwd   one lane per row for dx; gamma/beta partial sums per workgroup written to a
//                   workspace slab and summed in a fixed order by a second launch (deterministic)
//   linear_dw       dW[n][k] = sum_r dY[r][n] X[r][k], db[n] = sum_r dY[r][n] on the f32 MFMA
//                   (v_mfma_f32_16x16x4_f32, exact f32 FMA chains): each wave owns every output
//                   tile and reduces over its row slice (4 rows per MFMA), partial tiles go to a
//                   workspace slab reduced in a fixed order by a second launch.
#include "mmni_common.h"

namespace mmni {

template <int C>
__device__ __forceinline__ void ldrow(float (&d)[C], const float* s) {
    if constexpr (C % 4 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 4) {
            const float4 t = *reinterpret_cast<const float4*>(s + c);
            d[c] = t.x; d[c + 1] = t.y; d[c + 2] = t.z; d[c + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) d[c] = s[c];
    }
}

template <int C>
__device__ __forceinline__ void strow(float* d, const float (&s)[C]) {
    if constexpr (C % 4 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 4)
            *reinterpret_cast<float4*>(d + c) = make_float4(s[c], s[c + 1], s[c + 2], s[c + 3]);
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) d[c] = s[c];
    }
}

template <int C>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(int64_t rows, const float* __restrict__ x,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            float* __restrict__ y, float* __restrict__ mean,
                                                            float* __restrict__ rstd) {
    float gm[C], bt[C];
#pragma unroll
    for (int c = 0; c < C; ++c) { gm[c] = gamma[c]; bt[c] = beta[c]; }
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        float v[C];
        ldrow<C>(v, x + r * C);
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) s += v[c];
        const float mu = s * (1.0f / C);
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) { const float d = v[c] - mu; ss = fmaf(d, d, ss); }
        const float rs = 1.0f / sqrtf(ss * (1.0f / C) + eps);
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = (v[c] - mu) * rs * gm[c] + bt[c];
        strow<C>(y + r * C, v);
        mean[r] = mu;
        rstd[r] = rs;
    }
}

template <int C>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(int64_t rows, const float* __restrict__ dy,
                                                            const float* __restrict__ x,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, float* __restrict__ dx,
                                                            float* __restrict__ part) {
    __shared__ float red[4 * 2 * C];   // [wave][2C]
    float gm[C], dg[C], db[C];
#pragma unroll
    for (int c = 0; c < C; ++c) { gm[c] = gamma[c]; dg[c] = 0.f; db[c] = 0.f; }
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        float g[C], xv[C];
        ldrow<C>(g, dy + r * C);
        ldrow<C>(xv, x + r * C);
        const float mu = mean[r], rs = rstd[r];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float xh = (xv[c] - mu) * rs;
            const float gg = g[c] * gm[c];
            dg[c] = fmaf(g[c], xh, dg[c]);
            db[c] += g[c];
            s1 += gg;
            s2 = fmaf(gg, xh, s2);
            xv[c] = xh;
        }
        s1 *= (1.0f / C);
        s2 *= (1.0f / C);
#pragma unroll
        for (int c = 0; c < C; ++c) g[c] = rs * (g[c] * gm[c] - s1 - xv[c] * s2);
        strow<C>(dx + r * C, g);
    }
    // workgroup partial sums of dgamma / dbeta -> part[blockIdx][2C]: a butterfly over the wave's
    // lanes (every lane ends with the same, fixed-order sum), then the 4 wave sums in wave order.
    // (A 256-wide LDS tree per channel cost 2C x 9 barriers: ~110 us for a 108-row C = 48 call.)
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 2 * C; ++c) {
        float v = c < C ? dg[c] : db[c - C];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) red[wib * 2 * C + c] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x)
        part[(int64_t)blockIdx.x * 2 * C + c] = ((red[c] + red[2 * C + c]) + red[4 * C + c]) + red[6 * C + c];
}

// out[j] = sum_b part[b][j] in a fixed order (columns j >= split go to out2[j - split]);
// deterministic for a given nparts.  Two stages so that the grid is wide (the per-wave partial
// slabs are ~2k rows x <= 1k columns; one block per 64 columns left most of the GPU idle):
//   stage 1  block (column group, row slice): CW columns x rps rows, RG = 1024 / CW interleaved
//            row groups with four double accumulators each, combined in order through LDS; the
//            double result is split into hi + lo floats stored IN PLACE in the slice's first two
//            rows (same column: no other block reads them);
//   stage 2  one lane per column adds the slices' (hi + lo) in slice order, in double.
constexpr int kColSlices = 16;   // row slices of stage 1 (stage 2 holds one value pair per slice)

template <int CW>
__global__ __launch_bounds__(1024) void column_sum_stage1_kernel(float* __restrict__ part, int nparts, int ncols,
                                                                 int rps) {
    constexpr int RG = 1024 / CW;
    __shared__ double red[RG][CW];
    const int tx = threadIdx.x % CW, ty = threadIdx.x / CW;
    const int j = blockIdx.x * CW + tx;
    const int r0 = blockIdx.y * rps;
    const int r1 = r0 + rps < nparts ? r0 + rps : nparts;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    if (j < ncols) {
        int b = r0 + ty;
        for (; b + 3 * RG < r1; b += 4 * RG) {
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] += part[(int64_t)(b + u * RG) * ncols + j];
        }
        for (int u = 0; b < r1; b += RG, ++u) s[u & 3] += part[(int64_t)b * ncols + j];
    }
    red[ty][tx] = (s[0] + s[1]) + (s[2] + s[3]);
    __syncthreads();
    if (ty == 0 && j < ncols) {
        double t = 0.0;
        for (int g = 0; g < RG; ++g) t += red[g][tx];
        const float hi = (float)t;
        part[(int64_t)r0 * ncols + j] = hi;
        if (r1 - r0 > 1) part[(int64_t)(r0 + 1) * ncols + j] = (float)(t - (double)hi);
    }
}

__global__ __launch_bounds__(256) void column_sum_stage2_kernel(const float* __restrict__ part, int nparts, int ncols,
                                                                int rps, int nslices, ColSegs segs) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= ncols) return;
    // all slice loads issued before the (in-order, double) sum: one memory latency, not 2 x nslices.
    // The row indices are clamped instead of the loads being guarded: guarded loads became one
    // branch and one full memory wait each (32 waits, ~10 us per launch)
    float hi[kColSlices], lo[kColSlices];
#pragma unroll
    for (int sl = 0; sl < kColSlices; ++sl) {
        const int r0 = sl * rps < nparts ? sl * rps : nparts - 1;
        const int r1 = r0 + 1 < nparts ? r0 + 1 : nparts - 1;
        hi[sl] = part[(int64_t)r0 * ncols + j];
        lo[sl] = part[(int64_t)r1 * ncols + j];
    }
    double t = 0.0;
#pragma unroll
    for (int sl = 0; sl < kColSlices; ++sl) {
        if (sl < nslices) {
            t += (double)hi[sl];
            if (nparts - sl * rps > 1) t += (double)lo[sl];
        }
    }
    // column j -> segment k (columns [end[k-1], end[k]) go to dst[k]; a null dst drops them)
    int k = 0, begin = 0;
#pragma unroll
    for (int i = 0; i < ColSegs::kMax - 1; ++i) {
        if (i < segs.n - 1 && j >= segs.end[i]) {
            k = i + 1;
            begin = segs.end[i];
        }
    }
    float* d = segs.dst[k];
    if (d == nullptr) return;
    if (segs.accumulate) d[j - begin] += (float)t;
    else d[j - begin] = (float)t;
}

void column_sum_segs(const float* part_c, int nparts, int ncols, const ColSegs& segs, hipStream_t s) {
    float* part = const_cast<float*>(part_c);   // scratch: stage 1 leaves its sums in place
    const int want = kColSlices;                // row slices
    int rps = (nparts + want - 1) / want;
    if (rps < 2) rps = 2;
    const int nslices = (nparts + rps - 1) / rps;
    if (ncols <= 16)
        column_sum_stage1_kernel<16><<<dim3((ncols + 15) / 16, nslices), 1024, 0, s>>>(part, nparts, ncols, rps);
    else if (ncols <= 32)
        column_sum_stage1_kernel<32><<<dim3((ncols + 31) / 32, nslices), 1024, 0, s>>>(part, nparts, ncols, rps);
    else
        column_sum_stage1_kernel<64><<<dim3((ncols + 63) / 64, nslices), 1024, 0, s>>>(part, nparts, ncols, rps);
    column_sum_stage2_kernel<<<(ncols + 255) / 256, 256, 0, s>>>(part, nparts, ncols, rps, nslices, segs);
}

void column_sum(const float* part, int nparts, int ncols, float* out, int split, float* out2, hipStream_t s) {
    ColSegs segs{};
    segs.n = 2;
    segs.end[0] = split;
    segs.end[1] = ncols;
    segs.dst[0] = out;
    segs.dst[1] = out2;
    column_sum_segs(part, nparts, ncols, segs, s);
}

using f4 = __attribute__((ext_vector_type(4))) float;

// Weight gradient of a token Linear: dW (N, K) = dY^T X, db (N) = colsum(dY).
// Each wave: NT x KT output tiles of 16x16 in accumulators, rows [r0, r1) in steps of 4.
template <int NT, int KT>
__global__ __launch_bounds__(256) void linear_dw_kernel(int64_t rows, int N, int K, const float* __restrict__ x,
                                                        int64_t ldx, const float* __restrict__ dy, int64_t lddy,
                                                        float* __restrict__ part, int with_bias) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    const int64_t steps = (rows + 3) / 4;
    const int64_t per = (steps + nwaves - 1) / nwaves;
    const int64_t s0 = (int64_t)wave * per;
    const int64_t s1 = s0 + per < steps ? s0 + per : steps;
    const int li = lane & 15, lk = lane >> 4;
    f4 acc[NT][KT];
    float bsum[NT];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        bsum[m] = 0.f;
#pragma unroll
        for (int n = 0; n < KT; ++n) acc[m][n] = f4{0.f, 0.f, 0.f, 0.f};
    }
    // branch-free loads (clamped addresses, select after the load) so the loop unrolls and the
    // loads of several 4-row steps are in flight together
    int noff[NT], koff[KT];
    bool nok[NT], kok[KT];
#pragma unroll
    for (int m = 0; m < NT; ++m) { const int n = m * 16 + li; nok[m] = n < N; noff[m] = nok[m] ? n : N - 1; }
#pragma unroll
    for (int t = 0; t < KT; ++t) { const int k = t * 16 + li; kok[t] = k < K; koff[t] = kok[t] ? k : K - 1; }
    // MFMA is convergent, so hipcc will not runtime-unroll this loop: unroll by hand (4 steps =
    // 16 rows per iteration, all loads issued before the MFMAs), then a remainder loop.
    auto load_step = [&](int64_t st, float (&a)[NT], float (&b)[KT]) {
        const int64_t r = st * 4 + lk;
        const bool rv = r < rows;
        const int64_t rc = rv ? r : rows - 1;
#pragma unroll
        for (int m = 0; m < NT; ++m) {
            const float v = dy[rc * lddy + noff[m]];
            a[m] = (rv && nok[m]) ? v : 0.f;
        }
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            const float v = x[rc * ldx + koff[t]];
            b[t] = (rv && kok[t]) ? v : 0.f;
        }
    };
    auto mma_step = [&](const float (&a)[NT], const float (&b)[KT]) {
#pragma unroll
        for (int m = 0; m < NT; ++m) {
            bsum[m] += a[m];
#pragma unroll
            for (int t = 0; t < KT; ++t)
                acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[t], acc[m][t], 0, 0, 0);
        }
    };
    int64_t st = s0;
    for (; st + 4 <= s1; st += 4) {
        float a0[NT], b0[KT], a1[NT], b1[KT], a2[NT], b2[KT], a3[NT], b3[KT];
        load_step(st, a0, b0);
        load_step(st + 1, a1, b1);
        load_step(st + 2, a2, b2);
        load_step(st + 3, a3, b3);
        mma_step(a0, b0);
        mma_step(a1, b1);
        mma_step(a2, b2);
        mma_step(a3, b3);
    }
    for (; st < s1; ++st) {
        float a0[NT], b0[KT];
        load_step(st, a0, b0);
        mma_step(a0, b0);
    }
    // fold the block's 4 wave tiles in LDS in wave order (deterministic), then write one partial
    // per block: part[block][N*K + N]
    extern __shared__ float tile[];   // [N*K + N]
    const int wib = threadIdx.x >> 6;
    for (int w = 0; w < 4; ++w) {
        if (wib == w) {
#pragma unroll
            for (int m = 0; m < NT; ++m)
#pragma unroll
                for (int t = 0; t < KT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int n = m * 16 + lk * 4 + e;   // C/D row
                        const int k = t * 16 + li;           // C/D col
                        if (n < N && k < K) tile[n * K + k] = (w ? tile[n * K + k] : 0.f) + acc[m][t][e];
                    }
            if (with_bias) {
#pragma unroll
                for (int m = 0; m < NT; ++m) {
                    float v = bsum[m];
                    v += __shfl_xor(v, 16);
                    v += __shfl_xor(v, 32);
                    const int n = m * 16 + li;
                    if (lk == 0 && n < N) tile[N * K + n] = (w ? tile[N * K + n] : 0.f) + v;
                }
            }
        }
        __syncthreads();
    }
    float* pw = part + (int64_t)blockIdx.x * (N * K + N);
    for (int e = threadIdx.x; e < N * K + N; e += blockDim.x) pw[e] = tile[e];
}

}  // namespace mmni

using namespace mmni;

#define MMNI_LN_DISPATCH(KER, ...)                                                               \
    switch (C) {                                                                                 \
        case 12: KER<12><<<grid, 256, 0, (hipStream_t)stream>>>(__VA_ARGS__); break;              \
        case 24: KER<24><<<grid, 256, 0, (hipStream_t)stream>>>(__VA_ARGS__); break;              \
        case 48: KER<48><<<grid, 256, 0, (hipStream_t)stream>>>(__VA_ARGS__); break;              \
        case 96: KER<96><<<grid, 256, 0, (hipStream_t)stream>>>(__VA_ARGS__); break;              \
        default: set_error("layernorm: unsupported C=%d (12, 24, 48, 96)", C); return -2;         \
    }

static int ln_grid(int64_t rows) {
    int64_t g = (rows + 255) / 256;
    return (int)(g < 2048 ? g : 2048);
}

extern "C" int mmni_layernorm_fwd(int64_t rows, int C, const float* x, const float* gamma, const float* beta,
                                  float eps, float* y, float* mean, float* rstd, void* stream) {
    MMNI_ARG_CHECK(rows > 0 && x && gamma && beta && y && mean && rstd, "layernorm_fwd: bad arguments");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0,
                   "layernorm_fwd: x/y must be 16-byte aligned");
    const int grid = ln_grid(rows);
    MMNI_LN_DISPATCH(layernorm_fwd_kernel, rows, x, gamma, beta, eps, y, mean, rstd)
    return launch_status("layernorm_fwd");
}

extern "C" size_t mmni_layernorm_bwd_workspace_bytes(int64_t rows, int C) {
    const size_t own = (size_t)ln_grid(rows) * 2 * C * sizeof(float);
    const size_t small = rows <= kSmallRows ? enc_row_ln_bwd_workspace(rows, C) : 0;
    return own > small ? own : small;
}

extern "C" int mmni_layernorm_bwd(int64_t rows, int C, const float* dy, const float* x, const float* gamma,
                                  const float* mean, const float* rstd, float* dx, float* dgamma, float* dbeta,
                                  void* workspace, void* stream) {
    MMNI_ARG_CHECK(rows > 0 && dy && x && gamma && mean && rstd && dx && dgamma && dbeta && workspace,
                   "layernorm_bwd: bad arguments");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(dy) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(dx) % 16 == 0,
                   "layernorm_bwd: tensors must be 16-byte aligned");
    if (rows <= kSmallRows && C <= 256)   // a wave per row: one lane per row left a short call serial
        return enc_row_ln_bwd(rows, C, dy, C, x, C, gamma, mean, rstd, nullptr, 0, dx, C, dgamma, dbeta, workspace,
                              (hipStream_t)stream);
    const int grid = ln_grid(rows);
    float* part = reinterpret_cast<float*>(workspace);
    MMNI_LN_DISPATCH(layernorm_bwd_kernel, rows, dy, x, gamma, mean, rstd, dx, part)
    int rc = launch_status("layernorm_bwd");
    if (rc) return rc;
    // columns [0, C) -> dgamma, [C, 2C) -> dbeta: two fixed-order column sums
    column_sum(part, grid, 2 * C, dgamma, C, dbeta, (hipStream_t)stream);   // [0,C) dgamma, [C,2C) dbeta
    return launch_status("layernorm_colsum");
}

static int dw_waves() { return 4096; }

// waves of one linear_dw call: at least 16 four-row steps per wave, so short calls (a few hundred
// rows at the deep Swin-V2 stages) do not reduce 1024 mostly-empty partial rows
static int dw_waves_for(int64_t rows) {
    const int64_t steps = (rows + 3) / 4;
    int64_t w = (steps + 15) / 16;
    w = (w + 3) / 4 * 4;
    return (int)(w < 4 ? 4 : (w > dw_waves() ? dw_waves() : w));
}

extern "C" size_t mmni_linear_dw_workspace_bytes(int N, int K) {
    // per-block partials; covers the short-row path too (at most 256 row chunks)
    return (size_t)(dw_waves() / 4) * (N * K + N) * sizeof(float);
}

extern "C" int mmni_linear_dw(int64_t rows, int N, int K, const float* x, int64_t ldx, const float* dy,
                              int64_t lddy, float* dw, float* db, void* workspace, void* stream) {
    MMNI_ARG_CHECK(rows > 0 && N > 0 && K > 0 && x && dy && dw && workspace, "linear_dw: bad arguments");
    MMNI_ARG_CHECK(ldx >= K && lddy >= N, "linear_dw: leading dimensions too small");
    if (rows <= kSmallRows)   // row chunks x 64 x 64 output tiles: many workgroups for a short call
        return enc_rowgemm_dw(rows, N, K, x, ldx, dy, lddy, nullptr, nullptr, nullptr, nullptr, dw, db, workspace,
                              (hipStream_t)stream);
    const int NT = (N + 15) / 16, KT = (K + 15) / 16;
    float* part = reinterpret_cast<float*>(workspace);
    const int waves = dw_waves_for(rows);
    const int grid = waves * 64 / 256;
    const int wb = db != nullptr;
    const size_t lds = (size_t)(N * K + N) * sizeof(float);
    MMNI_ARG_CHECK(lds <= 64 * 1024, "linear_dw: N*K too large");
    hipStream_t s = (hipStream_t)stream;
#define MMNI_DW_CASE(A, B)                                                                     \
    if (NT == A && KT == B) {                                                                  \
        linear_dw_kernel<A, B><<<grid, 256, lds, s>>>(rows, N, K, x, ldx, dy, lddy, part, wb);    \
    } else
    MMNI_DW_CASE(1, 1) MMNI_DW_CASE(1, 2) MMNI_DW_CASE(1, 3) MMNI_DW_CASE(2, 1) MMNI_DW_CASE(3, 1)
    MMNI_DW_CASE(2, 2) MMNI_DW_CASE(3, 3) MMNI_DW_CASE(1, 4) MMNI_DW_CASE(4, 1) MMNI_DW_CASE(2, 3)
    MMNI_DW_CASE(3, 2) MMNI_DW_CASE(9, 3) MMNI_DW_CASE(3, 9) MMNI_DW_CASE(6, 2) MMNI_DW_CASE(2, 6)
    MMNI_DW_CASE(4, 2) MMNI_DW_CASE(2, 4) MMNI_DW_CASE(5, 3) MMNI_DW_CASE(3, 5) MMNI_DW_CASE(6, 3)
    MMNI_DW_CASE(3, 6) MMNI_DW_CASE(8, 2) MMNI_DW_CASE(2, 8) MMNI_DW_CASE(12, 3) MMNI_DW_CASE(3, 12)
    MMNI_DW_CASE(4, 4) MMNI_DW_CASE(6, 6) MMNI_DW_CASE(4, 12) MMNI_DW_CASE(12, 4)
    {
        set_error("linear_dw: unsupported tile grid %dx%d (N=%d, K=%d)", NT, KT, N, K);
        return -2;
    }
#undef MMNI_DW_CASE
    int rc = launch_status("linear_dw");
    if (rc) return rc;
    const int cols = N * K + N;
    column_sum(part, waves / 4, cols, dw, N * K, db, s);
    rc = launch_status("linear_dw_colsum");
    if (rc) return rc;
    return 0;
}
