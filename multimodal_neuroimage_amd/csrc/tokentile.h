// 16-token tiles on the f32 MFMA for the C = 12 token kernels (mlp.hip, blockops.hip).
// Internal, not part of the ABI.
//
// v_mfma_f32_16x16x4_f32 operand maps (cdna_hip_programming.md §FP32-input MFMA): lane l = 16 g + t
// (g = l >> 4, t = l & 15) supplies A[row t][k g] and B[k g][col t]; the accumulator holds
// D[row 4 g + i][col t] in register i.  In every kernel here the tile's 16 tokens are the
// columns, so a lane's accumulator registers are 4 consecutive features of ONE token:
//   feature-major operand (B):  x[t0 + t][4 s + g],  s = 0..2  (12 channels in 3 k-steps)
//   token-major operand  (A/B):  x[t0 + 4 s + g][t]           (contraction over tokens)
//   accumulator row chunk      :  y[t0 + t][16 nt + 4 g + i]
// Token rows are contiguous (C = 12 floats): a tile sits at a wave-uniform base + a per-lane
// offset, so loads and stores take immediate offsets.  Only the last, partial tile is clamped.
#pragma once
#include "mmni_common.h"

namespace mmni {
namespace tt {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int C = 12;    // channels of a token row
constexpr int CS = 3;    // k-steps over the channels

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 zero4() { return (f4){0.f, 0.f, 0.f, 0.f}; }

struct Tile {
    int64_t rows;
    int t, g;   // lane & 15, lane >> 4

    __device__ __forceinline__ bool full(int64_t t0) const { return t0 + 16 <= rows; }
    // x[t0 + t][4 s + g] of a (rows, W) tensor, s = 0..S-1
    template <int S, int W>
    __device__ __forceinline__ void load_fm(const float* base, int64_t t0, float (&v)[S]) const {
        const float* p = base + t0 * W;
        const bool ok = full(t0) || t0 + t < rows;
#pragma unroll
        for (int s = 0; s < S; ++s) v[s] = ok ? p[t * W + 4 * s + g] : 0.f;
    }
    // x[t0 + 4 s + g][col0 + t] of a (rows, W) tensor (t < ncol, else 0), s = 0..3
    template <int W>
    __device__ __forceinline__ void load_tm(const float* base, int64_t t0, int col0, int ncol, float (&v)[4]) const {
        const float* p = base + t0 * W + col0;
        const int cc = t < ncol ? t : 0;
        const bool f = full(t0);
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = (t < ncol && (f || t0 + 4 * s + g < rows)) ? p[(4 * s + g) * W + cc] : 0.f;
    }
    // per-token scalar of token t0 + 4 s + g (token-major), s = 0..3
    __device__ __forceinline__ void load_tm_scalar(const float* base, int64_t t0, float (&v)[4]) const {
        const bool f = full(t0);
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = (f || t0 + 4 * s + g < rows) ? base[t0 + 4 * s + g] : 0.f;
    }
    // the lane's accumulator chunk of token t0 + t is valid (lane groups 0..2 hold the 12 channels)
    __device__ __forceinline__ bool chunk_ok(int64_t t0) const { return g < 3 && t0 + t < rows; }
    __device__ __forceinline__ bool token_ok(int64_t t0) const { return t0 + t < rows; }
};

// Sum of a per-lane value over the 4 lane groups (the 12 channels of the lane's token).
__device__ __forceinline__ float sum_groups(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// Sum over the 16 token lanes of a lane group.
__device__ __forceinline__ float sum_tokens(float v) {
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    return v;
}

// LayerNorm statistics of the lane's token from its 3 feature-major channels (nn.LayerNorm:
// biased variance, eps inside the square root).
__device__ __forceinline__ void ln_stats(const float (&v)[CS], float eps, float& mean, float& rstd) {
    mean = sum_groups(v[0] + v[1] + v[2]) * (1.0f / C);
    float q = 0.f;
#pragma unroll
    for (int s = 0; s < CS; ++s) q = fmaf(v[s] - mean, v[s] - mean, q);
    const float var = sum_groups(q) * (1.0f / C);
    rstd = 1.0f / sqrtf(var + eps);
}

// LayerNorm backward of one token from its accumulator chunk (channels 4 g + i, g < 3; lanes of
// group 3 pass zeros): dxn = dL/dxhat-side gradient of the LN output, xh = normalized input.
//   dx = rstd * (gamma*dxn - mean(gamma*dxn) - xh * mean(gamma*dxn*xh))
__device__ __forceinline__ f4 ln_bwd_chunk(f4 dxn, f4 xh, f4 gm, float rstd) {
    const f4 gd = dxn * gm;
    const float s1 = sum_groups(gd[0] + gd[1] + gd[2] + gd[3]) * (1.0f / C);
    const float s2 = sum_groups(gd[0] * xh[0] + gd[1] * xh[1] + gd[2] * xh[2] + gd[3] * xh[3]) * (1.0f / C);
    f4 dx;
#pragma unroll
    for (int i = 0; i < 4; ++i) dx[i] = rstd * (gd[i] - s1 - xh[i] * s2);
    return dx;
}

// Persistent grids sized to what is resident at once (occupancy query): a grid-stride launch of
// more blocks runs a partial second wave of blocks at a fraction of the occupancy.
inline int resident_blocks(const void* kern, int threads, size_t lds) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    return per_cu * kNumCU;
}

}  // namespace tt
}  // namespace mmni
