// Internal helpers shared by the libmmni.so translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdint.h>
#include "../../include/mmni.h"

namespace mmni {

// Thread-local last-error message behind mmni_last_error().
void set_error(const char* fmt, ...);

#define MMNI_ARG_CHECK(cond, ...)                 \
    do {                                          \
        if (!(cond)) {                            \
            ::mmni::set_error(__VA_ARGS__);       \
            return -1;                            \
        }                                         \
    } while (0)

inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// Number of resident 64-lane waves a launch should aim for: 256 CUs x occupancy.
constexpr int kNumCU = 256;

// out[j] = sum_b part[b][j] over a (nparts, ncols) slab in a fixed order (deterministic); columns
// j >= split go to out2[j - split] (tokenops.hip).
void column_sum(const float* part, int nparts, int ncols, float* out, int split, float* out2, hipStream_t s);
// Column sums of one partial matrix into up to kMax destination segments: columns
// [end[k-1], end[k]) go to dst[k] (end[-1] = 0; a null dst drops them), written or, with
// accumulate, added.  Same fixed-order reduction as column_sum.
struct ColSegs {
    static constexpr int kMax = 6;
    int n;
    int end[kMax];
    float* dst[kMax];
    int accumulate;
};
void column_sum_segs(const float* part, int nparts, int ncols, const ColSegs& segs, hipStream_t s);

// Row-GEMM weight gradient and row LayerNorm backward (encoder.hip), also used by the token ops
// for short row counts (a few hundred to ~64k rows: the deep Swin stages), where the row-chunk
// grid keeps many workgroups busy.  Workspace bytes first; the launches return 0 / hipError.
size_t enc_rowgemm_dw_workspace(int64_t rows, int N, int K);
int enc_rowgemm_dw(int64_t rows, int N, int K, const float* x, int64_t ldx, const float* dy, int64_t lddy,
                   const float* gamma, const float* beta, const float* mean, const float* rstd, float* dw, float* db,
                   void* workspace, hipStream_t s);
size_t enc_row_ln_bwd_workspace(int64_t rows, int C);
int enc_row_ln_bwd(int64_t rows, int C, const float* dxn, int64_t lddxn, const float* x, int64_t ldx,
                   const float* gamma, const float* mean, const float* rstd, const float* dres, int64_t ldres,
                   float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace, hipStream_t s);
// the same with the input gradient dxn in fp32 (dxn_bf16 = 0) or bf16 (1)
int enc_row_ln_bwd_t(int64_t rows, int C, const void* dxn, int dxn_bf16, int64_t lddxn, const float* x, int64_t ldx,
                     const float* gamma, const float* mean, const float* rstd, const float* dres, int64_t ldres,
                     float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace, hipStream_t s);
constexpr int64_t kSmallRows = 65536;   // token ops at or below this row count take the encoder kernels

}  // namespace mmni
