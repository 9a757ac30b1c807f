// Issue-cost micro-benchmark for the window-attention inner loops: v_exp_f32 vs v_pk_fma_f32 vs a
// mix, at a chosen number of waves per SIMD.  Build: hipcc -O3 --offload-arch=gfx950 -o
// /tmp/ubench_valu scripts/ubench_valu.hip ; run: ubench_valu  (prints cycles per wave-instruction)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int NEXP, int NPK>
__global__ __launch_bounds__(256) void mix_kernel(float* out, int iters, float seed) {
    f2 a[8], b = (f2){seed * 0.5f, seed * 0.25f}, c = (f2){1e-7f, 2e-7f};
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (f2){seed + threadIdx.x * 1e-6f + i, seed - i};
        e[i] = seed * 1e-3f * i;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NPK; ++i) a[i & 7] = __builtin_elementwise_fma(a[i & 7], b, c);
#pragma unroll
        for (int i = 0; i < NEXP; ++i) e[i & 7] = __builtin_amdgcn_exp2f(e[i & 7]) * -0.5f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y + e[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NEXP, int NPK>
static void run(const char* name, int waves_per_simd) {
    float* out;
    hipMalloc(&out, 1024 * 4);
    const int iters = 4096;
    const int blocks = 256 * waves_per_simd;   // 256-thread blocks = 4 waves, one per SIMD
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    mix_kernel<NEXP, NPK><<<blocks, 256>>>(out, iters, 1.0f);
    hipEventRecord(t0);
    mix_kernel<NEXP, NPK><<<blocks, 256>>>(out, iters, 1.0f);
    hipEventRecord(t1);
    hipEventSynchronize(t1);
    float ms;
    hipEventElapsedTime(&ms, t0, t1);
    // cycles per SIMD at 2.4 GHz / (iterations x waves per SIMD)
    const double cyc = ms * 1e-3 * 2.4e9 / ((double)iters * waves_per_simd);
    printf("%-22s waves/SIMD %d: %8.3f ms  %7.1f cyc per iteration per wave  (%d exp + %d pk_fma)\n", name,
           waves_per_simd, ms, cyc, NEXP, NPK);
    hipFree(out);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<8, 0>("exp x8", w);
        run<0, 8>("pk_fma x8", w);
        run<0, 16>("pk_fma x16", w);
        run<8, 8>("exp x8 + pk x8", w);
        run<8, 20>("exp x8 + pk x20", w);
        run<8, 36>("exp x8 + pk x36", w);
    }
    return 0;
}
