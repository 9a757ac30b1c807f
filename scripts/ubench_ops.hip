// Issue-cost micro-benchmark of the merged window-attention backward's non-FMA instructions:
// v_mov_b64, v_permlane32_swap, v_permlane16_swap, v_add_f32 with a DPP operand, v_cndmask, against
// v_pk_fma_f32 and v_exp_f32, at 1 and 2 waves per SIMD.  Each loop body issues 8 independent
// instructions of one kind (8 register chains).  Build: hipcc -O3 --offload-arch=gfx950 -o
// /tmp/ubench_ops scripts/ubench_ops.hip ; run: /tmp/ubench_ops (cycles per wave-instruction at 2.4 GHz)
#include <hip/hip_runtime.h>
#include <cstdio>

enum Op { PKFMA, EXP, MOV64, PERM32, PERM16, DPPADD, CNDMASK, ADDF32, CNDSGPR, BFI, BPERM, MOVDPP };

template <int OP>
__global__ __launch_bounds__(256) void op_kernel(float* out, int iters, float seed) {
    float r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = seed + threadIdx.x * 1e-6f + i;
    unsigned long long msk;
    asm volatile("v_cmp_gt_u32 %0, 32, %1" : "=s"(msk) : "v"((unsigned)threadIdx.x));
    const unsigned vm = (threadIdx.x & 8) ? ~0u : 0u;
    const unsigned vaddr = ((threadIdx.x ^ 8) & 63) * 4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float& a = r[2 * i];
            float& b = r[2 * i + 1];
            if constexpr (OP == PKFMA) {
                asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(*reinterpret_cast<double*>(&a)));
            } else if constexpr (OP == EXP) {
                asm volatile("v_exp_f32 %0, %0" : "+v"(a));
            } else if constexpr (OP == MOV64) {
                asm volatile("v_mov_b64 %0, 0" : "=v"(*reinterpret_cast<double*>(&a)));
            } else if constexpr (OP == PERM32) {
                asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
            } else if constexpr (OP == PERM16) {
                asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
            } else if constexpr (OP == DPPADD) {
                asm volatile("v_add_f32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b));
            } else if constexpr (OP == CNDMASK) {
                asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));   // vcc: whatever it holds
            } else if constexpr (OP == ADDF32) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
            } else if constexpr (OP == CNDSGPR) {   // select on an SGPR-pair lane mask set once
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(msk));
            } else if constexpr (OP == BFI) {       // bit-select with a per-lane mask VGPR
                asm volatile("v_bfi_b32 %0, %2, %1, %0" : "+v"(a) : "v"(b), "v"(vm));
            } else if constexpr (OP == BPERM) {     // LDS crossbar lane exchange
                asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a) : "v"(vaddr));
            } else if constexpr (OP == MOVDPP) {
                asm volatile("v_mov_b32_dpp %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf" : "=v"(a) : "v"(b));
            }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += r[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int OP>
static void run(const char* name, int waves_per_simd) {
    float* out;
    hipMalloc(&out, 1024 * 4);
    const int iters = 8192;
    const int blocks = 256 * waves_per_simd;   // 256-thread blocks = 4 waves, one per SIMD
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    op_kernel<OP><<<blocks, 256>>>(out, iters, 1.0f);
    hipEventRecord(t0);
    op_kernel<OP><<<blocks, 256>>>(out, iters, 1.0f);
    hipEventRecord(t1);
    hipEventSynchronize(t1);
    float ms;
    hipEventElapsedTime(&ms, t0, t1);
    // SIMD cycles at 2.4 GHz per wave-instruction (8 per iteration, waves_per_simd waves per SIMD)
    const double cyc = ms * 1e-3 * 2.4e9 / ((double)iters * 8 * waves_per_simd);
    printf("%-10s waves/SIMD %d: %8.3f ms  %6.2f cyc per wave-instruction\n", name, waves_per_simd, ms, cyc);
    hipFree(out);
}

int main() {
    for (int w : {1, 2}) {
        run<PKFMA>("pk_fma", w);
        run<EXP>("exp", w);
        run<MOV64>("mov_b64", w);
        run<PERM32>("perm32", w);
        run<PERM16>("perm16", w);
        run<DPPADD>("dpp_add", w);
        run<CNDMASK>("cndmask", w);
        run<ADDF32>("add_f32", w);
        run<CNDSGPR>("cnd_sgpr", w);
        run<BFI>("bfi", w);
        run<BPERM>("bperm+wait", w);
        run<MOVDPP>("mov_dpp", w);
    }
    return 0;
}
