// Semantics check of the cross-lane primitives the merged window-attention backward reduces with
// (v_permlane32_swap, v_permlane16_swap, DPP row_ror:8 / row_half_mirror / quad perms).
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/check_permlane scripts/check_permlane.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* out) {
    const int l = threadIdx.x;
    unsigned a = __float_as_uint((float)l), b = __float_as_uint((float)(100 + l));
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto s = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[l] = __uint_as_float(r[0]);
    out[l + 64] = __uint_as_float(r[1]);
    out[l + 128] = __uint_as_float(s[0]);
    out[l + 192] = __uint_as_float(s[1]);
    const float x = (float)l;
    out[l + 256] = __builtin_amdgcn_update_dpp(0.f, x, 0x128, 0xf, 0xf, false);
    out[l + 320] = __builtin_amdgcn_update_dpp(0.f, x, 0x141, 0xf, 0xf, false);
    out[l + 384] = __builtin_amdgcn_update_dpp(0.f, x, 0x4E, 0xf, 0xf, false);
    out[l + 448] = __builtin_amdgcn_update_dpp(0.f, x, 0xB1, 0xf, 0xf, false);
}
int main() {
    float* d;
    hipMalloc(&d, 512 * 4);
    k<<<1, 64>>>(d);
    float h[512];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[8] = {"p32 vdst", "p32 vsrc", "p16 vdst", "p16 vsrc", "ror8", "half_mirror", "qxor2", "qxor1"};
    for (int t = 0; t < 8; ++t) {
        printf("%-12s", names[t]);
        for (int l = 0; l < 64; ++l) printf(" %g", h[t * 64 + l]);
        printf("\n");
    }
    return 0;
}
