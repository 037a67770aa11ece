// Probe of the cross-lane primitives the PPO2 FD kernel's weight-gradient butterflies use
// (v_permlane16/32_swap_b32, DPP row_mirror / row_half_mirror / quad_perm): prints, for input
// x[l] = l, y[l] = 100 + l, what each primitive returns per lane. Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(float *o) {
    const int l = threadIdx.x;
    const unsigned x = __float_as_uint((float)l), y = __float_as_uint(100.f + l);
    const auto a = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    o[0 * 64 + l] = __uint_as_float(a[0]);
    o[1 * 64 + l] = __uint_as_float(a[1]);
    o[2 * 64 + l] = __uint_as_float(b[0]);
    o[3 * 64 + l] = __uint_as_float(b[1]);
    o[4 * 64 + l] = __uint_as_float(__builtin_amdgcn_update_dpp(0u, x, 0x140, 0xF, 0xF, true));
    o[5 * 64 + l] = __uint_as_float(__builtin_amdgcn_update_dpp(0u, x, 0x141, 0xF, 0xF, true));
    o[6 * 64 + l] = __uint_as_float(__builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, true));
    o[7 * 64 + l] = __uint_as_float(__builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, true));
}
int main() {
    float *d, h[8 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    probe<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char *nm[8] = {"pl16 r0", "pl16 r1", "pl32 r0", "pl32 r1", "mirror", "halfmir", "xor2", "xor1"};
    for (int k = 0; k < 8; ++k) {
        printf("%-8s", nm[k]);
        for (int l = 0; l < 64; ++l) printf(" %g", h[k * 64 + l]);
        printf("\n");
    }
    return hipFree(d) == hipSuccess ? 0 : 3;
}
