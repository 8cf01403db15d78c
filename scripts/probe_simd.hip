// Dev probe: which SIMD each wave of a 512-thread (8-wave) workgroup lands on (HW_REG_HW_ID bits [5:4] on gfx9),
// for a few workgroups.  Build: hipcc --offload-arch=gfx950 -O2 scripts/probe_simd.hip -o scripts/_build/probe_simd
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void k_where(int* out) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | ((32 - 1) << 11));   // HW_REG_HW_ID, all bits
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        out[blockIdx.x * 8 + w] = (int)hw;
    }
}

int main() {
    int* d;
    const int nb = 512;
    (void)hipMalloc(&d, nb * 8 * sizeof(int));
    k_where<<<nb, 512, 96 * 1024>>>(d);
    int h[nb * 8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int same_w_w4 = 0, same_pair = 0;
    for (int b = 0; b < nb; ++b) {
        for (int w = 0; w < 4; ++w) same_w_w4 += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 4] >> 4) & 3);
        for (int w = 0; w < 8; w += 2) same_pair += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 1] >> 4) & 3);
    }
    for (int b = 0; b < 4; ++b) {
        printf("block %d simd of waves 0..7:", b);
        for (int w = 0; w < 8; ++w) printf(" %d", (h[b * 8 + w] >> 4) & 3);
        printf("   (cu %d)\n", (h[b * 8] >> 8) & 15);
    }
    printf("{\"waves_w_and_w+4_same_simd\": %d, \"waves_2k_and_2k+1_same_simd\": %d, \"of\": %d}\n", same_w_w4, same_pair,
           nb * 4);
    return 0;
}
