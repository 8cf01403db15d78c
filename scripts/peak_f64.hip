// Measures the fp64 peaks the regression and separable kernels are priced against on gfx950:
//   v_mfma_f64_16x16x4_f64 (2048 flop/instr) back-to-back with independent accumulators, and
//   v_fma_f64 (VALU, 2 flop/lane) with independent chains.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/peak_f64.hip -o scripts/_build/peak_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a0, double b0) {
    f64x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    const f64x4 s = c0 + c1 + c2 + c3;
    if (s[0] == 12345.678) out[threadIdx.x] = s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void k_fma(double* out, int iters, double a0, double b0) {
    double c[8];
    for (int k = 0; k < 8; ++k) c[k] = k * 1e-3 + threadIdx.x * 1e-9;
    const double a = a0, b = b0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_fma(c[k], a, b);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k];
    if (s == 12345.678) out[threadIdx.x] = s;
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    double* out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = cus * 8;           // 8 blocks x 4 waves per CU: 8 waves per SIMD
    const int iters = 20000;
    float ms;
    k_mfma<<<blocks, 256>>>(out, 100, 1.0, 1.0);
    hipEventRecord(e0);
    k_mfma<<<blocks, 256>>>(out, iters, 1.0000001, 0.9999999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double mfma_flop = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * 2048.0;
    printf("{\"cus\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, ", cus, mfma_flop / (ms * 1e-3) / 1e12);
    k_fma<<<blocks, 256>>>(out, 100, 1.0, 1.0);
    hipEventRecord(e0);
    k_fma<<<blocks, 256>>>(out, iters, 0.9999999, 1e-9);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double fma_flop = (double)blocks * 256 * iters * 8 * 2.0;
    printf("\"valu_fma_f64_tflops\": %.2f}\n", fma_flop / (ms * 1e-3) / 1e12);
    return 0;
}
