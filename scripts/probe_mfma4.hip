// Dev probe: v_mfma_f64_4x4x4_4b_f64 (four independent 4x4x4 blocks a wave, 512 flop) against
// v_mfma_f64_16x16x4_f64 (2 048 flop) on gfx950.
//   layout:  raw per-lane A, B, C -> D of one 4x4x4_4b on random wide-exponent operands, written to a file for
//            scripts/probe_mfma4.py (operand layout and the accumulation order of each output);
//   rate:    back-to-back issue, NCH accumulators a wave, 1 / 2 waves per SIMD, with and without one ds_read_b64
//            (the A operand from LDS, read LA MFMAs ahead) per MFMA; the 16x16x4 form alike for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_mfma4.hip -o scripts/_build/probe_mfma4
// Run:   scripts/_build/probe_mfma4 <layout.bin>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const double* A, const double* B, const double* C, double* D) {
    const int l = threadIdx.x;
    D[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], C[l], 0, 0, 0);
}

// NCH accumulators, LDS=1: the A operand of every MFMA from LDS (one ds_read_b64, LA ahead)
template <int NCH, int LDS, bool BIG>
__global__ __launch_bounds__(256) void k_rate(double* out, long long* clk, int iters) {
    __shared__ double xs[4][64 * 33];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int i = l; i < 64 * 33; i += 64) xs[w][i] = 1.0 + 1e-9 * i;
    __syncthreads();
    double c4[NCH];
    f64x4 c16[NCH];
    for (int k = 0; k < NCH; ++k) { c4[k] = 0.0; c16[k] = f64x4{0, 0, 0, 0}; }
    double b = 1.0 - threadIdx.x * 1e-9;
    const double* src = &xs[w][(l & 3) * 33 + 4 * ((l >> 2) & 3)];
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        double av[NCH];
        if (LDS) {
#pragma unroll
            for (int k = 0; k < NCH; ++k) av[k] = src[(k * 5 + i) & 31];
        }
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const double a = LDS ? av[k] : 1.0 + threadIdx.x * 1e-9;
            if (BIG) c16[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c16[k], 0, 0, 0);
            else c4[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c4[k], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    for (int k = 0; k < NCH; ++k) s += c4[k] + c16[k][0] + c16[k][3];
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    if (s == 12345.678) out[threadIdx.x] = s;
}

template <int NCH, int LDS, bool BIG>
static void rate(int waves_per_simd, int cus, double* d, long long* c) {
    const int blocks = cus * waves_per_simd;
    const int iters = (BIG ? 20000 : 80000) / NCH;
    k_rate<NCH, LDS, BIG><<<blocks, 256>>>(d, c, 50);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_rate<NCH, LDS, BIG><<<blocks, 256>>>(d, c, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    const double flop = (double)blocks * 4 * iters * NCH * (BIG ? 2048.0 : 512.0);
    const double tf = flop / (ms * 1e-3) / 1e12;
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    printf("{\"op\": \"%s\", \"nch\": %d, \"lds_a\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f, "
           "\"shader_ghz\": %.3f, \"wave_cycles_per_mfma\": %.1f, \"frac_of_78.6\": %.3f}\n",
           BIG ? "16x16x4f64" : "4x4x4_4b_f64", NCH, LDS, waves_per_simd, ms, tf, ghz,
           (double)h[0] / ((double)iters * NCH), tf / 78.6);
    fflush(stdout);
}

int main(int argc, char** argv) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    // layout: 8 trials of random wide-exponent operands
    {
        const int T = 8;
        std::vector<double> h(4 * 64 * T);
        srand(12345);
        auto rnd = [] {
            const double u = (rand() + 0.5) / (RAND_MAX + 1.0) - 0.5;
            const int e = rand() % 41 - 20;
            return u * __builtin_ldexp(1.0, e);
        };
        double *dA, *dB, *dC, *dD;
        (void)hipMalloc(&dA, 512);
        (void)hipMalloc(&dB, 512);
        (void)hipMalloc(&dC, 512);
        (void)hipMalloc(&dD, 512);
        for (int t = 0; t < T; ++t) {
            double* A = &h[(4 * t + 0) * 64];
            double* B = &h[(4 * t + 1) * 64];
            double* C = &h[(4 * t + 2) * 64];
            double* D = &h[(4 * t + 3) * 64];
            for (int l = 0; l < 64; ++l) { A[l] = rnd(); B[l] = rnd(); C[l] = rnd(); }
            (void)hipMemcpy(dA, A, 512, hipMemcpyHostToDevice);
            (void)hipMemcpy(dB, B, 512, hipMemcpyHostToDevice);
            (void)hipMemcpy(dC, C, 512, hipMemcpyHostToDevice);
            k_layout<<<1, 64>>>(dA, dB, dC, dD);
            (void)hipMemcpy(D, dD, 512, hipMemcpyDeviceToHost);
        }
        if (argc > 1) {
            FILE* f = fopen(argv[1], "wb");
            if (f) { fwrite(h.data(), 8, h.size(), f); fclose(f); }
        }
        (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dC); (void)hipFree(dD);
    }
    double* d;
    long long* c;
    (void)hipMalloc(&d, 1 << 16);
    (void)hipMalloc(&c, 16);
    rate<1, 0, false>(1, cus, d, c);
    rate<2, 0, false>(1, cus, d, c);
    rate<4, 0, false>(1, cus, d, c);
    rate<8, 0, false>(1, cus, d, c);
    rate<1, 0, false>(2, cus, d, c);
    rate<4, 0, false>(2, cus, d, c);
    rate<8, 0, false>(2, cus, d, c);
    rate<4, 1, false>(1, cus, d, c);
    rate<8, 1, false>(1, cus, d, c);
    rate<4, 1, false>(2, cus, d, c);
    rate<8, 1, false>(2, cus, d, c);
    rate<1, 0, true>(1, cus, d, c);
    rate<4, 0, true>(1, cus, d, c);
    rate<8, 0, true>(1, cus, d, c);
    rate<8, 0, true>(2, cus, d, c);
    rate<8, 1, true>(2, cus, d, c);
    return 0;
}
