// Dev probe: the shader clock and fp64 MFMA rate under a sustained v_mfma_f64_16x16x4_f64 load.
// Each wave runs NCH independent accumulators; FILL integer VALU ops (no fp64) sit between MFMA groups to
// lower the MFMA duty cycle.  Wave 0 of block 0 reads s_memtime (shader clock) and s_memrealtime (100 MHz)
// around the loop, so every line carries the clock the SIMDs actually ran at.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_f64_clock.hip -o scripts/_build/probe_f64_clock
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NCH, int FILL>
__global__ __launch_bounds__(256) void k_mf(double* out, long long* clk, int iters) {
    f64x4 c[NCH];
    for (int k = 0; k < NCH; ++k) c[k] = f64x4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    unsigned u = threadIdx.x * 7u + 1u;
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
#pragma unroll
        for (int f = 0; f < FILL; ++f) u = (u ^ 0x9e3779b9u) + (u >> 3);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    f64x4 s = c[0];
    for (int k = 1; k < NCH; ++k) s += c[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    if (s[0] == 12345.678 || u == 12345u) out[threadIdx.x] = s[1] + u;
}

template <int NCH, int FILL>
static void run(int blocks_per_cu, int cus, double* d, long long* c) {
    const int blocks = cus * blocks_per_cu;
    const int iters = 40000 / NCH;
    k_mf<NCH, FILL><<<blocks, 256>>>(d, c, 100);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_mf<NCH, FILL><<<blocks, 256>>>(d, c, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    const double mfma = (double)blocks * 4 * iters * NCH;
    const double tf = mfma * 2048.0 / (ms * 1e-3) / 1e12;
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    const double cyc_per_mfma = (double)h[0] / ((double)iters * NCH);
    printf("{\"nch\": %d, \"fill\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f, \"shader_ghz\": %.3f, "
           "\"wave_cycles_per_mfma\": %.1f, \"frac_of_78.6\": %.3f}\n",
           NCH, FILL, blocks_per_cu, ms, tf, ghz, cyc_per_mfma, tf / 78.6);
}


template <int NCH>
__global__ __launch_bounds__(256) void k_mf4(double* out, long long* clk, int iters) {
    double c[NCH];
    for (int k = 0; k < NCH; ++k) c[k] = 0.0;
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) c[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[k], 0, 0, 0);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    for (int k = 0; k < NCH; ++k) s += c[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    if (s == 12345.678) out[threadIdx.x] = s;
}

template <int NCH>
static void run4(int blocks_per_cu, int cus, double* d, long long* c) {
    const int blocks = cus * blocks_per_cu;
    const int iters = 160000 / NCH;
    k_mf4<NCH><<<blocks, 256>>>(d, c, 100);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_mf4<NCH><<<blocks, 256>>>(d, c, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    const double mfma = (double)blocks * 4 * iters * NCH;
    const double tf = mfma * 512.0 / (ms * 1e-3) / 1e12;
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    printf("{\"op\": \"4x4x4f64 (512 flop)\", \"nch\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f, "
           "\"shader_ghz\": %.3f, \"wave_cycles_per_mfma\": %.1f}\n",
           NCH, blocks_per_cu, ms, tf, ghz, (double)h[0] / ((double)iters * NCH));
}

// FILLF f64 FMAs (independent of the MFMAs) between MFMA groups in the same wave
template <int NCH, int FILLF>
__global__ __launch_bounds__(256) void k_mff(double* out, long long* clk, int iters) {
    f64x4 c[NCH];
    for (int k = 0; k < NCH; ++k) c[k] = f64x4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    double f[4] = {threadIdx.x * 1e-3, 1.0, 2.0, 3.0};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
#pragma unroll
        for (int g = 0; g < FILLF; ++g) f[g & 3] = __builtin_fma(f[g & 3], 0.9999999, 1e-9);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    f64x4 s = c[0];
    for (int k = 1; k < NCH; ++k) s += c[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
    if (s[0] == 12345.678 || f[0] + f[1] + f[2] + f[3] == 1.5) out[threadIdx.x] = s[1];
}

// co-execution: waves 0-3 of a 512-thread block run MFMA chains, waves 4-7 (same SIMDs) run PK-kind VALU work
// (0: f64 FMA, 1: int32 xor/shift/add), NV instructions per MFMA of the partner
template <int KIND, int NV>
__global__ __launch_bounds__(512) void k_co(double* out, long long* clk, int iters, int mode) {
    const int w = threadIdx.x >> 6;
    if (w < 4) {
        if (mode == 2) return;
        f64x4 c[8];
        for (int k = 0; k < 8; ++k) c[k] = f64x4{0, 0, 0, 0};
        double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
        const long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        f64x4 s = c[0];
        for (int k = 1; k < 8; ++k) s += c[k];
        if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
        if (s[0] == 12345.678) out[threadIdx.x] = s[1];
    } else {
        if (mode == 1) return;
        const long long t0 = __builtin_amdgcn_s_memtime();
        if (KIND == 0) {
            double f[8];
            for (int k = 0; k < 8; ++k) f[k] = k * 1e-3 + threadIdx.x * 1e-9;
            for (int i = 0; i < iters * NV; ++i) {
#pragma unroll
                for (int k = 0; k < 8; ++k) f[k] = __builtin_fma(f[k], 0.9999999, 1e-9);
            }
            double s = 0;
            for (int k = 0; k < 8; ++k) s += f[k];
            if (s == 12345.678) out[threadIdx.x] = s;
        } else {
            unsigned u[8];
            for (int k = 0; k < 8; ++k) u[k] = threadIdx.x * 7u + k;
            for (int i = 0; i < iters * NV; ++i) {
#pragma unroll
                for (int k = 0; k < 8; ++k) u[k] = (u[k] ^ 0x9e3779b9u) + (u[k] >> 3);
            }
            unsigned s = 0;
            for (int k = 0; k < 8; ++k) s += u[k];
            if (s == 12345u) out[threadIdx.x] = s;
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0 && blockIdx.x == 0 && w == 4) clk[1] = t1 - t0;
    }
}

template <int KIND, int NV>
static void run_co(int cus, double* d, long long* c) {
    const int iters = 4000;
    float ms[3];
    long long h[3][2];
    for (int mode = 0; mode < 3; ++mode) {       // 0 both, 1 MFMA waves only, 2 VALU waves only
        k_co<KIND, NV><<<cus, 512>>>(d, c, 50, mode);
        (void)hipDeviceSynchronize();
        (void)hipMemset(c, 0, 16);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        k_co<KIND, NV><<<cus, 512>>>(d, c, iters, mode);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[mode], e0, e1);
        (void)hipMemcpy(h[mode], c, 16, hipMemcpyDeviceToHost);
    }
    printf("{\"coexec\": \"%s\", \"partner_valu_per_mfma\": %d, \"both_ms\": %.3f, \"mfma_only_ms\": %.3f, "
           "\"valu_only_ms\": %.3f, \"both_over_max\": %.3f, \"both_over_sum\": %.3f, \"mfma_cyc_both\": %lld, "
           "\"mfma_cyc_alone\": %lld, \"valu_cyc_both\": %lld, \"valu_cyc_alone\": %lld}\n",
           KIND == 0 ? "f64 fma" : "int32", NV, ms[0], ms[1], ms[2], ms[0] / (ms[1] > ms[2] ? ms[1] : ms[2]),
           ms[0] / (ms[1] + ms[2]), h[0][0], h[1][0], h[0][1], h[2][1]);
}

template <int NCH, int FILLF>
static void runf(int cus, double* d, long long* c) {
    const int iters = 40000 / NCH;
    k_mff<NCH, FILLF><<<cus, 256>>>(d, c, 100);
    (void)hipDeviceSynchronize();
    k_mff<NCH, FILLF><<<cus, 256>>>(d, c, iters);
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("{\"same_wave_f64_fma_fill\": %d, \"nch\": %d, \"wave_cycles_per_mfma\": %.1f}\n", FILLF, NCH,
           (double)h[0] / ((double)iters * NCH));
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double* d;
    long long* c;
    (void)hipMalloc(&d, 1 << 16);
    (void)hipMalloc(&c, 16);
    if (getenv("PROBE_DEP")) {              // dependent-chain issue interval: 1 or 2 chains, 1 or 2 waves per SIMD
        run<1, 0>(1, cus, d, c);
        run<2, 0>(1, cus, d, c);
        run<1, 0>(2, cus, d, c);
        run<2, 0>(2, cus, d, c);
        run<1, 8>(1, cus, d, c);
        return 0;
    }
    if (getenv("PROBE_CO")) {
        runf<8, 8>(cus, d, c);
        runf<8, 16>(cus, d, c);
        runf<8, 32>(cus, d, c);
        run_co<0, 1>(cus, d, c);
        run_co<0, 4>(cus, d, c);
        run_co<1, 1>(cus, d, c);
        run_co<1, 4>(cus, d, c);
        return 0;
    }
    run<4, 0>(1, cus, d, c);
    run<8, 0>(1, cus, d, c);
    run<4, 0>(2, cus, d, c);
    run<4, 0>(8, cus, d, c);
    run<8, 8>(1, cus, d, c);
    run<8, 16>(1, cus, d, c);
    run<8, 32>(1, cus, d, c);
    run<8, 64>(1, cus, d, c);
    run<8, 128>(1, cus, d, c);
    run<4, 0>(1, cus, d, c);
    run<16, 0>(1, cus, d, c);
    run<8, 0>(2, cus, d, c);
    run<8, 0>(4, cus, d, c);
    run4<8>(1, cus, d, c);
    run4<16>(1, cus, d, c);
    run4<8>(2, cus, d, c);
    run4<8>(4, cus, d, c);
    return 0;
}
