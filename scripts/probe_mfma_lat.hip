// Dev probe: issue cost and dependent latency of v_mfma_f64_16x16x4_f64 on one SIMD, in shader clocks (s_memtime):
// one wave per SIMD running a single dependent accumulator chain, 2 or 4 interleaved chains, and a dependent chain
// next to a VALU-only partner wave on the same SIMD (waves w and w+4 of a 512-thread block share a SIMD).
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probe_mfma_lat.hip -o scripts/_build/probe_mfma_lat
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NCH, bool PARTNER_VALU, bool PARTNER_MFMA>
__global__ __launch_bounds__(512) void k_lat(double* out, long long* cyc, int iters) {
    const int w = threadIdx.x >> 6;
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    if (w < 4) {
        f64x4 c[NCH];
        for (int k = 0; k < NCH; ++k) c[k] = f64x4{0, 0, 0, 0};
        const long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < NCH; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
        }
        f64x4 s = c[0];
        for (int k = 1; k < NCH; ++k) s += c[k];
        const long long t1 = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0 && blockIdx.x == 0 && w == 0) cyc[0] = t1 - t0;
        if (s[0] == 12345.678) out[threadIdx.x] = s[1];
    } else if (PARTNER_VALU) {
        double c[8];
        for (int k = 0; k < 8; ++k) c[k] = k * 1e-3 + threadIdx.x * 1e-9;
        const long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters * 4; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __builtin_fma(c[k], 0.9999999, 1e-9);
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        double s = 0;
        for (int k = 0; k < 8; ++k) s += c[k];
        if ((threadIdx.x & 63) == 0 && blockIdx.x == 0 && w == 4) cyc[1] = t1 - t0;
        if (s == 12345.678) out[threadIdx.x] = s;
    } else if (PARTNER_MFMA) {
        f64x4 c = f64x4{0, 0, 0, 0};
        for (int i = 0; i < iters; ++i) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
        if (c[0] == 12345.678) out[threadIdx.x] = c[1];
    }
}

template <int NCH, bool PV, bool PM>
static void run(const char* name, double* d, long long* c, int cus) {
    const int iters = 4096 / NCH;
    k_lat<NCH, PV, PM><<<cus, 512>>>(d, c, 16);
    (void)hipDeviceSynchronize();
    (void)hipMemset(c, 0, 16);
    k_lat<NCH, PV, PM><<<cus, 512>>>(d, c, iters);
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("{\"case\": \"%s\", \"mfma\": %d, \"cycles_per_mfma\": %.1f, \"partner_valu_cycles_per_fma\": %.2f}\n", name,
           iters * NCH, (double)h[0] / (iters * NCH), PV ? (double)h[1] / (iters * 4.0 * 8) : 0.0);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double* d;
    long long* c;
    (void)hipMalloc(&d, 1 << 16);
    (void)hipMalloc(&c, 16);
    run<1, false, false>("1 chain, alone", d, c, cus);
    run<2, false, false>("2 chains, alone", d, c, cus);
    run<4, false, false>("4 chains, alone", d, c, cus);
    run<8, false, false>("8 chains, alone", d, c, cus);
    run<1, true, false>("1 chain + VALU partner", d, c, cus);
    run<4, true, false>("4 chains + VALU partner", d, c, cus);
    run<1, false, true>("1 chain + MFMA-chain partner", d, c, cus);
    return 0;
}
