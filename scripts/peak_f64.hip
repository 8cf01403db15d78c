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

__global__ __launch_bounds__(256) void k_mad64(unsigned long long* out, int iters, unsigned a0) {
    unsigned long long c[8];
    for (int k = 0; k < 8; ++k) c[k] = threadIdx.x + k;
    unsigned a = a0 + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = (unsigned long long)a * (unsigned)(c[k] >> 7) + (c[k] & 0xffffffffull);
    }
    unsigned long long s = 0;
    for (int k = 0; k < 8; ++k) s += c[k];
    if (s == 12345) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_xor(unsigned* out, int iters, unsigned a0) {
    unsigned c[8];
    for (int k = 0; k < 8; ++k) c[k] = threadIdx.x * 7 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = (c[k] ^ a0) + (c[k] >> 3);
    }
    unsigned s = 0;
    for (int k = 0; k < 8; ++k) s += c[k];
    if (s == 12345) out[threadIdx.x] = s;
}

// dependent-issue latency of v_fma_f64: NCH independent chains in one wave per SIMD (cus * 4 waves)
template <int NCH>
__global__ __launch_bounds__(64) void k_fma_chain(double* out, int iters) {
    double c[NCH];
    for (int k = 0; k < NCH; ++k) c[k] = k * 1e-3 + threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) c[k] = __builtin_fma(c[k], 0.9999999, 1e-9);
    }
    double s = 0;
    for (int k = 0; k < NCH; ++k) s += c[k];
    if (s == 12345.678) out[threadIdx.x] = s;
}

// co-execution probe: waves 0-3 of a 512-thread block run k_mfma's loop, waves 4-7 run k_fma's loop (one of
// each per SIMD).  Time ~ max(mfma, fma) if the fp64 matrix and vector pipes run concurrently, ~ the sum if not.
__global__ __launch_bounds__(512) void k_coexec(double* out, int iters, double a0, double b0) {
    if ((threadIdx.x >> 6) < 4) {
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
    } else {
        double c[8];
        for (int k = 0; k < 8; ++k) c[k] = k * 1e-3 + threadIdx.x * 1e-9;
        const double a = 0.9999999, b = 1e-9;
        // 8 fma per iteration per wave vs 4 mfma: scaled so each half alone takes about as long
        for (int i = 0; i < 4 * iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __builtin_fma(c[k], a, b);
        }
        double s = 0;
        for (int k = 0; k < 8; ++k) s += c[k];
        if (s == 12345.678) out[threadIdx.x] = s;
    }
}

static float time_it(void (*launch)(int), int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch(100);
    (void)hipEventRecord(e0);
    launch(iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

static double* g_out;
static int g_blocks;

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipMalloc(&g_out, 4096);
    g_blocks = cus * 8;                    // 8 blocks x 4 waves per CU: 8 waves per SIMD
    const int iters = 20000;
    const double waves = (double)g_blocks * 4;
    const float t_mfma = time_it([](int it) { k_mfma<<<g_blocks, 256>>>(g_out, it, 1.0000001, 0.9999999); }, iters);
    const float t_fma = time_it([](int it) { k_fma<<<g_blocks, 256>>>(g_out, it, 0.9999999, 1e-9); }, iters);
    const float t_mad = time_it([](int it) { k_mad64<<<g_blocks, 256>>>((unsigned long long*)g_out, it, 3u); }, iters);
    const float t_xor = time_it([](int it) { k_xor<<<g_blocks, 256>>>((unsigned*)g_out, it, 5u); }, iters);
    // co-execution: 4 MFMA waves + 4 FMA waves per SIMD pair-up in one block (cus*4 blocks = 8 waves/SIMD)
    const float t_co = time_it([](int it) { k_coexec<<<g_blocks / 2, 512>>>(g_out, it, 1.0000001, 0.9999999); }, iters);
    const float t_m4 = time_it([](int it) { k_mfma<<<g_blocks / 2, 256>>>(g_out, it, 1.0000001, 0.9999999); }, iters);
    const float t_f4 = time_it([](int it) { k_fma<<<g_blocks / 2, 256>>>(g_out, 4 * it, 0.9999999, 1e-9); }, iters);
    printf("{\"coexec_ms\": %.3f, \"mfma_alone_ms\": %.3f, \"fma_alone_ms\": %.3f, \"coexec_over_max\": %.3f, "
           "\"coexec_over_sum\": %.3f}\n", t_co, t_m4, t_f4, t_co / (t_m4 > t_f4 ? t_m4 : t_f4), t_co / (t_m4 + t_f4));
    // fma latency: cycles per dependent step, from one wave per SIMD at NCH = 1, 2, 4, 8 chains (clock from the
    // 8-chain, issue-bound case: 4 cycles per wave-fma assumed there)
    {
        static int it2 = 200000;
        const float l1 = time_it([](int it) { k_fma_chain<1><<<g_blocks / 2, 64>>>(g_out, it2 * it / 20000); }, iters);
        const float l2 = time_it([](int it) { k_fma_chain<2><<<g_blocks / 2, 64>>>(g_out, it2 * it / 20000); }, iters);
        const float l4 = time_it([](int it) { k_fma_chain<4><<<g_blocks / 2, 64>>>(g_out, it2 * it / 20000); }, iters);
        const float l8 = time_it([](int it) { k_fma_chain<8><<<g_blocks / 2, 64>>>(g_out, it2 * it / 20000); }, iters);
        const double cyc8 = 8.0 * 4.0;             // cycles per iteration at 8 chains if issue-bound
        printf("{\"fma_chain_ms\": [%.3f, %.3f, %.3f, %.3f], \"cycles_per_dependent_fma_1chain\": %.1f, "
               "\"cycles_per_iter_2chain\": %.1f, \"cycles_per_iter_4chain\": %.1f}\n", l1, l2, l4, l8,
               l1 / l8 * cyc8, l2 / l8 * cyc8, l4 / l8 * cyc8);
    }
    // wave-instructions per second for 8 independent chains per iteration
    const double wi = waves * iters * 8;
    printf("{\"cus\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, \"valu_fma_f64_tflops\": %.2f, "
           "\"fma_f64_Gwave_instr_per_s\": %.1f, \"mad_u64_u32_Gwave_instr_per_s\": %.1f, "
           "\"xad_shift_Gwave_instr_per_s\": %.1f}\n",
           cus, waves * iters * 4 * 2048.0 / (t_mfma * 1e-3) / 1e12, waves * 64 * iters * 8 * 2.0 / (t_fma * 1e-3) / 1e12,
           wi / (t_fma * 1e-3) / 1e9, wi / (t_mad * 1e-3) / 1e9, 2 * wi / (t_xor * 1e-3) / 1e9);
    return 0;
}
