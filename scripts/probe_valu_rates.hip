// Dev probe: VALU issue cost per instruction class on one SIMD at 1, 2, 4 and 8 waves per SIMD, in shader clocks
// (s_memtime), to price the normal generator's instruction mix: fp64 fma / mul / add, int32
// bit operations, v_mad_u64_u32 (Philox), conversions, and mixes of them.  Each wave runs 8 independent chains
// of one instruction (inline asm, so the instruction is exactly the one named); a 256 k-thread block per CU puts
// k waves on every SIMD (k = 8: two 1024-thread blocks per CU).  cycles/instr/SIMD = wave time / (instructions per wave x k).
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probe_valu_rates.hip -o scripts/_build/probe_valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

enum Op { FMA64, MUL64, ADD64, BITOP3, XOR32, MAD64, CVT64, FMA32, MIX_FMA_BIT, MIX_FMA_MAD, DEP_FMA64, MIX_2FMA_1BIT };

template <int OP>
__device__ __forceinline__ void body(double (&c)[8], uint32_t (&x)[8], uint64_t (&p)[8], float (&f)[8], double a,
                                     double b, uint32_t y, uint32_t z) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (OP == FMA64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[k]) : "v"(a), "v"(b));
        if (OP == MUL64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(c[k]) : "v"(a));
        if (OP == ADD64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(c[k]) : "v"(b));
        if (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[k]) : "v"(y), "v"(z));
        if (OP == XOR32) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[k]) : "v"(y));
        if (OP == MAD64) asm volatile("v_mad_u64_u32 %0, s[90:91], %1, %2, %0" : "+v"(p[k]) : "v"(y), "v"(z) : "s90", "s91");
        if (OP == CVT64) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(c[k]) : "v"(x[k]));
        if (OP == FMA32) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[k]) : "v"((float)a), "v"((float)b));
        if (OP == MIX_FMA_BIT) {
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[k]) : "v"(a), "v"(b));
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[k]) : "v"(y), "v"(z));
        }
        if (OP == MIX_FMA_MAD) {
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[k]) : "v"(a), "v"(b));
            asm volatile("v_mad_u64_u32 %0, s[90:91], %1, %2, %0" : "+v"(p[k]) : "v"(y), "v"(z) : "s90", "s91");
        }
        if (OP == MIX_2FMA_1BIT) {
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[k]) : "v"(a), "v"(b));
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[k]) : "v"(y), "v"(z));
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[k]) : "v"(b), "v"(a));
        }
        if (OP == DEP_FMA64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[0]) : "v"(a), "v"(b));
    }
}

template <int OP>
__global__ void k_rate(long long* cyc, double* sink, int iters) {
    double c[8];
    uint32_t x[8];
    uint64_t p[8];
    float f[8];
    for (int k = 0; k < 8; ++k) {
        c[k] = 1.0 + k * 1e-3 + threadIdx.x * 1e-9;
        x[k] = threadIdx.x * 7919u + k;
        p[k] = x[k];
        f[k] = (float)c[k];
    }
    const double a = 0.9999999, b = 1e-9;
    const uint32_t y = threadIdx.x * 2654435761u, z = blockIdx.x + 12345u;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) body<OP>(c, x, p, f, a, b, y, z);
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k] + (double)x[k] + (double)p[k] + f[k];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
    if (s == 12345.678) sink[threadIdx.x] = s;
}

static int instrs_per_iter(int op) {
    if (op == MIX_FMA_BIT || op == MIX_FMA_MAD) return 16;
    if (op == MIX_2FMA_1BIT) return 24;
    return 8;
}

template <int OP>
static void run(const char* name, long long* c, double* d, int cus) {
    const int iters = 2048;
    for (int k = 1; k <= 8; k *= 2) {
        const int threads = k <= 4 ? 256 * k : 1024;              // k = 8: two 1024-thread blocks per CU
        const int blocks = k <= 4 ? cus : 2 * cus;
        k_rate<OP><<<blocks, threads>>>(c, d, 8);
        (void)hipDeviceSynchronize();
        (void)hipMemset(c, 0, (size_t)blocks * 16 * sizeof(long long));
        k_rate<OP><<<blocks, threads>>>(c, d, iters);
        (void)hipDeviceSynchronize();
        static long long h[512 * 16];
        (void)hipMemcpy(h, c, (size_t)blocks * 16 * sizeof(long long), hipMemcpyDeviceToHost);
        long long mx = 0;
        double mean = 0;
        const int wpb = threads / 64;
        for (int b = 0; b < blocks; ++b)
            for (int w = 0; w < wpb; ++w) {
                const long long v = h[b * 16 + w];
                mx = v > mx ? v : mx;
                mean += (double)v;
            }
        mean /= (double)(blocks * wpb);
        const double n = (double)iters * instrs_per_iter(OP);
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr_per_simd\": %.3f, "
               "\"cycles_per_instr_per_wave\": %.3f}\n",
               name, k, mean / (n * k), mean / n);
    }
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    long long* c;
    double* d;
    (void)hipMalloc(&c, (size_t)2 * cus * 16 * sizeof(long long));
    (void)hipMalloc(&d, 1 << 16);
    run<FMA64>("v_fma_f64", c, d, cus);
    run<MUL64>("v_mul_f64", c, d, cus);
    run<ADD64>("v_add_f64", c, d, cus);
    run<BITOP3>("v_bitop3_b32", c, d, cus);
    run<XOR32>("v_xor_b32", c, d, cus);
    run<MAD64>("v_mad_u64_u32", c, d, cus);
    run<CVT64>("v_cvt_f64_u32", c, d, cus);
    run<FMA32>("v_fma_f32", c, d, cus);
    run<MIX_FMA_BIT>("fma_f64 + bitop3", c, d, cus);
    run<MIX_FMA_MAD>("fma_f64 + mad_u64_u32", c, d, cus);
    run<MIX_2FMA_1BIT>("2 fma_f64 + bitop3", c, d, cus);
    run<DEP_FMA64>("v_fma_f64 dependent chain", c, d, cus);
    return 0;
}
