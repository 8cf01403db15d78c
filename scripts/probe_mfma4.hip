// Dev probe: v_mfma_f64_4x4x4_4b_f64 (four independent 4x4x4 blocks a wave, 512 flop) against
// v_mfma_f64_16x16x4_f64 (2 048 flop) on gfx950.
//   layout:  raw per-lane A, B, C -> D of one 4x4x4_4b on random wide-exponent operands, written to a file for
//            scripts/probe_mfma4.py (operand layout and the accumulation order of each output);
//   rate:    back-to-back issue, NCH accumulators a wave, 1 / 2 waves per SIMD, with and without one ds_read_b64
//            (the A operand from LDS, read LA MFMAs ahead) per MFMA; the 16x16x4 form alike for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_mfma4.hip -o scripts/_build/probe_mfma4
// Run:   scripts/_build/probe_mfma4 <layout.bin>   (PROBE_PAT=1: the kernels' operand-read patterns only)
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


// the regression kernels' pattern: 64 MFMAs an iteration over NCH rotating accumulators, each A operand read from
// LDS LA MFMAs ahead at an immediate offset (volatile: no ds_read2 pairing); MODE 0: 4x4x4_4b + ds_read_b64 per MFMA,
// 1: 4x4x4_4b + ds_read_b128 per two MFMAs, 2: 16x16x4 + ds_read_b64 per MFMA
typedef const volatile __attribute__((address_space(3))) double lds_d;
typedef double f64x2v __attribute__((ext_vector_type(2)));
typedef const volatile __attribute__((address_space(3))) f64x2v lds_d2;
constexpr int kPatW = 2 * 64 * 16 + 64;                 // doubles of LDS a wave
template <int MODE, int NCH, int LA>
__global__ __launch_bounds__(1024) void k_pat(double* out, long long* clk, int iters) {
    extern __shared__ double xsd[];                     // one workgroup a CU (>= 96 KB), 256 wps threads
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    double* const xw = xsd + w * kPatW;
    for (int i = l; i < kPatW; i += 64) xw[i] = 1.0 + 1e-9 * i;
    __syncthreads();
    double c4[NCH];
    f64x4 c16[NCH];
    for (int k = 0; k < NCH; ++k) { c4[k] = 0.0; c16[k] = f64x4{0, 0, 0, 0}; }
    const double b = 1.0 - threadIdx.x * 1e-9;
    const double* base = xw + 2 * ((l & 3) * 33 + 4 * ((l >> 2) & 3));
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        double av[64];
        auto rd = [&](int j) {
            if (MODE == 1) {
                if ((j & 1) == 0) {
                    const f64x2v v = *(lds_d2*)(base + 2 * (j >> 1) * 8);
                    av[j] = v[0];
                    av[j + 1] = v[1];
                }
            } else {
                av[j] = *(lds_d*)(base + j * 8);
            }
        };
#pragma unroll
        for (int j = 0; j < LA; ++j) rd(j);
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            if (j + LA < 64) rd(j + LA);
            if (MODE == 2) c16[j % NCH] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j], b, c16[j % NCH], 0, 0, 0);
            else c4[j % NCH] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[j], b, c4[j % NCH], 0, 0, 0);
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

template <int MODE, int NCH, int LA>
static void pat(int waves_per_simd, int cus, double* d, long long* c) {
    const int blocks = cus;
    const int iters = MODE == 2 ? 400 : 1600;
    size_t lds = (size_t)4 * waves_per_simd * kPatW * 8;
    if (lds < 96 * 1024) lds = 96 * 1024;
    (void)hipFuncSetAttribute((const void*)k_pat<MODE, NCH, LA>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    k_pat<MODE, NCH, LA><<<blocks, 256 * waves_per_simd, lds>>>(d, c, 5);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_pat<MODE, NCH, LA><<<blocks, 256 * waves_per_simd, lds>>>(d, c, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)blocks * 4 * waves_per_simd * iters * 64 * (MODE == 2 ? 2048.0 : 512.0);
    const double tf = flop / (ms * 1e-3) / 1e12;
    printf("{\"pattern\": \"%s\", \"nch\": %d, \"la\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f, "
           "\"frac_of_78.6\": %.3f}\n",
           MODE == 0 ? "4x4x4_4b + ds_read_b64 each" : MODE == 1 ? "4x4x4_4b + ds_read_b128 per two" : "16x16x4 + ds_read_b64 each",
           NCH, LA, waves_per_simd, ms, tf, tf / 78.6);
    fflush(stdout);
}

// co-residence made certain: ONE workgroup per CU (96 KB of dynamic LDS each), 256 WPS threads, so WPS waves on every
// SIMD; NCH rotating accumulators, no memory operands; the number that matters is the time of the whole grid
template <bool BIG, int NCH>
__global__ __launch_bounds__(1024) void k_res(double* out, int iters) {
    extern __shared__ double pad[];
    double c4[NCH];
    f64x4 c16[NCH];
    for (int k = 0; k < NCH; ++k) { c4[k] = 0.0; c16[k] = f64x4{0, 0, 0, 0}; }
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            if (BIG) c16[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c16[k], 0, 0, 0);
            else c4[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c4[k], 0, 0, 0);
        }
    }
    double s = 0;
    for (int k = 0; k < NCH; ++k) s += c4[k] + c16[k][0] + c16[k][3];
    if (s == 12345.678) out[threadIdx.x] = s + pad[0];
}
template <bool BIG, int NCH>
static void res(int wps, int cus, double* d) {
    const int iters = (BIG ? 8000 : 32000) / NCH;
    const size_t lds = 96 * 1024;
    (void)hipFuncSetAttribute((const void*)k_res<BIG, NCH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    k_res<BIG, NCH><<<cus, 256 * wps, lds>>>(d, 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_res<BIG, NCH><<<cus, 256 * wps, lds>>>(d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double mfma_per_simd = (double)wps * iters * NCH;
    const double flop = (double)cus * 4 * mfma_per_simd * (BIG ? 2048.0 : 512.0);
    const double tf = flop / (ms * 1e-3) / 1e12;
    printf("{\"resident\": \"%s\", \"nch\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.2f, "
           "\"frac_of_78.6\": %.3f, \"ns_per_mfma_per_simd\": %.3f}\n",
           BIG ? "16x16x4f64" : "4x4x4_4b_f64", NCH, wps, ms, tf, tf / 78.6, ms * 1e6 / mfma_per_simd);
    fflush(stdout);
}

// co-issue with co-residence certain (one 512-thread workgroup a CU, 96 KB LDS): waves 0-3 (one a SIMD) run NCH = 8
// independent 16x16x4 accumulators, waves 4-7 (the same SIMDs) KIND 0: f64 FMAs, 1: int32 xor/shift/add, NV
// instructions per partner MFMA; mode 0 both, 1 MFMA waves only, 2 VALU waves only
template <int KIND, int NV>
__global__ __launch_bounds__(512) void k_cor(double* out, int iters, int mode) {
    extern __shared__ double pad[];
    const int w = threadIdx.x >> 6;
    if (w < 4) {
        if (mode == 2) return;
        f64x4 c[8];
        for (int k = 0; k < 8; ++k) c[k] = f64x4{0, 0, 0, 0};
        const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
        }
        f64x4 s = c[0];
        for (int k = 1; k < 8; ++k) s += c[k];
        if (s[0] == 12345.678) out[threadIdx.x] = s[1] + pad[0];
    } else {
        if (mode == 1) return;
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
    }
}
template <int KIND, int NV>
static void cor(int cus, double* d) {
    const int iters = 2000;
    const size_t lds = 96 * 1024;
    (void)hipFuncSetAttribute((const void*)k_cor<KIND, NV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    float ms[3];
    for (int mode = 0; mode < 3; ++mode) {
        k_cor<KIND, NV><<<cus, 512, lds>>>(d, 20, mode);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        k_cor<KIND, NV><<<cus, 512, lds>>>(d, iters, mode);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[mode], e0, e1);
    }
    printf("{\"coexec_resident\": \"%s\", \"partner_valu_per_mfma\": %d, \"both_ms\": %.3f, \"mfma_only_ms\": %.3f, "
           "\"valu_only_ms\": %.3f, \"both_over_max\": %.3f, \"both_over_sum\": %.3f}\n",
           KIND == 0 ? "f64 fma" : "int32", NV, ms[0], ms[1], ms[2], ms[0] / (ms[1] > ms[2] ? ms[1] : ms[2]),
           ms[0] / (ms[1] + ms[2]));
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
    if (getenv("PROBE_CO")) {
        cor<0, 1>(cus, d);
        cor<0, 4>(cus, d);
        cor<1, 1>(cus, d);
        cor<1, 4>(cus, d);
        return 0;
    }
    if (getenv("PROBE_RES")) {
        res<true, 8>(1, cus, d);
        res<true, 8>(2, cus, d);
        res<true, 8>(4, cus, d);
        res<true, 1>(1, cus, d);
        res<true, 1>(2, cus, d);
        res<false, 8>(1, cus, d);
        res<false, 8>(2, cus, d);
        res<false, 4>(1, cus, d);
        res<false, 4>(2, cus, d);
        res<false, 1>(1, cus, d);
        return 0;
    }
    if (getenv("PROBE_PAT")) {
        pat<0, 4, 8>(1, cus, d, c);
        pat<0, 4, 8>(2, cus, d, c);
        pat<0, 8, 8>(2, cus, d, c);
        pat<0, 8, 12>(2, cus, d, c);
        pat<1, 4, 8>(1, cus, d, c);
        pat<1, 4, 8>(2, cus, d, c);
        pat<1, 8, 8>(2, cus, d, c);
        pat<1, 8, 12>(2, cus, d, c);
        pat<2, 1, 4>(1, cus, d, c);
        pat<2, 1, 4>(2, cus, d, c);
        pat<2, 8, 4>(2, cus, d, c);
        return 0;
    }
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
