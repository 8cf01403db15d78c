// util.hip -- small device helpers: fills, layout transposes and the
// deterministic-math probes used by the parity tests (tests/test_gpu_detmath.py).
#include "../common.hpp"
#include "../detmath.hpp"

namespace mcmc {

__global__ void k_fill_f64(double* p, int64_t n, double v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
// p[b * stride + e] = v, e < w, b < nb
__global__ void k_fill_f64_strided(double* p, int64_t nb, int64_t w, int64_t stride, double v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb * w) p[(i / w) * stride + i % w] = v;
}
__global__ void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
// dst[j][c] (stride ldd) <- v[j] for c < C  (every chain starts at model.init, RWM.jl:53)
__global__ void k_broadcast_cols(double* dst, int64_t ldd, const double* v, int d, int64_t C) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    for (int j = 0; j < d; ++j) dst[(size_t)j * ldd + c] = v[j];
}
// dst[c][j] (row stride ldr) <- v[j]  (chain-major layout of the wave-per-chain kernels)
__global__ void k_broadcast_rows(double* dst, int64_t ldr, const double* v, int d, int64_t C) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C * (int64_t)ldr) return;
    const int64_t j = i % ldr;
    dst[i] = j < d ? v[j] : 0.0;
}
// dst[j][c] (stride ldd) <- src[j][c] (stride lds)
__global__ void k_copy_cols(double* dst, int64_t ldd, const double* src, int64_t lds, int d, int64_t C) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    for (int j = 0; j < d; ++j) dst[(size_t)j * ldd + c] = src[(size_t)j * lds + c];
}
// Tiled transpose, batched: dst[b][s][r] (row stride ldd) <- src[b][r][s] (row stride lds).
__global__ void k_transpose(double* dst, int64_t ldd, const double* src, int64_t lds, int64_t R, int64_t S) {
    __shared__ double tile[32][33];
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * 32, s0 = (int64_t)blockIdx.y * 32;
    const double* sb = src + (size_t)b * (size_t)R * (size_t)lds;
    double* db = dst + (size_t)b * (size_t)S * (size_t)ldd;
    for (int k = threadIdx.y; k < 32; k += blockDim.y) {
        const int64_t r = r0 + k, s = s0 + threadIdx.x;
        if (r < R && s < S) tile[k][threadIdx.x] = sb[(size_t)r * lds + s];
    }
    __syncthreads();
    for (int k = threadIdx.y; k < 32; k += blockDim.y) {
        const int64_t s = s0 + k, r = r0 + threadIdx.x;
        if (r < R && s < S) db[(size_t)s * ldd + r] = tile[threadIdx.x][k];
    }
}

__global__ void k_detmath(int op, int64_t n, const double* x, const double* y, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double a = x[i];
    double r = 0.0;
    switch (op) {
        case 0: r = det_log(a); break;
        case 1: r = det_exp(a); break;
        case 2: { double s, c; det_sincos2pi(a, s, c); r = s; } break;
        case 3: { double s, c; det_sincos2pi(a, s, c); r = c; } break;
        case 4: r = __builtin_sqrt(a); break;
        case 5: r = a / y[i]; break;
        case 6: {
            // x[i] holds (chain, step, block) packed: chain = bits 0-31 of the integer value, step = y[i]
            const uint64_t packed = (uint64_t)a;
            const u32x4 w = philox4x32_10((uint32_t)packed, (uint32_t)y[i], (uint32_t)(packed >> 32), TAG_NORMAL,
                                          0u, 0u);
            double z0, z1, z2, z3;
            normals4(w, z0, z1, z2, z3);
            out[4 * i] = z0; out[4 * i + 1] = z1; out[4 * i + 2] = z2; out[4 * i + 3] = z3;
            return;
        }
        case 7: r = round_away(a); break;
        case 8: { const u32x4 w = philox4x32_10((uint32_t)(uint64_t)a, 0u, 0u, TAG_ACCEPT, 0u, 0u);
                  r = uniform52(w.x, w.y); } break;
        case 9: r = bm_log_u32((uint32_t)(uint64_t)a); break;
        case 10: { double s, c; det_sincos2pi_u32((uint32_t)(uint64_t)a, s, c); r = s; } break;
        case 11: { double s, c; det_sincos2pi_u32((uint32_t)(uint64_t)a, s, c); r = c; } break;
        case 12: r = sqrt_pos_normal(a); break;
        case 13: r = det_exp_tab(a); break;
        case 14: r = det_log_tab(a); break;
        case 15: r = gt_det_log(a, y[i]) ? 1.0 : 0.0; break;      // the screened accept test: a > det_log(y)
        case 16: r = bm_rad2_u32((uint32_t)(uint64_t)a); break;    // the Box-Muller radius^2, -2 log u
        case 17: r = bm_radius_u32((uint32_t)(uint64_t)a, rad_tab_global()); break;   // the radius polynomial
        case 18: r = det_erfc(a); break;                           // probit model: erfc, log1p, normal log-cdf
        case 19: r = det_log1p(a); break;
        case 20: r = det_normlogcdf(a); break;
        case 22: { double tm, rv; det_logi(a, y[i], tm, rv); r = tm; } break;   // logistic term of (eta, w)
        case 23: { double tm, rv; det_logi(a, y[i], tm, rv); r = rv; } break;   // ... and its weight
        default: r = 0.0;
    }
    out[i] = r;
}

// op 21: bm_radius_u32 reading its coefficients from an LDS copy of the table, as the hot kernels do (samplers.hpp
// kTabLds).  Tail lanes (v < 2^21, including v = 0) form an out-of-range LDS row address there and discard what it
// reads (detmath.hpp bm_radius_u32, RadTab.lds): this kernel drives those inputs so the tests see the LDS path give
// the global path's values (the hardware returns 0 for an LDS read outside the allocation, MI355X ISA).
__global__ void k_radius_lds(int64_t n, const double* x, double* out) {
    extern __shared__ __attribute__((aligned(16))) double tab[];
    for (int j = threadIdx.x; j < 4 * BM_RADP_NROWS * 2; j += blockDim.x) tab[j] = (&kBmRadPTab[0][0])[j];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = bm_radius_u32((uint32_t)(uint64_t)x[i], RadTab{reinterpret_cast<const double (*)[2]>(tab), true});
}

__global__ void k_philox(int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32x4 w = philox4x32_10(ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3], key[2 * i], key[2 * i + 1]);
    out[4 * i] = w.x; out[4 * i + 1] = w.y; out[4 * i + 2] = w.z; out[4 * i + 3] = w.w;
}

// v_mfma_f64_16x16x4_f64 probe: D = A[16x4] * B[4x16] + C, with the lane maps of
// cdna_hip_programming.md §3 (A/B as the f32 16x16x4 form; C/D col = l&15, row = (l>>4) + 4*reg).
// nk MFMAs chained over K = 4*nk: A [16][4nk], B [4nk][16], C/D [16][16] row-major.
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void k_mfma_probe(const double* A, const double* B, const double* C, double* D, int nk) {
    const int l = threadIdx.x;
    f64x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = C[((l >> 4) + 4 * r) * 16 + (l & 15)];
    for (int kk = 0; kk < nk; ++kk) {
        const double a = A[(l & 15) * (4 * nk) + 4 * kk + (l >> 4)];
        const double b = B[(4 * kk + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

}  // namespace mcmc

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

hipError_t mcmc_fill_f64(double* p, int64_t n, double v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    mcmc::k_fill_f64<<<nblk(n, 256), 256, 0, st>>>(p, n, v);
    return hipGetLastError();
}
hipError_t mcmc_fill_f64_strided(double* p, int64_t nb, int64_t w, int64_t stride, double v, hipStream_t st) {
    if (nb <= 0 || w <= 0) return hipSuccess;
    mcmc::k_fill_f64_strided<<<nblk(nb * w, 256), 256, 0, st>>>(p, nb, w, stride, v);
    return hipGetLastError();
}
hipError_t mcmc_fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    mcmc::k_fill_i32<<<nblk(n, 256), 256, 0, st>>>(p, n, v);
    return hipGetLastError();
}
hipError_t mcmc_broadcast_cols(double* dst, int64_t ldd, const double* v, int d, int64_t C, hipStream_t st) {
    mcmc::k_broadcast_cols<<<nblk(C, 256), 256, 0, st>>>(dst, ldd, v, d, C);
    return hipGetLastError();
}
hipError_t mcmc_broadcast_rows(double* dst, int64_t ldr, const double* v, int d, int64_t C, hipStream_t st) {
    mcmc::k_broadcast_rows<<<nblk(C * ldr, 256), 256, 0, st>>>(dst, ldr, v, d, C);
    return hipGetLastError();
}
hipError_t mcmc_copy_cols(double* dst, int64_t ldd, const double* src, int64_t lds, int d, int64_t C, hipStream_t st) {
    mcmc::k_copy_cols<<<nblk(C, 256), 256, 0, st>>>(dst, ldd, src, lds, d, C);
    return hipGetLastError();
}
hipError_t mcmc_transpose(double* dst, int64_t ldd, const double* src, int64_t lds, int64_t batch, int64_t R,
                          int64_t S, hipStream_t st) {
    if (batch <= 0 || R <= 0 || S <= 0) return hipSuccess;
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        const dim3 grid(nblk(R, 32), nblk(S, 32), (unsigned)nb);
        mcmc::k_transpose<<<grid, dim3(32, 8), 0, st>>>(dst + (size_t)b0 * S * ldd, ldd,
                                                        src + (size_t)b0 * R * lds, lds, R, S);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t mcmc_detmath(int op, int64_t n, const double* x, const double* y, double* out, hipStream_t st) {
    if (op == 21)
        mcmc::k_radius_lds<<<nblk(n, 256), 256, 4 * BM_RADP_NROWS * 2 * sizeof(double), st>>>(n, x, out);
    else
        mcmc::k_detmath<<<nblk(n, 256), 256, 0, st>>>(op, n, x, y, out);
    return hipGetLastError();
}
hipError_t mcmc_philox(int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out, hipStream_t st) {
    mcmc::k_philox<<<nblk(n, 256), 256, 0, st>>>(n, ctr, key, out);
    return hipGetLastError();
}
hipError_t mcmc_mfma_probe(const double* A, const double* B, const double* C, double* D, int nk, hipStream_t st) {
    mcmc::k_mfma_probe<<<1, 64, 0, st>>>(A, B, C, D, nk);
    return hipGetLastError();
}
