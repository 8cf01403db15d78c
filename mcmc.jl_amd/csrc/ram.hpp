// ram.hpp -- the jump-factor arithmetic of the robust adaptive Metropolis sampler (RAM.jl:55-78),
// shared by the lane-per-chain (samplers.hpp ram_body) and regression (glm.hip glm_ram) kernels.
//
// Storage.  S is the chain's d x d lower-triangular jump factor, kept in HBM as packed rows padded to
// the kernel's compile-time width DF >= d: element (r, c), c <= r < DF, at
// L[(r(r+1)/2 + c) * ram_ld + chain] -- consecutive chains are consecutive doubles, so every access is
// one coalesced 512 B row per wave.  The padding block (rows/columns d..DF-1) holds the identity and
// the padded normals are 0, so the update below maps it to itself exactly (r = 1, c = 1, s = 0) and it
// never feeds a real coordinate: the loops carry no runtime bounds.  The factor is stored twice: a step
// reads one half of the pair and writes the other (ram_half), so no load waits behind a store; each
// half ends with one trash row that absorbs the masked-off stores of the regression kernel.
// ram_ld is a multiple of 256, so lanes past the last chain own padding columns and store freely.
//
// Arithmetic.  The reference forms SS = S (I + a z z'/|z|^2) S' and takes S = chol(SS)'; the kernels
// apply the same product as a rank-1 Cholesky update (a >= 0) or downdate (a < 0) of S with the vector
// sqrt(|a|/|z|^2) S z, which yields the lower factor with positive diagonal of the same SS.  The
// operation order is restated by oracle/oracle.c orc_ram_update.
#pragma once
#include "common.hpp"
#include "detmath.hpp"

namespace mcmc {

// eta * (min(1, exp(ratio)) - rate), eta = min(1, d i^(-2/3))   (RAM.jl:74-76)
__device__ __forceinline__ double ram_alpha(int64_t i, int d, double ratio, double rate) {
    const double eta = __builtin_fmin(1.0, (double)d * det_exp((-2.0 / 3.0) * det_log((double)i)));
    return eta * (__builtin_fmin(1.0, det_exp(ratio)) - rate);
}

__host__ __device__ constexpr int64_t ram_rows(int dpad) { return (int64_t)dpad * (dpad + 1) / 2; }

// Callers pass the chain stride through ram_opaque once per step: the DF(DF+1)/2 products idx * ld are
// then scalar work of the step instead of loop-invariant values hoisted into (and spilled out of) the
// scalar file.
__device__ __forceinline__ uint64_t ram_opaque(uint64_t ld) {
    asm volatile("" : "+s"(ld));
    return ld;
}

// the factor read by step i (1-based) is half (i - 1) & 1 of the pair, the one it writes half i & 1;
// a half is ram_rows(DF) + 1 rows (the last one a trash row for masked-off stores)
template <int DF>
__device__ __forceinline__ double* ram_half(double* L, int64_t i, uint64_t ld) {
    return L + (uint64_t)(i & 1) * (uint64_t)(ram_rows(DF) + 1) * ld;
}

// Addressing: every element of a chain's factor is (wave-uniform row base)[lane], so the loads and
// stores take the scalar-base + 32-bit lane-offset form: no 64-bit VGPR address per access.
// L = the half's uniform base, c = the lane's chain column.

// u[r] = sum_{c <= r} S[r][c] z[c], an fma chain over c = 0..r
template <int DF>
__device__ __forceinline__ void ram_matvec(const double* __restrict__ L, uint32_t c, uint64_t ld,
                                           const double (&z)[DF], double (&u)[DF]) {
#pragma unroll
    for (int r = 0; r < DF; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j <= r; ++j) acc = __builtin_fma((L + (uint64_t)(r * (r + 1) / 2 + j) * ld)[c], z[j], acc);
        u[r] = acc;
        __builtin_amdgcn_sched_barrier(0);     // one row's loads in flight at a time (register pressure)
    }
}

// S <- chol(S S' + beta u u')' with beta = alpha / |z|^2 (nz = |z|^2), read from Ls, written to Ld.
// u is consumed.
template <int DF>
__device__ __forceinline__ void ram_update(const double* __restrict__ Ls, double* __restrict__ Ld, uint32_t c,
                                           uint64_t ld, double alpha, double nz, double (&u)[DF]) {
    const double beta = alpha / nz;
    const bool up = beta >= 0.0;
    const double sb = __builtin_sqrt(__builtin_fabs(beta));
#pragma unroll
    for (int k = 0; k < DF; ++k) u[k] = sb * u[k];
#pragma unroll
    for (int k = 0; k < DF; ++k) {
        const uint64_t okk = (uint64_t)(k * (k + 1) / 2 + k) * ld;
        const double lkk = (Ls + okk)[c];
        const double xk = u[k];
        const double t2 = xk * xk;
        const double l2 = lkk * lkk;
        const double r = __builtin_sqrt(up ? l2 + t2 : l2 - t2);
        const double cc = r / lkk;
        const double sn = xk / lkk;
        const double ic = 1.0 / cc;
        (Ld + okk)[c] = r;
#pragma unroll
        for (int q = k + 1; q < DF; ++q) {
            const uint64_t oq = (uint64_t)(q * (q + 1) / 2 + k) * ld;
            const double l0 = (Ls + oq)[c];
            const double su = sn * u[q];
            const double l = (up ? l0 + su : l0 - su) * ic;
            (Ld + oq)[c] = l;
            u[q] = cc * u[q] - sn * l;
        }
        __builtin_amdgcn_sched_barrier(0);     // one column's loads in flight at a time
    }
}

}  // namespace mcmc
