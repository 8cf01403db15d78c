// ram.hpp -- the jump-factor arithmetic of the robust adaptive Metropolis sampler (RAM.jl:55-78),
// shared by the lane-per-chain (samplers.hpp ram_body) and regression (glm.hip glm_ram) kernels; the wave-per-chain
// layout is ram_wave.hpp.
//
// Storage.  S is the chain's d x d lower-triangular jump factor, kept in HBM as packed rows padded to
// the kernel's compile-time width DF >= d: element (r, c), c <= r < DF, is row idx = r(r+1)/2 + c.  The
// chains are grouped in tiles of 64 (one wave of the lane-per-chain kernel): a half of the factor store is
// [ram_ld / 64 tiles][ram_rows(DF) + 1 rows][64 chains], so chain ch's row idx is at
// ((ch >> 6) (R + 1) + idx) 64 + (ch & 63).  A wave's whole factor is one contiguous block, every row of
// it one 512 B transaction, and the row offsets are compile-time constants (no per-row address arithmetic).
// The padding block (rows/columns d..DF-1) holds the identity and the padded normals are 0, so the update
// below maps it to itself exactly (r = 1, c = 1, s = 0) and it never feeds a real coordinate: the loops
// carry no runtime bounds.  The factor is stored twice: a step reads one half of the pair and writes the
// other (ram_half), so no load waits behind a store; each tile ends with one trash row that absorbs the
// masked-off stores of the regression kernel.  ram_ld is a multiple of 256, so lanes past the last chain
// own padding columns and store freely.
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
// doubles of one 64-chain tile of a half (its rows and the trash row)
__host__ __device__ constexpr int64_t ram_tile_doubles(int dpad) { return (ram_rows(dpad) + 1) * 64; }

// the factor read by step i (1-based) is half (i - 1) & 1 of the pair, the one it writes half i & 1;
// a half is (ram_rows(DF) + 1) ld doubles
template <int DF>
__device__ __forceinline__ double* ram_half(double* L, int64_t i, uint64_t ld) {
    return L + (uint64_t)(i & 1) * (uint64_t)(ram_rows(DF) + 1) * ld;
}

// ------------------------------------------------------------------ lane-per-chain: one tile per wave
// The wave's tile of a half as a buffer resource: row idx at the scalar offset idx * 512 (a constant), the
// lane's chain at the vector offset lane * 8 -- buffer_load/store with no address registers at all, which
// leaves the VGPRs to the column's loads in flight.
using ram_rsrc_t = __amdgpu_buffer_rsrc_t;
typedef unsigned int ram_u32x2 __attribute__((ext_vector_type(2)));

template <int DF>
__device__ __forceinline__ ram_rsrc_t ram_tile_rsrc(const double* tile) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(tile), (short)0, (int)(ram_tile_doubles(DF) * 8),
                                             0x00020000);
}
__device__ __forceinline__ double ram_tload(ram_rsrc_t r, uint32_t vo, int idx) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, idx * 512, 0));
}
__device__ __forceinline__ void ram_tstore(ram_rsrc_t r, uint32_t vo, int idx, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ram_u32x2, v), r, vo, idx * 512, 0);
}

// u[r] = sum_{c <= r} S[r][c] z[c], an fma chain over c = 0..r
template <int DF>
__device__ __forceinline__ void ram_matvec(ram_rsrc_t S, uint32_t vo, const double (&z)[DF], double (&u)[DF]) {
#pragma unroll
    for (int r = 0; r < DF; ++r) {
        double v[DF];
#pragma unroll
        for (int j = 0; j <= r; ++j) v[j] = ram_tload(S, vo, r * (r + 1) / 2 + j);
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j <= r; ++j) acc = __builtin_fma(v[j], z[j], acc);
        u[r] = acc;
        __builtin_amdgcn_sched_barrier(0);     // a row's loads issued together, one row at a time
    }
}

// S <- chol(S S' + beta u u')' with beta = alpha / |z|^2 (nz = |z|^2), read from Ss, written to Sd; u is
// consumed.  NEXT: the next step's S z is folded in -- as column k of the new factor is formed, its entries
// feed un[q] = fma(S'[q][k], z'[k], un[q]), q >= k: per row the fma chain over c = 0..q of ram_matvec, taken
// one column at a time, so a step reads its factor once.  zblock(b, z4) draws the next step's normals
// 4b..4b+3 when the columns reach them.
template <int DF, bool NEXT, class ZB>
__device__ __forceinline__ void ram_update(ram_rsrc_t Ss, ram_rsrc_t Sd, uint32_t vo, double alpha, double nz,
                                           double (&u)[DF], ZB&& zblock, double (&un)[DF]) {
    const double beta = alpha / nz;
    const bool up = beta >= 0.0;
    const double sb = __builtin_sqrt(__builtin_fabs(beta));
#pragma unroll
    for (int k = 0; k < DF; ++k) u[k] = sb * u[k];
    if (NEXT) {
#pragma unroll
        for (int k = 0; k < DF; ++k) un[k] = 0.0;
    }
    double z4[4] = {0.0, 0.0, 0.0, 0.0};
    double l0[DF];                             // column k, rows q >= k: issued together, one column ahead
#pragma unroll
    for (int q = 0; q < DF; ++q) l0[q] = ram_tload(Ss, vo, q * (q + 1) / 2);
#pragma unroll
    for (int k = 0; k < DF; ++k) {
        double l1[DF];
#pragma unroll
        for (int q = k + 1; q < DF; ++q) l1[q] = ram_tload(Ss, vo, q * (q + 1) / 2 + k + 1);
        if (NEXT && (k & 3) == 0) zblock(k >> 2, z4);
        const double zk = z4[k & 3];
        const double lkk = l0[k];
        const double xk = u[k];
        const double t2 = xk * xk;
        const double l2 = lkk * lkk;
        const double r = __builtin_sqrt(up ? l2 + t2 : l2 - t2);
        const double cc = r / lkk;
        const double sn = xk / lkk;
        const double sns = up ? sn : -sn;      // l0 - sn u == l0 + (-sn) u exactly: one add, no select per entry
        const double ic = 1.0 / cc;
        ram_tstore(Sd, vo, k * (k + 1) / 2 + k, r);
        if (NEXT) un[k] = __builtin_fma(r, zk, un[k]);
#pragma unroll
        for (int q = k + 1; q < DF; ++q) {
            const double l = (l0[q] + sns * u[q]) * ic;
            ram_tstore(Sd, vo, q * (q + 1) / 2 + k, l);
            u[q] = cc * u[q] - sn * l;
            if (NEXT) un[q] = __builtin_fma(l, zk, un[q]);
        }
#pragma unroll
        for (int q = k + 1; q < DF; ++q) l0[q] = l1[q];
        __builtin_amdgcn_sched_barrier(0);     // one column at a time
    }
}

}  // namespace mcmc
