// glm_layout.hpp -- the covariate image the regression kernels stage into LDS (host packing and device addressing).
//
// X is uploaded once, at model creation, as a sequence of 16-observation tiles.  Tile t is TS doubles: 16 rows of S
// doubles (row r = observation 16t + r, coordinate k at position k) followed by the tile's 16 responses Y (the logistic
// model: w = s (2y - 1), det_logi) and 16 per-observation bounds B (the logistic model: -T(y), detmath.hpp
// logi_bound; -inf on padded rows; 0 otherwise), zero-padded to a multiple of 128 doubles (1 KiB).  A tile therefore
// moves global -> LDS as whole 1-KiB wave-instructions
// (`global_load_lds_dwordx4`, or plain 16-byte loads) with no per-lane address arithmetic: the LDS image is the HBM
// image byte for byte.
//
// The row stride S = d_pad + 1 is odd.  hipcc merges each lane's MFMA operand reads pairwise into ds_read2_b64, which
// the LDS serves as lane groups of 16 consecutive lanes over 32 four-byte banks (MI355X_MICROARCH.md §LDS): a group is
// conflict-free when its 16 doubles sit at distinct indices mod 16.  Lanes 16q .. 16q+15 of a wave are (q, cl = 0..15):
//   eta = X beta, A operand: lane (q, cl) reads row cl, coordinate 16 m + 4 q + e  ->  D = cl S + const: S odd makes
//        cl S mod 16 a permutation of 0..15;
//   G = X^T r, A operand: lane (q, cl) reads row 4 kk + q, coordinate 16 T + 4 (cl & 3) + (cl >> 2)
//        ->  D = 4 (cl & 3) + (cl >> 2) + const: 0..15.
// (Rounds 1-3 used S = d_pad + 2, which puts two lanes of a group on one bank pair in the eta read: 0.39-0.41 of the
// LDS-active cycles were conflicts, profiles/r03s2_fp64_config{3,5}.md.)  tests/test_api_cpu.py checks both
// reads for every geometry.
#pragma once
#include <stdint.h>

namespace mcmc {

__host__ __device__ constexpr int glm_row_stride(int d_pad) { return d_pad + 1; }
// doubles per staged tile: 16 rows, then Y[16] and B[16], rounded up to 1 KiB
__host__ __device__ constexpr int glm_tile_doubles(int d_pad) { return (16 * glm_row_stride(d_pad) + 32 + 127) / 128 * 128; }
__host__ __device__ constexpr int glm_y_offset(int d_pad) { return 16 * glm_row_stride(d_pad); }
__host__ __device__ constexpr int glm_b_offset(int d_pad) { return 16 * glm_row_stride(d_pad) + 16; }
// eta A operand: slot (m, e) of a lane, relative to the lane base cl S + 4 q + (slice base coordinate)
__host__ __device__ constexpr int glm_eta_off(int slot) { return 16 * (slot >> 2) + (slot & 3); }
// G A operand: coordinate tile T of a slice, relative to the lane base q S + 4 (cl & 3) + (cl >> 2) + (slice base)
__host__ __device__ constexpr int glm_g_off(int T) { return 16 * T; }

// The logistic model's bound column: b = -T(y).  The reference's p = 1/(1+exp(-s eta)) makes log(1 - p) (y = 0) or
// log(p) (y = 1) -Inf where p rounds to 1 or 0; with u = -w eta (detmath.hpp det_logi) that is u >= T(y).  y = 0:
// 1 + exp(-u) rounds to 1 iff exp(-u) <= 2^-53 (ties to even), u >= RU(53 ln 2); y = 1: p = 1/(1+exp(u)) is 0 iff
// exp(u) overflows, u > fdlibm's o_threshold 0x1.62e42fefa39efp+9.  The oracle restates both (orc_glm_eval).
constexpr double kLogiT0 = 0x1.25e4f7b2737fbp+5;
constexpr double kLogiT1 = 0x1.62e42fefa39f0p+9;
__host__ __device__ constexpr double logi_bound(double y) { return y == 1.0 ? -kLogiT1 : -kLogiT0; }

}  // namespace mcmc
