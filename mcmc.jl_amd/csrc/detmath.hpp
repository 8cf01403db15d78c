// detmath.hpp -- device-side random stream and deterministic fp64 math for gfx950.
//
// Specification: DESIGN.md §3.  Every function here has a CPU twin in
// oracle/detmath.h that performs the same IEEE operations in the same order,
// so kernel and oracle agree bit for bit.  Rules that make that hold:
//   * the whole library is compiled with -ffp-contract=off; each fused
//     multiply-add is an explicit __builtin_fma;
//   * '/' and sqrt are the IEEE correctly-rounded operations (hipcc's default
//     f64 lowering; checked on the device by tests/test_gpu_detmath.py);
//   * no OCML transcendentals (their last-ulp behaviour differs from glibc).
//
// The reference draws with Julia's global dSFMT + ziggurat (src/samplers/RWM.jl:59,
// src/samplers/HMC.jl:136); the build replaces that with a counter-based
// Philox4x32-10 stream keyed by the run seed, counter = (global chain, step,
// block, tag), so every (chain, step) draw is addressable without state and the
// result does not depend on how chains are sharded over GPUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bm_log_table.inc"
#include "erfc_table.inc"
#include "softplus_table.inc"

namespace mcmc {

enum : uint32_t { TAG_NORMAL = 0u, TAG_ACCEPT = 1u, TAG_DATA = 7u };

struct u32x4 { uint32_t x, y, z, w; };

// U: c1 and c3 are wave-uniform (a step index and a tag): round 0's c1 ^ k0 and c3 ^ k1 are then scalar xors and
// its two three-input xors single v_xor_b32 (v_bitop3_b32 reads at most one scalar operand, so with two it needs
// a v_mov first)
template <bool U = false>
__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        uint32_t n0, n2;
        if (U && r == 0) {
            n0 = (uint32_t)(p1 >> 32) ^ (c1 ^ k0);
            n2 = (uint32_t)(p0 >> 32) ^ (c3 ^ k1);
        } else {
            // three-input xor in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler's own
            // combine leaves most of these as two v_xor_b32
            n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
            n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        }
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    return {c0, c1, c2, c3};
}

struct Stream {
    uint32_t k0, k1;
    __device__ __forceinline__ u32x4 block(uint32_t chain, uint32_t step, uint32_t blk, uint32_t tag) const {
        return philox4x32_10(chain, step, blk, tag, k0, k1);
    }
    // step wave-uniform
    __device__ __forceinline__ u32x4 block_us(uint32_t chain, uint32_t step, uint32_t blk, uint32_t tag) const {
        return philox4x32_10<true>(chain, step, blk, tag, k0, k1);
    }
};

__device__ __forceinline__ double bits2d(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t d2bits(double d) { return (uint64_t)__double_as_longlong(d); }

// 52-bit uniform on [0, 1) (Julia rand() semantics: 0 possible, 1 not): a:b's top 52 bits as the mantissa of a
// double in [1, 2) -- two v_alignbit_b32 -- less 1 (round 3; was (a>>5 : b>>6) 2^-53, nine instructions)
__device__ __forceinline__ double uniform52(uint32_t a, uint32_t b) {
    const uint32_t hi = __builtin_amdgcn_alignbit(0x3ffu, a, 12);     // 0x3ff00000 | a >> 12
    const uint32_t lo = __builtin_amdgcn_alignbit(a, b, 12);          // a << 20 | b >> 12
    return bits2d(((uint64_t)hi << 32) | lo) - 1.0;
}
__device__ __forceinline__ double uniform32_open(uint32_t a) { return ((double)a + 0.5) * 0x1p-32; }
__device__ __forceinline__ double uniform32(uint32_t a) { return (double)a * 0x1p-32; }
__device__ __forceinline__ double pow2i(int k) { return bits2d((uint64_t)(k + 1023) << 52); }

// fdlibm e_log.c general path.  Special cases resolved by selects so the
// common path stays branch-free across the wave.  Written as stages (det_log = s1, s2, s3, fin) so that a
// caller can interleave independent work between them (glm.hip); the operations are the same either way.
struct LogState {
    double x, m, f, s, dk, z, w, R;
    uint64_t bx;
    int k;
};
__device__ __forceinline__ void det_log_s1(double x, LogState& L) {   // reduction to m in [sqrt(2)/2, sqrt(2))
    uint64_t bx = d2bits(x);
    const bool sub = bx < 0x0010000000000000ull;            // zero or subnormal (or negative: handled below)
    const bool scl = sub && x > 0.0;                         // subnormal: scale by 2^54 (selects, no branch)
    x = scl ? x * 0x1p54 : x;
    int k = scl ? -54 : 0;
    bx = d2bits(x);
    uint32_t hx = (uint32_t)(bx >> 32);
    k += (int)((hx >> 20) & 0x7ff) - 1023;
    hx &= 0x000fffffu;
    const uint32_t i = (hx + 0x95f64u) & 0x100000u;
    const uint64_t nb = ((uint64_t)(hx | (i ^ 0x3ff00000u)) << 32) | (bx & 0xffffffffull);
    L.m = bits2d(nb);
    L.k = k + (int)(i >> 20);
    L.x = x;
    L.bx = bx;
}
__device__ __forceinline__ void det_log_s2(LogState& L) {             // s = f / (2 + f)
    L.f = L.m - 1.0;
    L.s = L.f / (2.0 + L.f);
    L.dk = (double)L.k;
}
__device__ __forceinline__ void det_log_s3(LogState& L) {             // R(z), z = s^2
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2,
                 Lg3 = 0x1.2492494229359p-2, Lg4 = 0x1.c71c51d8e78afp-3,
                 Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    L.z = L.s * L.s;
    L.w = L.z * L.z;
    const double t1 = L.w * __builtin_fma(L.w, __builtin_fma(L.w, Lg6, Lg4), Lg2);
    const double t2 = L.z * __builtin_fma(L.w, __builtin_fma(L.w, __builtin_fma(L.w, Lg7, Lg5), Lg3), Lg1);
    L.R = t2 + t1;
}
__device__ __forceinline__ double det_log_fin(const LogState& L) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double x = L.x;
    const double hfsq = 0.5 * L.f * L.f;
    double res = L.dk * ln2_hi - ((hfsq - (L.s * (hfsq + L.R) + L.dk * ln2_lo)) - L.f);
    // special values, in the oracle's order: NaN, negative, zero, +inf
    if (x == 0.0) res = -__builtin_inf();
    if (L.bx >= 0x7ff0000000000000ull && x > 0.0) res = x;     // +inf
    if (x < 0.0) res = bits2d(0x7ff8000000000000ull);
    if (x != x) res = x;
    return res;
}
__device__ __forceinline__ double det_log(double x) {
    LogState L;
    det_log_s1(x, L);
    det_log_s2(L);
    det_log_s3(L);
    return det_log_fin(L);
}

// Cody-Waite reduction + degree-13 Taylor polynomial; stages as det_log.
struct ExpState {
    double x, xc, r, p;
    int k;
};
__device__ __forceinline__ void det_exp_s1(double x, ExpState& E) {   // k = round(x / ln2), r = x - k ln2
    const double inv_ln2 = 0x1.71547652b82fep+0;
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double shifter = 0x1.8p52;
    const double xc = __builtin_fmin(__builtin_fmax(x, -746.0), 710.0);  // keep k in range for NaN-free math
    const double t = __builtin_fma(xc, inv_ln2, shifter);
    const double kd = t - shifter;
    E.k = (int)kd;
    double r = __builtin_fma(-kd, ln2_hi, xc);
    E.r = __builtin_fma(-kd, ln2_lo, r);
    E.x = x;
    E.p = 0x1.6124613a86d09p-33;
}
__device__ __forceinline__ void det_exp_s2(ExpState& E) {             // Horner, first half
    double p = E.p;
    const double r = E.r;
    p = __builtin_fma(p, r, 0x1.1eed8eff8d898p-29);
    p = __builtin_fma(p, r, 0x1.ae64567f544e4p-26);
    p = __builtin_fma(p, r, 0x1.27e4fb7789f5cp-22);
    p = __builtin_fma(p, r, 0x1.71de3a556c734p-19);
    p = __builtin_fma(p, r, 0x1.a01a01a01a01ap-16);
    p = __builtin_fma(p, r, 0x1.a01a01a01a01ap-13);
    p = __builtin_fma(p, r, 0x1.6c16c16c16c17p-10);
    E.p = p;
}
__device__ __forceinline__ void det_exp_s3(ExpState& E) {             // Horner, second half
    double p = E.p;
    const double r = E.r;
    p = __builtin_fma(p, r, 0x1.1111111111111p-7);
    p = __builtin_fma(p, r, 0x1.5555555555555p-5);
    p = __builtin_fma(p, r, 0x1.5555555555555p-3);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    E.p = p;
}
__device__ __forceinline__ double det_exp_fin(const ExpState& E) {
    const int k1 = E.k / 2, k2 = E.k - k1;
    double res = (E.p * pow2i(k1)) * pow2i(k2);
    const double x = E.x;
    if (x > 709.782712893384) res = __builtin_inf();
    if (x < -745.1332191019412) res = 0.0;
    if (x != x) res = x;
    return res;
}
__device__ __forceinline__ double det_exp(double x) {
    ExpState E;
    det_exp_s1(x, E);
    det_exp_s2(E);
    det_exp_s3(E);
    return det_exp_fin(E);
}

__device__ __forceinline__ void det_sincos2pi(double u, double& s_out, double& c_out) {
    const double q = __builtin_floor(__builtin_fma(u, 4.0, 0.5));
    const double r = __builtin_fma(q, -0.25, u);
    const double r2 = r * r;
    double S = -0x1.6fadb9f155744p-1;
    S = __builtin_fma(S, r2, 0x1.e8f434d018d63p+1);
    S = __builtin_fma(S, r2, -0x1.e3074fde8871fp+3);
    S = __builtin_fma(S, r2, 0x1.50783487ee782p+5);
    S = __builtin_fma(S, r2, -0x1.32d2cce62bd86p+6);
    S = __builtin_fma(S, r2, 0x1.466bc6775aae2p+6);
    S = __builtin_fma(S, r2, -0x1.4abbce625be53p+5);
    S = __builtin_fma(S, r2, 0x1.921fb54442d18p+2);
    double C = 0x1.20c62c2f2d7f5p-2;
    C = __builtin_fma(C, r2, -0x1.b6e24f44b128fp+0);
    C = __builtin_fma(C, r2, 0x1.f9d38a3763cc3p+2);
    C = __builtin_fma(C, r2, -0x1.a6d1f2a204a8cp+4);
    C = __builtin_fma(C, r2, 0x1.e1f506891babbp+5);
    C = __builtin_fma(C, r2, -0x1.55d3c7e3cbffap+6);
    C = __builtin_fma(C, r2, 0x1.03c1f081b5ac4p+6);
    C = __builtin_fma(C, r2, -0x1.3bd3cc9be45dep+4);
    C = __builtin_fma(C, r2, 1.0);
    const double sn = r * S;
    const int qi = ((int)q) & 3;
    const double a = (qi & 1) ? C : sn;    // |sin| part
    const double b = (qi & 1) ? sn : C;    // |cos| part
    s_out = (qi & 2) ? -a : a;
    c_out = (qi == 1 || qi == 2) ? -b : b;
}

// log((w + 0.5) 2^-32) for the Box-Muller radius: table-driven (bm_log_table.inc), division- and
// branch-free, no special cases (the argument is always in [2^-33, 1)).  x = w + 0.5 = 2^e m, the
// top 9 mantissa bits select c (c = 1 for the intervals next to 1, so results near 0 keep full
// relative precision); r = m' inv_c - 1 with |r| < 2^-9; log = e ln2 + T + log1p(r), log1p by a
// degree-6 Horner polynomial (truncation r^7/7 < 2^-54 |r|).  Round 2: 512 rows and degree 6 in place of 128
// rows and degree 8 (two fmas fewer per normal pair).  kBmLogTab (128 rows) stays for det_log_tab.
static __device__ const double kBmLogTab[128][4] = {BM_LOG_TABLE_ROWS};
static __device__ const double kBmLog512Tab[512][4] = {BM_LOG512_TABLE_ROWS};

__device__ __forceinline__ double bm_log_u32(uint32_t w, const double (*tab)[4] = kBmLog512Tab) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double x = (double)w + 0.5;                                   // exact
    const uint64_t b = d2bits(x);
    // all on the high word xh (x > 0): top9 = xh[19:11], up = xh[19] (m in [1.5, 2): use m/2), e from xh[30:20];
    // m's high word is xh's mantissa bits under exponent 0x3ff - up = 0x3ff ^ up
    const uint32_t xh = (uint32_t)(b >> 32);
    const uint32_t up = (xh >> 19) & 1u;
    const int e = (int)(xh >> 20) + (int)up - (1023 + 32);
    const uint32_t mhi = ((0x3ffu ^ up) << 20) | (xh & 0x000fffffu);
    const double m = bits2d(((uint64_t)mhi << 32) | (b & 0xffffffffull));
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    const f64x2_t* row = reinterpret_cast<const f64x2_t*>(reinterpret_cast<const char*>(tab) + ((xh >> 6) & 0x3fe0u));
    const f64x2_t a = row[0], t = row[1];                               // (inv_c, T_hi), (T_lo, 0)
    const double r = __builtin_fma(m, a.x, -1.0);
    double P = __builtin_fma(r, -0x1.5555555555555p-3, 0x1.999999999999ap-3);   // -1/6, 1/5
    P = __builtin_fma(r, P, -0x1p-2);                                   // -1/4
    P = __builtin_fma(r, P, 0x1.5555555555555p-2);                      // 1/3
    P = __builtin_fma(r, P, -0x1p-1);                                   // -1/2
    const double p = __builtin_fma(r * r, P, r);
    const double de = (double)e;
    const double hi = __builtin_fma(de, ln2_hi, a.y);
    const double lo = __builtin_fma(de, ln2_lo, t.x) + p;
    return hi + lo;
}

// The Box-Muller radius^2, -2 log((w + 0.5) 2^-32): bm_log_u32 with every operation scaled by -2 -- the table rows
// (kBmRad512Tab = -2 x kBmLog512Tab's), the reduced argument r2 = fma(m, -2 inv_c, 2) = -2 r, the log1p stages
// (each an exact power-of-two multiple of bm_log_u32's) and the e ln2 terms -- so the result is bitwise
// -2.0 * bm_log_u32(w) (the oracle's -2.0 * orc_bm_log_u32) without the final multiply.  Round 3.
static __device__ const double kBmRad512Tab[512][4] = {BM_RAD512_TABLE_ROWS};

__device__ __forceinline__ double bm_rad2_u32(uint32_t w, const double (*tab)[4] = kBmRad512Tab) {
    const double m2ln2_hi = -0x1.62e42fee00000p+0;                      // -2 ln2_hi, -2 ln2_lo
    const double m2ln2_lo = -0x1.a39ef35793c76p-32;
    const double x = (double)w + 0.5;
    const uint64_t b = d2bits(x);
    const uint32_t xh = (uint32_t)(b >> 32);
    const uint32_t up = (xh >> 19) & 1u;
    const int e = (int)(xh >> 20) + (int)up - (1023 + 32);
    const uint32_t mhi = ((0x3ffu ^ up) << 20) | (xh & 0x000fffffu);
    const double m = bits2d(((uint64_t)mhi << 32) | (b & 0xffffffffull));
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    const f64x2_t* row = reinterpret_cast<const f64x2_t*>(reinterpret_cast<const char*>(tab) + ((xh >> 6) & 0x3fe0u));
    const f64x2_t a = row[0], t = row[1];                               // (-2 inv_c, -2 T_hi), (-2 T_lo, 0)
    const double r2 = __builtin_fma(m, a.x, 2.0);                       // -2 r
    double Q = __builtin_fma(r2, 0x1.5555555555555p-8, 0x1.999999999999ap-7);   // P stages x 1/16, -1/8, 1/4, -1/2
    Q = __builtin_fma(r2, Q, 0x1p-5);
    Q = __builtin_fma(r2, Q, 0x1.5555555555555p-4);
    Q = __builtin_fma(r2, Q, 0x1p-2);
    const double p2 = __builtin_fma(r2 * r2, Q, r2);                   // -2 log1p(r)
    const double de = (double)e;
    const double hi = __builtin_fma(de, m2ln2_hi, a.y);
    const double lo = __builtin_fma(de, m2ln2_lo, t.x) + p2;
    return hi + lo;
}

// The Box-Muller radius sqrt(-2 log u) as a polynomial (round 3; scripts/gen_bm_log_table.py BM_RADP / BM_RADT):
// side = w >> 31 folds u >= 1/2 onto 1 - u = (~w + 1/2) 2^-32 (exact), so both halves are x 2^-32 with x = v + 1/2
// in [1/2, 2^31).  v >= 2^21 (all but 2^-11 of the draws): the binade e = 21..30 and top 5 mantissa bits k of v
// pick a degree-7 polynomial in the exact residual t = m - (1 + (2k+1)/64), |t| <= 1/64, of v's mantissa (the 1/2
// is inside the polynomial, so x is never formed); kBmRadPTab, the table a kernel may stage into LDS, rows chunk-
// major (row i's chunk j -- (a0, a1), (a2, a3), (a4, a5), (a6, a7) -- at j * NROWS + i, so a wave's gathers of one
// chunk spread over the LDS banks).  v < 2^21 re-reads its coefficients and residual from the global tail table
// (binades -1..20 of x itself) on the lanes that need it: four loads under a branch a wave takes with probability
// 3% per radius, the polynomial itself shared.  <= 1 ulp (1.4 ulp on the few segments whose radius crosses a power
// of two: a0 is one double); 16 VALU operations against 32 for a log and an IEEE sqrt.
static __device__ const double kBmRadPTab[4 * BM_RADP_NROWS][2] = {BM_RADP_TABLE_ROWS};
static __device__ const double kBmRadTTab[4 * BM_RADT_NROWS][2] = {BM_RADT_TABLE_ROWS};

struct RadTab {                      // the radius polynomial table: a kernel's LDS copy or the global one
    const double (*d)[2];
    bool lds;                        // LDS: an out-of-range row (the tail lanes') reads harmlessly; global: clamped
};
__device__ __forceinline__ RadTab rad_tab_global() { return RadTab{kBmRadPTab, false}; }

__device__ __forceinline__ double bm_radius_u32(uint32_t w, RadTab rt) {
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    const uint32_t sm = (uint32_t)((int32_t)w >> 31);                   // side mask
    const uint32_t v = w ^ sm;
    const double y = (double)v;                                         // exact
    const uint64_t b = d2bits(y);
    const uint32_t yh = (uint32_t)(b >> 32);
    const bool tail = v < (1u << 21);
    // byte offset of row (yh >> 15) - ((1023 + 21) << 5) + side * NROWS/2 (yh >> 15 = biased exponent, k)
    constexpr uint32_t kOff0 = 0u - ((uint32_t)((1023 + 21) << 5) << 4);
    constexpr uint32_t kOff1 = kOff0 + (uint32_t)(BM_RADP_NROWS / 2) * 16u;
    // the side select as one v_bfi_b32, the offset as one v_lshl_add_u32 and the residual's high word as one
    // v_and_or_b32: the compiler spends two instructions on each (VOP3 takes no literal on gfx9)
    uint32_t sel;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(sel) : "v"(sm), "v"(kOff1), "s"(kOff0));
    uint32_t off;
    asm("v_lshl_add_u32 %0, %1, 4, %2" : "=v"(off) : "v"(yh >> 15), "v"(sel));   // ((yh >> 15) << 4) + sel
    uint32_t th = yh;                                                   // in place: y's high word is dead now
    asm("v_and_or_b32 %0, %0, %1, %2" : "+v"(th) : "s"(0x7fffu), "v"(0x3ff00000u));
    if (!rt.lds) off = tail ? 0u : off;
    double t = bits2d(((uint64_t)th << 32) | (b & 0xffffffffull)) - (1.0 + 1.0 / 64.0);     // exact (Sterbenz)
    const char* base = reinterpret_cast<const char*>(rt.d) + off;
    f64x2_t c0 = *reinterpret_cast<const f64x2_t*>(base);
    f64x2_t c1 = *reinterpret_cast<const f64x2_t*>(base + 16 * BM_RADP_NROWS);
    f64x2_t c2 = *reinterpret_cast<const f64x2_t*>(base + 32 * BM_RADP_NROWS);
    f64x2_t c3 = *reinterpret_cast<const f64x2_t*>(base + 48 * BM_RADP_NROWS);
    if (tail) {
        // x = v + 1/2 itself in the tail table.  The volatile asm keeps this arithmetic inside the branch (the
        // compiler would otherwise hoist it onto every lane), and the loads are explicit: as plain C++ they would
        // be merged with the main-table loads above into one load through a selected pointer.  (A fully unrolled
        // region with many of these branches can still spill: the fused RAM update draws its normals before it,
        // samplers.hpp ram_body kZLds.)
        uint32_t vv = v;                                                // (v again, not y: y's registers are reused)
        asm volatile("" : "+v"(vv));
        const double x = (double)vv + 0.5;
        const uint64_t bx = d2bits(x);
        const uint32_t xh = (uint32_t)(bx >> 32);
        const uint32_t rw = (uint32_t)((int)(xh >> 15) - ((1023 - 1) << 5)) * 16u + (sm & (16u * (BM_RADT_NROWS / 2)));
        t = bits2d(((uint64_t)((xh & 0x7fffu) | 0x3ff00000u) << 32) | (bx & 0xffffffffull)) - (1.0 + 1.0 / 64.0);
        asm volatile(
            "global_load_dwordx4 %0, %4, %5\n\t"
            "global_load_dwordx4 %1, %4, %6\n\t"
            "global_load_dwordx4 %2, %4, %7\n\t"
            "global_load_dwordx4 %3, %4, %8\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
            : "v"(rw), "s"(&kBmRadTTab[0][0]), "s"(&kBmRadTTab[BM_RADT_NROWS][0]),
              "s"(&kBmRadTTab[2 * BM_RADT_NROWS][0]), "s"(&kBmRadTTab[3 * BM_RADT_NROWS][0])
            : "memory");
    }
    double q = __builtin_fma(c3.y, t, c3.x);
    q = __builtin_fma(q, t, c2.y);
    q = __builtin_fma(q, t, c2.x);
    q = __builtin_fma(q, t, c1.y);
    q = __builtin_fma(q, t, c1.x);
    q = __builtin_fma(q, t, c0.y);
    double r = __builtin_fma(q, t, c0.x);
    asm volatile("" : "+v"(r));     // computed here: not sunk past the next radius's branch with its coefficients live
    return r;
}

typedef double dm_f64x2 __attribute__((ext_vector_type(2)));

// exp for the logistic likelihood (prob = 1/(1+exp(-X*vars)), examples/logistic_regression.jl:19), table-
// driven: x = (64 E + j) ln2/64 + r with |r| <= ln2/128, exp(x) = 2^E (T_hi + (T_hi expm1(r) + T_lo)), where
// (T_hi, T_lo) = 2^(j/64) (EXP2_TABLE_ROWS) and expm1(r) is Taylor to degree 6 (truncation < 2^-66 relative).
// The argument is clamped to [-746, 710], so overflow and underflow come out of the 2^E scaling itself (inf,
// 0); NaN passes through.  Stages as det_exp (the caller may interleave work between them); oracle twin
// orc_exp_tab.  Against det_exp: a 6-term instead of a 13-term polynomial.
static __device__ const double kExp2Tab[64][2] = {EXP2_TABLE_ROWS};

struct ExpTState {
    double x, r, em;
    dm_f64x2 t;
    int e;
};
__device__ __forceinline__ void det_exp_tab_s1(double x, ExpTState& E, const double (*tab)[2] = kExp2Tab) {
    const double k64 = 0x1.71547652b82fep+6;                 // 64 / ln2
    const double l_hi = 0x1.62e42fee00000p-7;                // ln2 / 64, high part (kd l_hi is exact)
    const double l_lo = 0x1.a39ef35793c76p-39;               // ln2 / 64, low part
    const double shifter = 0x1.8p52;
    const double xc = __builtin_fmin(__builtin_fmax(x, -746.0), 710.0);
    const double kd = __builtin_fma(xc, k64, shifter) - shifter;
    const int k = (int)kd;
    E.t = *reinterpret_cast<const dm_f64x2*>(tab[k & 63]);
    E.e = k >> 6;                                            // floor(k / 64), in [-1077, 1024]
    const double r = __builtin_fma(-kd, l_hi, xc);
    E.r = __builtin_fma(-kd, l_lo, r);
    E.x = x;
}
__device__ __forceinline__ void det_exp_tab_s2(ExpTState& E) {
    const double r = E.r;
    double P = __builtin_fma(r, 0x1.6c16c16c16c17p-10, 0x1.1111111111111p-7);   // 1/720, 1/120
    P = __builtin_fma(r, P, 0x1.5555555555555p-5);                               // 1/24
    P = __builtin_fma(r, P, 0x1.5555555555555p-3);                               // 1/6
    P = __builtin_fma(r, P, 0.5);
    P = __builtin_fma(r, P, 1.0);
    E.em = r * P;                                                                // expm1(r)
}
__device__ __forceinline__ double det_exp_tab_fin(const ExpTState& E) {
    const int e1 = E.e / 2, e2 = E.e - e1;
    double res = E.t.x + __builtin_fma(E.t.x, E.em, E.t.y);
    res = (res * pow2i(e1)) * pow2i(e2);
    return E.x != E.x ? E.x : res;
}
__device__ __forceinline__ double det_exp_tab(double x, const double (*tab)[2] = kExp2Tab) {
    ExpTState E;
    det_exp_tab_s1(x, E, tab);
    det_exp_tab_s2(E);
    return det_exp_tab_fin(E);
}

// log of v in [0, 1] for the logistic Bernoulli term (logpdf(Bernoulli(prob), y) = log(prob) or log(1 - prob)):
// bm_log_u32's table reduction applied to any double, v = 2^e m; a subnormal v is pre-scaled by 2^54 (a
// select), log(0) = -inf, NaN passes through.  Division-free (det_log has one IEEE division); stages as
// det_log; oracle twin orc_log_tab.  Not for negative or infinite v (unreachable: v = p or 1 - p, p in [0, 1]).
struct LogTState {
    double v, m, p;
    dm_f64x2 a, t;
    int e;
};
#ifndef GLM_LOG_FREXP
#define GLM_LOG_FREXP 0
#endif
__device__ __forceinline__ void det_log_tab_s1(double v, LogTState& L, const double (*tab)[4] = kBmLogTab) {
#if GLM_LOG_FREXP
    // round-1 experiment, rebuilt for the fault investigation (not the shipped form): exponent and
    // mantissa from the hardware frexp, v = mh 2^eh with mh in [0.5, 1); m' = 2 mh in [1, 2) as below
    const double mh = __builtin_amdgcn_frexp_mant(v);
    const int eh = __builtin_amdgcn_frexp_exp(v);
    const uint64_t b = d2bits(mh);
    const uint32_t top7 = (uint32_t)(b >> 45) & 0x7fu;
    const uint32_t up = top7 >> 6;
    L.e = eh - 1 + (int)up;
    L.m = bits2d((b & 0x000fffffffffffffull) | ((uint64_t)(0x3ffu - up) << 52));
    const dm_f64x2* row = reinterpret_cast<const dm_f64x2*>(tab[top7]);
    L.a = row[0];
    L.t = row[1];
    L.v = v;
#else
    const bool sub = v < 0x1p-1022;                                  // zero or subnormal
    const double xs = sub ? v * 0x1p54 : v;
    const uint64_t b = d2bits(xs);
    const uint32_t top7 = (uint32_t)(b >> 45) & 0x7fu;
    const uint32_t up = top7 >> 6;                                   // m in [1.5, 2): use m/2
    L.e = (int)(uint32_t)(b >> 52) - 1023 + (int)up - (sub ? 54 : 0);
    L.m = bits2d((b & 0x000fffffffffffffull) | ((uint64_t)(0x3ffu - up) << 52));
    const dm_f64x2* row = reinterpret_cast<const dm_f64x2*>(tab[top7]);
    L.a = row[0];                                                    // (inv_c, T_hi)
    L.t = row[1];                                                    // (T_lo, 0)
    L.v = v;
#endif
}
__device__ __forceinline__ void det_log_tab_s2(LogTState& L) {
    const double r = __builtin_fma(L.m, L.a.x, -1.0);
    double P = __builtin_fma(r, -0x1p-3, 0x1.2492492492492p-3);         // -1/8, 1/7
    P = __builtin_fma(r, P, -0x1.5555555555555p-3);                     // -1/6
    P = __builtin_fma(r, P, 0x1.999999999999ap-3);                      // 1/5
    P = __builtin_fma(r, P, -0x1p-2);                                   // -1/4
    P = __builtin_fma(r, P, 0x1.5555555555555p-2);                      // 1/3
    P = __builtin_fma(r, P, -0x1p-1);                                   // -1/2
    L.p = __builtin_fma(r * r, P, r);                                   // log1p(r)
}
__device__ __forceinline__ double det_log_tab_fin(const LogTState& L) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double de = (double)L.e;
    const double hi = __builtin_fma(de, ln2_hi, L.a.y);
    const double lo = __builtin_fma(de, ln2_lo, L.t.x) + L.p;
    const double res = L.v == 0.0 ? -__builtin_inf() : hi + lo;
    return L.v != L.v ? L.v : res;
}
__device__ __forceinline__ double det_log_tab(double v, const double (*tab)[4] = kBmLogTab) {
    LogTState L;
    det_log_tab_s1(v, L, tab);
    det_log_tab_s2(L);
    return det_log_tab_fin(L);
}

// The logistic Bernoulli term of one observation (examples/logistic_regression.jl:19-21) and its eta-derivative
// (MCMCDerivRules.jl:111): lp = logpdf(Bernoulli(p), y), p = 1/(1+exp(-s eta)) (s = the link sign), and
// s (y - p).  The staged tile carries w = s (2y - 1) instead of y (glm_layout.hpp); with u = -w eta
//     lp = -softplus(u) = -(max(u, 0) + f(|u|)),          f(v) = log1p(exp(-v)),
//     s (y - p) = w sigmoid(u) = w (u >= 0 ? 1 - g : g),  g(v) = 1/(1+exp(v)) = -f'(v).
// v = min(|u|, 40) splits as j/8 + t (|t| <= 1/16, j from the low word of a shifter fma, t exact) and row j of
// kSoftplusTab holds the degree-9 polynomial of f in t (Chebyshev interpolation, scripts/gen_softplus_table.py): one
// Horner pass with derivative gives f = P(t) (<= 1.4 ulp) and g = -P'(t) (<= 1.9 ulp).  No exp, log or division.
// Beyond v = 40, f and g (< 4.3e-18) keep their v = 40 values.  The reference's own arithmetic (p rounded, then
// log(p) or log(1 - p)) makes the term -Inf where p rounds to 1 with y = 0 or to 0 with y = 1: u >= T(y)
// (glm_layout.hpp logi_bound).  The kernels keep that: the tile carries b = -T(y) beside w and a lane whose max of u + b over its
// observations is >= 0 contributes -Inf, so LLAcc puts the point out of support exactly where the reference does.
// A NaN eta is not propagated (fmin): it needs X beta to overflow with mixed signs, and mcmc_model_create refuses
// data for which that can happen at any beta of finite prior density (row L1 norm x sqrt(DBL_MAX) prior_sigma <
// 2^1022; X and Y finite).  Stages as det_exp (the caller interleaves work between them); oracle twin orc_logi.
static __device__ const double kSoftplusTab[SP_NROWS][10] = {SP_TABLE_ROWS};


struct LogiState {
    double u, t, p, d;
    const dm_f64x2* row;
};
__device__ __forceinline__ void det_logi_s1(double eta, double w, LogiState& S, const double (*tab)[10] = kSoftplusTab) {
    const double shifter = 0x1.8p52;
    const double u = -(w * eta);
    const double vs = __builtin_fmin(__builtin_fabs(u), (double)SP_VMAX);
    const double tt = __builtin_fma(vs, (double)SP_SEG, shifter);           // 1.5 2^52 + j, j = round(8 v)
    const uint32_t j = (uint32_t)d2bits(tt);                                   // in [0, 320]
    const double kd = tt - shifter;
    S.t = __builtin_fma(-kd, 1.0 / SP_SEG, vs);                                // exact
    S.row = reinterpret_cast<const dm_f64x2*>(tab[j]);
    S.u = u;
}
// Horner with derivative over c9 .. c5
__device__ __forceinline__ void det_logi_s2(LogiState& S) {
    const double t = S.t;
    const dm_f64x2 c89 = S.row[4], c67 = S.row[3], c45 = S.row[2];
    double p = c89.y, d = c89.y;
    p = __builtin_fma(p, t, c89.x);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c67.y);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c67.x);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c45.y);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c45.x);
    S.p = p;
    S.d = d;
}
// c4 .. c0, then the term and the weight
__device__ __forceinline__ void det_logi_fin(const LogiState& S, double w, double& term, double& rv) {
    const double t = S.t;
    const dm_f64x2 c23 = S.row[1], c01 = S.row[0];
    double p = S.p, d = S.d;
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c23.y);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c23.x);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c01.y);
    d = __builtin_fma(d, t, p); p = __builtin_fma(p, t, c01.x);
    term = -(__builtin_fmax(S.u, 0.0) + p);                                   // -softplus(u)
    const double sig = S.u >= 0.0 ? 1.0 + d : -d;                              // 1 - g or g
    rv = w * sig;
}
__device__ __forceinline__ void det_logi(double eta, double w, double& term, double& rv,
                                         const double (*tab)[10] = kSoftplusTab) {
    LogiState S;
    det_logi_s1(eta, w, S, tab);
    det_logi_s2(S);
    det_logi_fin(S, w, term, rv);
}

// sin, cos of 2 pi w 2^-32 (the Box-Muller angle), table-driven: the angle splits as k/1024 + j 2^-32 turns
// with k = (w + 2^21) >> 22 and |j| <= 2^21, so r = 2 pi j 2^-32 has |r| <= 2 pi 2^-11.  The row of k gives
// (sin a, cos a) (scripts/gen_bm_log_table.py, full circle: no quadrant selects); sin r = r - r^3/6 + r^5/120
// (truncation r^7/5040 < 2^-70) and cos r = 1 - r^2/2 + r^4/24 (truncation r^6/720 < 2^-59), in j;
// sin(a+r) = sa cos r + ca sin r, cos(a+r) = ca cos r - sa sin r, one fma each (within 2.3e-16 absolute: cos r
// rounded to a double).  Round 2: 1024 rows in place of 256; round 3: polynomials in j, 15 VALU operations.
static __device__ const double kBmSinCos1024Tab[1024][2] = {BM_SINCOS1024_TABLE_ROWS};

// sin / cos of r = 2 pi j 2^-32 as polynomials in the integer j (round 3; RN of 2 pi 2^-32 times 1, -1/6, 1/120 and
// of its square times -1/2, 1/24, mpmath)
constexpr double kSinJ1 = 0x1.921fb54442d18p-30, kSinJ3 = -0x1.4abbce625be53p-91, kSinJ5 = 0x1.466bc6775aae2p-154;
constexpr double kCosJ2 = -0x1.3bd3cc9be45dep-60, kCosJ4 = 0x1.03c1f081b5ac4p-122;

__device__ __forceinline__ void det_sincos2pi_u32(uint32_t w, double& s_out, double& c_out,
                                                  const double (*sct)[2] = kBmSinCos1024Tab) {
    // j = the sign-extended low 22 bits of w (w - 2^22 k), one v_bfe_i32, exact in a double, and so is j^2; the
    // polynomials are in j with 2 pi 2^-32 folded into their coefficients: sin r = j (A1 + j^2 (A3 + j^2 A5)),
    // cos r = 1 + j^2 (B2 + j^2 B4), r = 2 pi j 2^-32, |r| <= 2 pi 2^-11.  The row's byte offset 16 k is
    // (w - j) >> 18 (w - j = 2^22 k mod 2^32), two instructions from j.
    const int32_t ji = ((int32_t)(w << 10)) >> 10;
    const uint32_t off = (w - (uint32_t)ji) >> 18;                     // 16 k
    const double j = (double)ji;
    const double j2 = j * j;
    const double sr = j * __builtin_fma(j2, __builtin_fma(j2, kSinJ5, kSinJ3), kSinJ1);
    const double cr = __builtin_fma(j2, __builtin_fma(j2, kCosJ4, kCosJ2), 1.0);
    typedef double f64x2_t __attribute__((ext_vector_type(2)));
    const f64x2_t a = *reinterpret_cast<const f64x2_t*>(reinterpret_cast<const char*>(sct) + off);   // (sin a, cos a)
    s_out = __builtin_fma(a.x, cr, a.y * sr);
    c_out = __builtin_fma(a.y, cr, -(a.x * sr));
}

// IEEE sqrt of a positive normal finite x: the hardware rsq estimate refined by the same Newton/fma
// sequence hipcc emits for __builtin_sqrt (Goldschmidt, then two residual corrections), without its
// guards -- the 2^256 pre-scale of x < 2^-767 and the 0/inf class selects -- which never fire for the
// Box-Muller radius argument -2 log u in [2.3e-10, 46].  Correctly rounded, so the oracle's sqrt() is its
// twin (tests/test_gpu_parity.py checks it bit for bit over the normal range).
__device__ __forceinline__ double sqrt_pos_normal(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double e = __builtin_fma(-g, g, x);
    g = __builtin_fma(e, h, g);
    e = __builtin_fma(-g, g, x);
    return __builtin_fma(e, h, g);
}

// Two Box-Muller pairs from one Philox block: radius sqrt(-2 log u1), u1 = (w.x + 1/2) 2^-32 in (0,1);
// angle 2 pi u2, u2 = w.y 2^-32.
// rt, sct: the radius polynomial (bm_radius_u32) and angle tables, in global memory (default) or a kernel's LDS copies
__device__ __forceinline__ void normals4(const u32x4& w, double& z0, double& z1, double& z2, double& z3,
                                         RadTab rt = rad_tab_global(),
                                         const double (*sct)[2] = kBmSinCos1024Tab) {
    {
        const double rad = bm_radius_u32(w.x, rt);
        double s, c;
        det_sincos2pi_u32(w.y, s, c, sct);
        z0 = rad * c; z1 = rad * s;
    }
    {
        const double rad = bm_radius_u32(w.z, rt);
        double s, c;
        det_sincos2pi_u32(w.w, s, c, sct);
        z2 = rad * c; z3 = rad * s;
    }
    asm volatile("" : "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));   // likewise the products
}

// ratio > det_log(u), exactly (the RWM / MALA test `ratio > log(rand())`, RWM.jl:63, MALA.jl:108).  A
// single-precision log2 (v_log_f32) decides it when ratio is not within E = 2^-16 (1 + |L|) of L = log2f(u) ln2:
// |L - log u| <= ln2 (2^-23 |log2 u| + 2^-24 log2 e) plus the 1-ulp error of det_log is hundreds of times smaller
// than E, so a decided test agrees with the exact one.  The rest (probability ~1e-5 per test; u = 0; NaN ratios)
// takes det_log, on the lanes that need it.
// The undecided lanes' exact test, out of line: inlined, its det_log polynomial constants were hoisted out of the
// step loops into VGPRs and spilled (the metric kernel lpp_rwm<4, true, IsoDot, true> stored 64 B a lane to scratch
// per launch, ~134 MB at 2^21 lanes, to reload them on this 1-in-10^5 path).  A call saves the caller's live
// registers only on the lanes' rare way in.
__device__ __attribute__((noinline)) bool gt_det_log_exact(double ratio, double u) { return ratio > det_log(u); }
__device__ __forceinline__ bool gt_det_log(double ratio, double u) {
    const double L = (double)__builtin_amdgcn_logf((float)u) * 0x1.62e42fefa39efp-1;
    const double E = 0x1p-16 * (1.0 + __builtin_fabs(L));
    const bool sure_acc = ratio > L + E;
    const bool sure_rej = ratio <= L - E;
    bool acc = sure_acc;
    if (!sure_acc && !sure_rej) acc = gt_det_log_exact(ratio, u);
    return acc;
}

__device__ __forceinline__ double round_away(double x) {
    double t = __builtin_trunc(x);
    const double fr = x - t;
    if (fr >= 0.5) t += 1.0;
    else if (fr <= -0.5) t -= 1.0;
    return t;
}

// erfc, erfcx, log1p and the normal log-cdf of the probit model (examples/probit_regression.jl:26-30): the oracle's
// orc_erfcx_ge_half / orc_erfc / orc_log1p / orc_normlogcdf operation for operation (scripts/gen_erfc_table.py;
// DESIGN.md §3).
static __device__ const double kErfcTaylor[14] = {ERFC_TAYLOR_COEFS};
static __device__ const double kErfcPoly[32][13] = {ERFC_POLY_ROWS};
__device__ __forceinline__ double det_erfcx_ge_half(double x) {     // x >= 1/2
    if (x >= 128.0) {
        const double v = 1.0 / (x * x);
        const double s = __builtin_fma(__builtin_fma(__builtin_fma(v, -1.875, 0.75), v, -0.5), v, 1.0);
        return s / (x * 0x1.c5bf891b4ef6bp+0);
    }
    const uint64_t bx = d2bits(x);
    const uint32_t hx = (uint32_t)(bx >> 32);
    const int i = (int)(hx >> 18) - (1022 << 2);                   // binade quarter, 0..31
    const double c = bits2d((uint64_t)((hx & 0xfffc0000u) | 0x00020000u) << 32);
    const double sc = bits2d((uint64_t)(2046u - (hx >> 20) + 3u) << 52);   // 2^(3-e)
    const double t = (x - c) * sc;                                  // exact, in [-1, 1]
    const double* P = kErfcPoly[i];
    double p = P[12];
#pragma unroll
    for (int n = 11; n >= 0; --n) p = __builtin_fma(p, t, P[n]);
    return p;
}
__device__ __forceinline__ double det_erfc(double a) {
    const double x = __builtin_fabs(a);
    double r;
    if (x < 0.5) {
        const double u = x * x;
        double q = kErfcTaylor[13];
#pragma unroll
        for (int n = 12; n >= 0; --n) q = __builtin_fma(q, u, kErfcTaylor[n]);
        r = 1.0 - x * q;
    } else if (x < 32.0) {
        const double p = det_erfcx_ge_half(x);
        const double xh = bits2d(d2bits(x) & 0xfffffffff8000000ull);   // 26 significant bits: xh * xh exact
        const double e1 = det_exp(-(xh * xh));
        const double e2 = det_exp(-((x - xh) * (x + xh)));
        r = (e1 * e2) * p;
    } else {
        r = 0.0;
    }
    r = a < 0.0 ? 2.0 - r : r;
    return a != a ? a : r;
}
__device__ __forceinline__ double det_log1p(double t) {
    const double u = 1.0 + t;
    return u == 1.0 ? t : det_log(u) * (t / (u - 1.0));
}
__device__ __forceinline__ double det_normlogcdf(double z) {
    const double invsqrt2 = 0x1.6a09e667f3bcdp-1;
    const double r = z < -1.0 ? det_log(det_erfcx_ge_half(-z * invsqrt2) / 2.0) - (z * z) / 2.0
                              : det_log1p(-det_erfc(z * invsqrt2) / 2.0);
    return z != z ? z : r;
}

}  // namespace mcmc
