/*
 * oracle/detmath.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the build's random-number and fp64 math specification
 * (DESIGN.md §3 "RNG and deterministic math").  The reference (MCMC.jl, Julia
 * 0.2) draws with dSFMT + ziggurat `randn` / `rand` (src/samplers/RWM.jl:59,63)
 * and evaluates `log`/`exp` with openlibm; neither can run here (no Julia), so
 * the build defines its own counter-based stream and its own fp64 kernels, and
 * this header restates them operation for operation, so that the HIP path and
 * the oracle produce bit-identical draws and accept decisions.
 *
 *   Philox4x32-10 ..... Salmon et al., SC'11 (Random123); pinned by the
 *                       Random123 known-answer vectors (tests/golden/philox_kat.json)
 *   uniform52 ......... 52-bit uniform on [0,1)  (Julia `rand()` semantics: 0 possible, 1 not)
 *   det_log ........... fdlibm e_log.c algorithm (Sun, 1993), branch-free general
 *                       path, explicit fma in the polynomial
 *   det_exp ........... Cody-Waite reduction + degree-13 Taylor (fma Horner)
 *   det_sincos2pi ..... exact quarter-turn reduction + Taylor polynomials in r
 *   Box-Muller angle .. 1024-row sin/cos table + short Taylor polynomials (orc_sincos2pi_u32)
 *   Box-Muller radius . per-segment degree-7 polynomials of sqrt(-2 log u) (orc_bm_radius_u32)
 *   Box-Muller ........ normals from 32-bit uniforms, 4 normals per Philox block
 *
 * Compile with -ffp-contract=off: every fused multiply-add is an explicit fma();
 * no other product may be fused.  sqrt and '/' are IEEE correctly rounded.
 */
#ifndef MCMC_ORACLE_DETMATH_H
#define MCMC_ORACLE_DETMATH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

#include "bm_log_table.inc"
#include "erfc_table.inc"
#include "softplus_table.inc"

#define ORC_PHILOX_M0 0xD2511F53u
#define ORC_PHILOX_M1 0xCD9E8D57u
#define ORC_PHILOX_W0 0x9E3779B9u
#define ORC_PHILOX_W1 0xBB67AE85u

/* stream tags (counter word 3) */
#define ORC_TAG_NORMAL 0u   /* proposal / momentum normals            */
#define ORC_TAG_ACCEPT 1u   /* Metropolis-Hastings accept uniform      */
#define ORC_TAG_DATA   7u   /* synthetic data generation (bench configs) */

static inline void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += ORC_PHILOX_W0; k1 += ORC_PHILOX_W1; }
        uint64_t p0 = (uint64_t)ORC_PHILOX_M0 * (uint64_t)c0;
        uint64_t p1 = (uint64_t)ORC_PHILOX_M1 * (uint64_t)c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* One Philox block of the build's stream: counter = (chain, step, block, tag), key = seed. */
static inline void orc_block(uint64_t seed, uint32_t chain, uint32_t step, uint32_t block,
                             uint32_t tag, uint32_t out[4]) {
    uint32_t ctr[4] = {chain, step, block, tag};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    orc_philox4x32_10(ctr, key, out);
}

static inline double orc_bits2d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static inline uint64_t orc_d2bits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

/* 52-bit uniform on [0,1) from two 32-bit words: the top 52 bits of a:b as the mantissa of a double in [1, 2),
   less 1 (device twin: uniform52). */
static inline double orc_uniform52(uint32_t a, uint32_t b) {
    uint64_t bits = ((uint64_t)(0x3ff00000u | (a >> 12)) << 32) | (uint64_t)((a << 20) | (b >> 12));
    return orc_bits2d(bits) - 1.0;
}
/* 32-bit uniform on (0,1): never 0, never 1. */
static inline double orc_uniform32_open(uint32_t a) { return ((double)a + 0.5) * 0x1p-32; }
/* 32-bit uniform on [0,1). */
static inline double orc_uniform32(uint32_t a) { return (double)a * 0x1p-32; }

/* 2^k for k in [-1022, 1023], built from bits. */
static inline double orc_pow2i(int k) { return orc_bits2d((uint64_t)(k + 1023) << 52); }

/* ---------------------------------------------------------------- log */
static inline double orc_log(double x) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2,
                 Lg3 = 0x1.2492494229359p-2, Lg4 = 0x1.c71c51d8e78afp-3,
                 Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    if (x != x) return x;                                  /* NaN  */
    if (x < 0.0) return orc_bits2d(0x7ff8000000000000ull); /* NaN  */
    if (x == 0.0) return -INFINITY;
    uint64_t bx = orc_d2bits(x);
    if (bx >= 0x7ff0000000000000ull) return x;             /* +inf */
    int k = 0;
    if (bx < 0x0010000000000000ull) {                      /* subnormal: scale by 2^54 */
        x = x * 0x1p54; k = -54; bx = orc_d2bits(x);
    }
    uint32_t hx = (uint32_t)(bx >> 32);
    k += (int)(hx >> 20) - 1023;
    hx &= 0x000fffffu;
    uint32_t i = (hx + 0x95f64u) & 0x100000u;              /* != 0 iff mantissa >= sqrt(2) */
    uint64_t nb = ((uint64_t)(hx | (i ^ 0x3ff00000u)) << 32) | (bx & 0xffffffffull);
    double m = orc_bits2d(nb);                             /* m in [sqrt(2)/2, sqrt(2)) */
    k += (int)(i >> 20);
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double dk = (double)k;
    double z = s * s;
    double w = z * z;
    double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
    double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* ---------------------------------------------------------------- exp */
static inline double orc_exp(double x) {
    const double inv_ln2 = 0x1.71547652b82fep+0;
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    const double shifter = 0x1.8p52;
    if (x != x) return x;
    if (x > 709.782712893384) return INFINITY;
    if (x < -745.1332191019412) return 0.0;
    double t = fma(x, inv_ln2, shifter);
    double kd = t - shifter;                               /* nearest integer to x/ln2 */
    int k = (int)kd;
    double r = fma(-kd, ln2_hi, x);
    r = fma(-kd, ln2_lo, r);
    double p = 0x1.6124613a86d09p-33;                      /* 1/13! */
    p = fma(p, r, 0x1.1eed8eff8d898p-29);                  /* 1/12! */
    p = fma(p, r, 0x1.ae64567f544e4p-26);                  /* 1/11! */
    p = fma(p, r, 0x1.27e4fb7789f5cp-22);                  /* 1/10! */
    p = fma(p, r, 0x1.71de3a556c734p-19);                  /* 1/9!  */
    p = fma(p, r, 0x1.a01a01a01a01ap-16);                  /* 1/8!  */
    p = fma(p, r, 0x1.a01a01a01a01ap-13);                  /* 1/7!  */
    p = fma(p, r, 0x1.6c16c16c16c17p-10);                  /* 1/6!  */
    p = fma(p, r, 0x1.1111111111111p-7);                   /* 1/5!  */
    p = fma(p, r, 0x1.5555555555555p-5);                   /* 1/4!  */
    p = fma(p, r, 0x1.5555555555555p-3);                   /* 1/3!  */
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    int k1 = k / 2, k2 = k - k1;                           /* k in [-1075,1024] */
    return (p * orc_pow2i(k1)) * orc_pow2i(k2);
}

/* ------------------------------------------------------- sin/cos(2*pi*u) */
/* u finite with |4u| < 2^51; used for u in [0,1). */
static inline void orc_sincos2pi(double u, double* s_out, double* c_out) {
    double q = floor(fma(u, 4.0, 0.5));
    double r = fma(q, -0.25, u);                           /* exact, r in [-1/8, 1/8] */
    double r2 = r * r;
    double S = -0x1.6fadb9f155744p-1;                      /* (2pi)^15/15!, alternating */
    S = fma(S, r2, 0x1.e8f434d018d63p+1);
    S = fma(S, r2, -0x1.e3074fde8871fp+3);
    S = fma(S, r2, 0x1.50783487ee782p+5);
    S = fma(S, r2, -0x1.32d2cce62bd86p+6);
    S = fma(S, r2, 0x1.466bc6775aae2p+6);
    S = fma(S, r2, -0x1.4abbce625be53p+5);
    S = fma(S, r2, 0x1.921fb54442d18p+2);
    double C = 0x1.20c62c2f2d7f5p-2;                       /* (2pi)^16/16! */
    C = fma(C, r2, -0x1.b6e24f44b128fp+0);
    C = fma(C, r2, 0x1.f9d38a3763cc3p+2);
    C = fma(C, r2, -0x1.a6d1f2a204a8cp+4);
    C = fma(C, r2, 0x1.e1f506891babbp+5);
    C = fma(C, r2, -0x1.55d3c7e3cbffap+6);
    C = fma(C, r2, 0x1.03c1f081b5ac4p+6);
    C = fma(C, r2, -0x1.3bd3cc9be45dep+4);
    C = fma(C, r2, 1.0);
    double sn = r * S;
    int qi = ((int)q) & 3;
    double so, co;
    switch (qi) {
        case 0:  so = sn;  co = C;   break;
        case 1:  so = C;   co = -sn; break;
        case 2:  so = -sn; co = -C;  break;
        default: so = -C;  co = sn;  break;
    }
    *s_out = so; *c_out = co;
}

/* ------------------------------------------------------- Box-Muller radius logarithm */
/* log((w + 0.5) 2^-32), w a 32-bit draw: x = w + 0.5 = 2^e m (exact); the top 9 mantissa bits pick
   the table row (scripts/gen_bm_log_table.py, BM_LOG512_TABLE_ROWS): for m >= 1.5 the reduction uses m/2 and
   e+1, and the rows next to 1 have c = 1, so a result near 0 keeps its relative precision.  r = m' inv_c - 1
   (|r| < 2^-9), log = e ln2 + (T_hi + T_lo) + log1p(r), log1p by Horner to degree 6.  The device twin is
   bm_log_u32 (csrc/detmath.hpp).  The 128-row table (top 7 bits, degree 8) stays for orc_log_tab. */
static const double orc_bm_log_tab[128][4] = {BM_LOG_TABLE_ROWS};
static const double orc_bm_log512_tab[512][4] = {BM_LOG512_TABLE_ROWS};

static inline double orc_bm_log_u32(uint32_t w) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    double x = (double)w + 0.5;
    uint64_t b;
    memcpy(&b, &x, 8);
    uint32_t top9 = (uint32_t)(b >> 43) & 0x1ffu;
    uint32_t up = top9 >> 8;
    int e = (int)(uint32_t)(b >> 52) - 1023 + (int)up - 32;
    uint64_t mb = (b & 0x000fffffffffffffull) | ((uint64_t)(0x3ffu - up) << 52);
    double m;
    memcpy(&m, &mb, 8);
    const double* row = orc_bm_log512_tab[top9];
    double r = fma(m, row[0], -1.0);
    double P = fma(r, -0x1.5555555555555p-3, 0x1.999999999999ap-3);
    P = fma(r, P, -0x1p-2);
    P = fma(r, P, 0x1.5555555555555p-2);
    P = fma(r, P, -0x1p-1);
    double p = fma(r * r, P, r);
    double de = (double)e;
    double hi = fma(de, ln2_hi, row[1]);
    double lo = fma(de, ln2_lo, row[2]) + p;
    return hi + lo;
}

/* ------------------------------------------------------- logistic-likelihood exp and log */
/* exp for the logistic likelihood: x = (64 E + j) ln2/64 + r, |r| <= ln2/128; exp(x) = 2^E (T_hi + (T_hi
   expm1(r) + T_lo)), (T_hi, T_lo) = 2^(j/64) from the generated table, expm1 by Taylor to degree 6.  x is
   clamped to [-746, 710]: overflow / underflow come out of the 2^E scaling; NaN passes.  Device twin:
   det_exp_tab (csrc/detmath.hpp). */
static const double orc_exp2_tab[64][2] = {EXP2_TABLE_ROWS};

static inline double orc_exp_tab(double x) {
    const double k64 = 0x1.71547652b82fep+6;
    const double l_hi = 0x1.62e42fee00000p-7;
    const double l_lo = 0x1.a39ef35793c76p-39;
    const double shifter = 0x1.8p52;
    double xc = fmin(fmax(x, -746.0), 710.0);
    double kd = fma(xc, k64, shifter) - shifter;
    int k = (int)kd;
    const double* t = orc_exp2_tab[k & 63];
    int e = k >> 6;                                        /* floor(k / 64): arithmetic shift */
    double r = fma(-kd, l_hi, xc);
    r = fma(-kd, l_lo, r);
    double P = fma(r, 0x1.6c16c16c16c17p-10, 0x1.1111111111111p-7);
    P = fma(r, P, 0x1.5555555555555p-5);
    P = fma(r, P, 0x1.5555555555555p-3);
    P = fma(r, P, 0.5);
    P = fma(r, P, 1.0);
    double em = r * P;
    int e1 = e / 2, e2 = e - e1;
    double res = t[0] + fma(t[0], em, t[1]);
    res = (res * orc_pow2i(e1)) * orc_pow2i(e2);
    return x != x ? x : res;
}

/* log of v in [0, 1] (the logistic Bernoulli term): orc_bm_log_u32's table reduction for any double; subnormal
   v pre-scaled by 2^54, log(0) = -inf, NaN passes.  Device twin: det_log_tab. */
static inline double orc_log_tab(double v) {
    const double ln2_hi = 0x1.62e42fee00000p-1;
    const double ln2_lo = 0x1.a39ef35793c76p-33;
    int sub = v < 0x1p-1022;
    double xs = sub ? v * 0x1p54 : v;
    uint64_t b = orc_d2bits(xs);
    uint32_t top7 = (uint32_t)(b >> 45) & 0x7fu;
    uint32_t up = top7 >> 6;
    int e = (int)(uint32_t)(b >> 52) - 1023 + (int)up - (sub ? 54 : 0);
    double m = orc_bits2d((b & 0x000fffffffffffffull) | ((uint64_t)(0x3ffu - up) << 52));
    const double* row = orc_bm_log_tab[top7];
    double r = fma(m, row[0], -1.0);
    double P = fma(r, -0x1p-3, 0x1.2492492492492p-3);
    P = fma(r, P, -0x1.5555555555555p-3);
    P = fma(r, P, 0x1.999999999999ap-3);
    P = fma(r, P, -0x1p-2);
    P = fma(r, P, 0x1.5555555555555p-2);
    P = fma(r, P, -0x1p-1);
    double p = fma(r * r, P, r);
    double de = (double)e;
    double hi = fma(de, ln2_hi, row[1]);
    double lo = fma(de, ln2_lo, row[2]) + p;
    double res = v == 0.0 ? -INFINITY : hi + lo;
    return v != v ? v : res;
}

/* The logistic Bernoulli term and its eta-derivative (examples/logistic_regression.jl:19-21, MCMCDerivRules.jl:111),
   w = s (2y - 1) (s the link sign), u = -w eta:  term = -(max(u, 0) + f(|u|)), f(v) = log1p(exp(-v)), and
   rv = w (u >= 0 ? 1 - g : g), g = -f'(v); v = min(|u|, 40) = j/8 + t, f = P_j(t) and f' = P_j'(t) from row j of the
   generated degree-9 segment polynomials (scripts/gen_softplus_table.py), one Horner pass with derivative in the
   device's order.  Device twin: det_logi (csrc/detmath.hpp). */
static const double orc_softplus_tab[SP_NROWS][10] = {SP_TABLE_ROWS};

static inline void orc_logi(double eta, double w, double* term, double* rv) {
    const double shifter = 0x1.8p52;
    const double u = -(w * eta);
    const double vs = fmin(fabs(u), (double)SP_VMAX);
    const double tt = fma(vs, (double)SP_SEG, shifter);
    const uint32_t j = (uint32_t)orc_d2bits(tt);
    const double kd = tt - shifter;
    const double t = fma(-kd, 1.0 / SP_SEG, vs);
    const double* c = orc_softplus_tab[j];
    double p = c[9], d = c[9];
    p = fma(p, t, c[8]);
    for (int k = 7; k >= 0; --k) {
        d = fma(d, t, p);
        p = fma(p, t, c[k]);
    }
    *term = -(fmax(u, 0.0) + p);
    const double sig = u >= 0.0 ? 1.0 + d : -d;
    *rv = w * sig;
}

/* ------------------------------------------------------- Box-Muller angle */
/* sin, cos of 2 pi w 2^-32: angle = k/1024 + j 2^-32 turns, k = (w + 2^21) >> 22, |j| <= 2^21; the row of k
   holds RN(sin, cos of 2 pi k/1024) (scripts/gen_bm_log_table.py, BM_SINCOS1024_TABLE_ROWS); r = 2 pi j 2^-32
   (|r| <= 2 pi 2^-11): sin r to r^5 and cos r to r^4 as polynomials in the integer j (2 pi 2^-32 folded into the
   coefficients; j and j^2 exact), truncation < 2^-59, then the angle-addition formula sin = sa cos r + ca sin r,
   cos = ca cos r - sa sin r, one fma each.  Within 2.3e-16 absolute.  The device twin is det_sincos2pi_u32
   (csrc/detmath.hpp). */
static const double orc_bm_sincos1024_tab[1024][2] = {BM_SINCOS1024_TABLE_ROWS};

#define ORC_SIN_J1 0x1.921fb54442d18p-30
#define ORC_SIN_J3 (-0x1.4abbce625be53p-91)
#define ORC_SIN_J5 0x1.466bc6775aae2p-154
#define ORC_COS_J2 (-0x1.3bd3cc9be45dep-60)
#define ORC_COS_J4 0x1.03c1f081b5ac4p-122

static inline void orc_sincos2pi_u32(uint32_t w, double* s_out, double* c_out) {
    uint32_t k = (w + 0x200000u) >> 22;
    double j = (double)((int32_t)(w << 10) >> 10);        /* signed low 22 bits: w - 2^22 k */
    double j2 = j * j;
    double sr = j * fma(j2, fma(j2, ORC_SIN_J5, ORC_SIN_J3), ORC_SIN_J1);
    double cr = fma(j2, fma(j2, ORC_COS_J4, ORC_COS_J2), 1.0);
    double sa = orc_bm_sincos1024_tab[k][0], ca = orc_bm_sincos1024_tab[k][1];
    *s_out = fma(sa, cr, ca * sr);
    *c_out = fma(ca, cr, -(sa * sr));
}

/* ------------------------------------------------------- Box-Muller radius */
/* sqrt(-2 log((w + 0.5) 2^-32)) as a table of polynomials (scripts/gen_bm_log_table.py, BM_RADP / BM_RADT): side =
   w >> 31 folds u >= 1/2 onto 1 - u = (~w + 0.5) 2^-32 (the same radius law, exact), so x = v + 0.5 in [1/2, 2^31).
   v >= 2^21: the binade e (21..30) and top 5 mantissa bits k of v (x's are the same) pick row side * 320 +
   (e - 21) * 32 + k of the main table, whose polynomials are in the exact residual t = m - (1 + (2k+1)/64) of v's
   mantissa m (the 1/2 of x is inside them); v < 2^21: row side * 704 + (e + 1) * 32 + k of the tail table, binades
   e = -1..20 of x itself, t from x's mantissa.  Degree 7 by Horner, all coefficients doubles.  Device twin:
   bm_radius_u32 (csrc/detmath.hpp); the same operations in the same order, so the two agree bit for bit. */
static const double orc_bm_radp_tab[4 * BM_RADP_NROWS][2] = {BM_RADP_TABLE_ROWS};
static const double orc_bm_radt_tab[4 * BM_RADT_NROWS][2] = {BM_RADT_TABLE_ROWS};

static inline double orc_bm_radius_u32(uint32_t w) {
    uint32_t side = w >> 31;
    uint32_t v = w ^ (0u - side);
    const double (*d)[2];
    int row, n;
    double y;                                              /* v (main table) or x = v + 0.5 (tail) */
    if (v < (1u << 21)) {
        y = (double)v + 0.5;
        row = (int)(orc_d2bits(y) >> 47) - ((1023 - 1) << 5) + (int)side * (BM_RADT_NROWS / 2);
        d = orc_bm_radt_tab; n = BM_RADT_NROWS;
    } else {
        y = (double)v;
        row = (int)(orc_d2bits(y) >> 47) - ((1023 + 21) << 5) + (int)side * (BM_RADP_NROWS / 2);
        d = orc_bm_radp_tab; n = BM_RADP_NROWS;
    }
    uint64_t b = orc_d2bits(y);
    uint32_t yh = (uint32_t)(b >> 32);
    double t = orc_bits2d(((uint64_t)((yh & 0x7fffu) | 0x3ff00000u) << 32) | (b & 0xffffffffull)) -
               (1.0 + 1.0 / 64.0);
    double q = fma(d[3 * n + row][1], t, d[3 * n + row][0]);  /* a7 t + a6 */
    q = fma(q, t, d[2 * n + row][1]);
    q = fma(q, t, d[2 * n + row][0]);
    q = fma(q, t, d[n + row][1]);
    q = fma(q, t, d[n + row][0]);
    q = fma(q, t, d[row][1]);
    return fma(q, t, d[row][0]);
}

/* Four standard normals from one Philox block (two Box-Muller pairs). */
static inline void orc_normals4(const uint32_t w[4], double z[4]) {
    for (int p = 0; p < 2; ++p) {
        double rad = orc_bm_radius_u32(w[2 * p]);
        double s, c;
        orc_sincos2pi_u32(w[2 * p + 1], &s, &c);
        z[2 * p] = rad * c;
        z[2 * p + 1] = rad * s;
    }
}

/* Julia-0.2 round(): nearest, ties away from zero (HMCDA.jl:104). */
static inline double orc_round_away(double x) {
    double t = trunc(x);
    double fr = x - t;                                     /* exact */
    if (fr >= 0.5) t += 1.0;
    else if (fr <= -0.5) t -= 1.0;
    return t;
}

/* ------------------------------------------------------- erfc, erfcx and the normal log-cdf (probit model) */
/* erfcx(x) = exp(x^2) erfc(x) for x >= 1/2 (scripts/gen_erfc_table.py): x < 128: P_i(t) on the binade quarter i
   (i = (biased exponent, top two mantissa bits) - (1022 << 2), t = (x - c) 2^(3-e) exact); x >= 128: the asymptotic
   series 1/(x sqrt(pi)) (1 - 1/(2x^2) + 3/(4x^4) - 15/(8x^6)).
   erfc(x): |x| < 1/2: 1 - x Q(x^2) (Taylor); |x| < 32: exp(-x^2) erfcx(|x|), exp(-x^2) = exp(-xh^2) exp(-(x - xh)
   (x + xh)) with xh = x to 26 bits (xh^2 exact); beyond: 0; negative x: 2 - erfc(-x).  Device twins: det_erfcx,
   det_erfc (detmath.hpp), operation for operation. */
static const double orc_erfc_taylor[14] = {ERFC_TAYLOR_COEFS};
static const double orc_erfc_poly[32][13] = {ERFC_POLY_ROWS};
static inline double orc_erfcx_ge_half(double x) {
    if (x >= 128.0) {
        const double v = 1.0 / (x * x);
        const double s = fma(fma(fma(v, -1.875, 0.75), v, -0.5), v, 1.0);
        return s / (x * 0x1.c5bf891b4ef6bp+0);                     /* x sqrt(pi) */
    }
    const uint64_t bx = orc_d2bits(x);
    const uint32_t hx = (uint32_t)(bx >> 32);
    const int i = (int)(hx >> 18) - (1022 << 2);                   /* binade quarter, 0..31 */
    const double c = orc_bits2d((uint64_t)((hx & 0xfffc0000u) | 0x00020000u) << 32);
    const double sc = orc_bits2d((uint64_t)(2046u - (hx >> 20) + 3u) << 52);   /* 2^(3-e) */
    const double t = (x - c) * sc;                                 /* exact, in [-1, 1] */
    const double* P = orc_erfc_poly[i];
    double p = P[12];
    for (int n = 11; n >= 0; --n) p = fma(p, t, P[n]);
    return p;
}
static inline double orc_erfc(double a) {
    if (a != a) return a;
    const double x = fabs(a);
    double r;
    if (x < 0.5) {
        const double u = x * x;
        double q = orc_erfc_taylor[13];
        for (int n = 12; n >= 0; --n) q = fma(q, u, orc_erfc_taylor[n]);
        r = 1.0 - x * q;
    } else if (x < 32.0) {
        const double p = orc_erfcx_ge_half(x);
        const double xh = orc_bits2d(orc_d2bits(x) & 0xfffffffff8000000ull);   /* 26 significant bits */
        const double e1 = orc_exp(-(xh * xh));
        const double e2 = orc_exp(-((x - xh) * (x + xh)));
        r = (e1 * e2) * p;
    } else {
        r = 0.0;
    }
    return a < 0.0 ? 2.0 - r : r;
}

/* log1p(t) for t > -1: u = 1 + t; t when u == 1, else log(u) t / (u - 1) (Goldberg, What Every Computer Scientist
   ..., theorem 4: a few ulp with a faithful log) */
static inline double orc_log1p(double t) {
    const double u = 1.0 + t;
    if (u == 1.0) return t;
    return orc_log(u) * (t / (u - 1.0));
}

/* logcdf(Normal(), z) in StatsFuns.jl's form (normlogcdf; Distributions.jl, an unpinned REQUIRE dependency of the
   reference, absent here): z < -1: log(erfcx(-z/sqrt2)/2) - z^2/2 (finite down to -Inf: no erfc underflow);
   else log1p(-erfc(z/sqrt2)/2); 1/sqrt2 as a multiplication */
static inline double orc_normlogcdf(double z) {
    const double invsqrt2 = 0x1.6a09e667f3bcdp-1;
    if (z != z) return z;
    if (z < -1.0) return orc_log(orc_erfcx_ge_half(-z * invsqrt2) / 2.0) - (z * z) / 2.0;
    return orc_log1p(-orc_erfc(z * invsqrt2) / 2.0);
}

#endif
