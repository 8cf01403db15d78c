/*
 * oracle/oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of MCMC.jl's
 * model x sampler x SerialMC hot path, used by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg as the checker.  Never linked into, loaded by
 * or called from the product (mcmc.jl_amd/).
 *
 * Parity status: the reference is Julia 0.2 and cannot run here (no Julia, an
 * un-vendored ReverseDiffSource include at src/dsl/modelparser.jl:13); it holds
 * no golden vectors.  This restatement is pinned by
 *   - the Random123 Philox4x32-10 known-answer vectors (tests/golden/philox_kat.json),
 *   - the reference's distributional test restated (KS statistic, test/test_dists.jl:7-47),
 *   - the reference's finite-difference gradient test restated (test/dsl/helper_diff.jl:8-37),
 *   - the README's HMC statistics (README.md:110-154),
 * and is otherwise "parity unpinned" at the bit level against Julia.
 *
 * Each function names the reference lines it follows.  Arithmetic order is the
 * build's specification: sums left to right over coordinates
 * (order 0, lane-per-chain kernels) or per-lane partials + xor butterfly over 64
 * lanes (order 1, wave-per-chain kernels); order W > 1: a chain spread over W waves (lane l of 64 W owns
 * 4 (l + 64 W k) + e), each wave's butterfly, then the W wave sums left to right (block-per-chain kernels);
 * order ORC_ORDER_PAIR (-2): two lanes per chain (16 < d <= 32), each half left to right, then the halves added;
 * order ORC_ORDER_HALF (-3): two chains per wave, 32 lanes per chain (RAM steps on separable targets, 32 < d <= 256;
 * their chains' initial log-targets come from the wave-per-chain eval kernel, order 1: orc_eval_order).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "detmath.h"

#define ORC_MODEL_ISO 1
#define ORC_MODEL_NORMAL 2
#define ORC_MODEL_LOGISTIC 3
#define ORC_MODEL_LINEAR 4
#define ORC_MODEL_ABS_NORMAL 5
#define ORC_MODEL_DIST 6
#define ORC_MODEL_PROBIT 7
#define ORC_MODEL_DIST_OBS 8
#define ORC_MODEL_OU 9

#define ORC_RWM 1
#define ORC_MALA 2
#define ORC_HMC 3
#define ORC_HMCDA 4
#define ORC_RAM 5

typedef struct {
    int32_t kind;
    int32_t d;
    double mu, sigma;
    double prior_sigma, noise_sigma, link_sign;
    int64_t n;
    const double* X;      /* [n][d] */
    const double* Y;      /* [n]    */
    const double* scale;  /* [d] model.scale */
    int32_t dist;         /* ORC_MODEL_DIST: distribution (MCMC_DIST_* of include/mcmc_hip.h) */
} orc_model;

typedef struct {
    int32_t kind;
    int32_t tuner;
    double scale;
    double drift_step;
    int64_t n_leaps;
    double leap_step;
    double rate, len, shrinkage, t0, step;
    int64_t adapt_step, max_step;
    double target_path, target_rate;
    int64_t max_leaps;
} orc_sampler;

/* per-chain state, arrays of length nchains (x: [d][nchains]) */
typedef struct {
    double* x;
    double* lp;
    double* t_step;
    double* t_bar;
    double* t_h;
    int32_t* t_leaps;
    int32_t* t_acc;
    int32_t* t_prop;
    int64_t* n_evals;   /* log-target evaluations per chain (steps for RWM/MALA, leapfrogs for HMC) */
    double* ram_L;      /* RAM jump factor S: packed lower rows, element (r, c) at [r(r+1)/2 + c][nchains] */
} orc_state;

static const double ORC_LOG2PI = 0x1.d67f1c864beb5p+0;
static const double ORC_TWOPI = 0x1.921fb54442d18p+2;

/* ------------------------------------------------------------ reductions */
#define ORC_ORDER_PAIR (-2)
/* order 1: lane l of a 64-lane wave owns coordinates 4*(l + 64k) + e, e = 0..3, k = 0,1,...;
   each lane accumulates its coordinates in (k, e) order, then xor butterfly 32,16,...,1.
   order W > 1: lane l of 64 W owns 4*(l + 64 W k) + e; butterfly per wave, wave sums left to right. */
/* order ORC_ORDER_HALF (RAM on separable targets, 32 < d <= 256; samplers.hpp HalfWaveChain): two chains per wave,
   lane l of a chain's 32 owns 4*(l + 32k) + e; per lane in (k, e) order, then xor butterfly 16,...,1. */
#define ORC_ORDER_HALF (-3)
static double orc_butterfly_n(double* p, int nl) {
    for (int off = nl / 2; off >= 1; off >>= 1) {
        double q[64];
        for (int l = 0; l < nl; ++l) q[l] = p[l] + p[l ^ off];
        memcpy(p, q, sizeof(double) * (size_t)nl);
    }
    return p[0];
}
static double orc_butterfly(double p[64]) { return orc_butterfly_n(p, 64); }
/* the eval kernel's order for a run's order (the initial log-target of SamplerTask / SeqMC particles) */
static int orc_eval_order(int order) { return order == ORC_ORDER_HALF ? 1 : order; }

typedef struct { int d_pad, nw, ds; int64_t n_pad; } orc_glm_geo;
static orc_glm_geo orc_glm_geometry(const orc_model* m);
static double orc_glm_sum(const double* t, const orc_glm_geo* g, int d, int fused_sq);

static int orc_is_glm(const orc_model* m) {
    return m->kind == ORC_MODEL_LOGISTIC || m->kind == ORC_MODEL_LINEAR || m->kind == ORC_MODEL_PROBIT;
}

/* order ORC_ORDER_PAIR (16 < d <= 32, two lanes per chain, samplers.hpp PairChain): the first S = 4 ceil(ceil(d/4)/2)
   coordinates left to right, the rest left to right, then (first) + (second) */
static int orc_pair_split(int d) { return 4 * (((d + 3) / 4 + 1) / 2); }

static double orc_dot_lanes(const double* v, int d, int order);

static double orc_dot(const double* v, const orc_model* mdl, int order) {
    const int d = mdl->d;
    if (orc_is_glm(mdl)) {
        orc_glm_geo geo = orc_glm_geometry(mdl);
        return orc_glm_sum(v, &geo, d, 1);
    }
    return orc_dot_lanes(v, d, order);
}

/* v . v in a kernel family's order: 0 left to right, ORC_ORDER_PAIR, ORC_ORDER_HALF, or W = order
   waves of 64 lanes (lane partials, then the butterfly, waves left to right) */
static double orc_dot_lanes(const double* v, int d, int order) {
    if (order == ORC_ORDER_PAIR) {
        const int S = orc_pair_split(d);
        double a = 0.0, b = 0.0;
        for (int j = 0; j < d && j < S; ++j) a = fma(v[j], v[j], a);
        for (int j = S; j < d; ++j) b = fma(v[j], v[j], b);
        return a + b;
    }
    if (order == 0) {
        double a = 0.0;
        for (int j = 0; j < d; ++j) a = fma(v[j], v[j], a);
        return a;
    }
    const int half = order == ORC_ORDER_HALF;
    const int W = half ? 1 : order, NL = half ? 32 : 64, L = NL * W;   /* W waves per chain, lane l owns 4 (l + L k) + e */
    double tot = 0.0;
    for (int w = 0; w < W; ++w) {
        double p[64];
        for (int l = 0; l < NL; ++l) {
            double a = 0.0;
            for (int j0 = 4 * (NL * w + l); j0 < d; j0 += 4 * L)
                for (int e = 0; e < 4 && j0 + e < d; ++e) a = fma(v[j0 + e], v[j0 + e], a);
            p[l] = a;
        }
        const double sw = orc_butterfly_n(p, NL);
        tot = w == 0 ? sw : tot + sw;             /* waves left to right */
    }
    return tot;
}

static double orc_sum(const double* t, const orc_model* mdl, int order) {
    const int d = mdl->d;
    if (orc_is_glm(mdl)) {
        orc_glm_geo geo = orc_glm_geometry(mdl);
        return orc_glm_sum(t, &geo, d, 0);
    }
    if (order == ORC_ORDER_PAIR) {
        const int S = orc_pair_split(d);
        double a = 0.0, b = 0.0;
        for (int j = 0; j < d && j < S; ++j) a = a + t[j];
        for (int j = S; j < d; ++j) b = b + t[j];
        return a + b;
    }
    if (order == 0) {
        double a = 0.0;
        for (int j = 0; j < d; ++j) a = a + t[j];
        return a;
    }
    const int half = order == ORC_ORDER_HALF;
    const int W = half ? 1 : order, NL = half ? 32 : 64, L = NL * W;
    double tot = 0.0;
    for (int w = 0; w < W; ++w) {
        double p[64];
        for (int l = 0; l < NL; ++l) {
            double a = 0.0;
            for (int j0 = 4 * (NL * w + l); j0 < d; j0 += 4 * L)
                for (int e = 0; e < 4 && j0 + e < d; ++e) a = a + t[j0 + e];
            p[l] = a;
        }
        const double sw = orc_butterfly_n(p, NL);
        tot = w == 0 ? sw : tot + sw;
    }
    return tot;
}

/* ------------------------------------------------------------ regression models (MFMA kernels) */
/* Geometry of the regression kernels (glm.hip mcmc_glm_shape): d <= 128: one wave per 16-chain tile with
   DS = d_pad = 16 NM (NM a power of two); 128 < d <= 256: NW = 4 d-slices of DS = 64 coordinates (NM = 4),
   d_pad = 256; 256 < d <= 1024: NW = 4 or 8 d-slices of DS = 128 (NM = 8), d_pad = 128 NW; n_pad = round_up(n,16).
   Lane quarter q of the wave for slice s owns coordinates k = s*DS + 16m + 4q + e (m < DS/16, e < 4). */
static orc_glm_geo orc_glm_geometry(const orc_model* m) {
    orc_glm_geo g;
    int nm = 1, nw = 1;
    if (m->d <= 128) {                    /* one slice: glm.hip glm_eval1 */
        while (16 * nm < m->d) nm *= 2;
    } else if (m->d <= 256) {             /* 4 d-slices of 64: glm_eval */
        nm = 4;
        nw = 4;
    } else {                              /* 256 < d <= 1024: 4 or 8 d-slices of 128 (glm_eval) */
        nm = 8;
        nw = 4;
        while (128 * nw < m->d) nw *= 2;
    }
    g.ds = 16 * nm;
    g.nw = nw;
    g.d_pad = g.ds * nw;
    g.n_pad = (m->n + 15) / 16 * 16;
    return g;
}

/* sum of per-coordinate terms t[k] (k < d_pad, zero beyond d) in the regression kernels' order:
   lane partials in (m, e) order, quarter combine (p0+p2)+(p1+p3), slices combined left to right */
static double orc_glm_sum(const double* t, const orc_glm_geo* g, int d, int fused_sq) {
    double total = 0.0;
    for (int s = 0; s < g->nw; ++s) {
        double p[4];
        for (int q = 0; q < 4; ++q) {
            double a = 0.0;
            for (int mm = 0; mm < g->ds / 16; ++mm)
                for (int e = 0; e < 4; ++e) {
                    int k = s * g->ds + 16 * mm + 4 * q + e;
                    if (k < d) a = fused_sq ? fma(t[k], t[k], a) : a + t[k];
                }
            p[q] = a;
        }
        double w = (p[0] + p[2]) + (p[1] + p[3]);
        total = s == 0 ? w : total + w;
    }
    return total;
}

/* lp and gradient of the logistic / linear models (examples/logistic_regression.jl:16-22,
   examples/linear_regression.jl:14-20) with the DSL semantics (LLAcc: a non-finite running sum
   after either `~` statement gives (-Inf, zeros); modelparser.jl:64-72).  x: [d]. */
static double orc_glm_eval(const orc_model* m, const double* x, double* g, double* tmp) {
    const int d = m->d;
    const orc_glm_geo geo = orc_glm_geometry(m);
    const int dp = geo.d_pad;
    double* xp = tmp;                 /* [d_pad] */
    double* G = tmp + dp;             /* [d_pad] */
    double* t = tmp + 2 * dp;         /* [d_pad] */
    for (int k = 0; k < dp; ++k) { xp[k] = k < d ? x[k] : 0.0; G[k] = 0.0; }
    const double sp = m->prior_sigma, s2p = sp * sp, logsp = orc_log(sp);
    const double sn = m->noise_sigma, s2n = sn * sn, logsn = orc_log(sn);
    const double isn = 1.0 / sn, is2n = 1.0 / s2n;
    const double sgn = m->link_sign;
    /* likelihood: obs i = 16t + q + 4r belongs to slice wave s = r / RPW (RPW = 4/NW rows per wave, 1 for
       NW >= 4; with NW = 8 slices 4..7 own none); lane (chain, q) of that wave accumulates its obs in (t, r)
       order */
    const int rpw = geo.nw >= 4 ? 1 : 4 / geo.nw;
    double lik_part[8][4];
    int logi_oos = 0;
    for (int s = 0; s < 8; ++s)
        for (int q = 0; q < 4; ++q) lik_part[s][q] = 0.0;
    for (int64_t i = 0; i < geo.n_pad; ++i) {
        const double* Xi = (i < m->n) ? m->X + (size_t)i * d : NULL;
        /* eta_i: per slice an fma chain over (mm, e, q), slices added left to right */
        double eta = 0.0;
        for (int s = 0; s < geo.nw; ++s) {
            double a = 0.0;
            for (int mm = 0; mm < geo.ds / 16; ++mm)
                for (int e = 0; e < 4; ++e)
                    for (int q = 0; q < 4; ++q) {
                        int k = s * geo.ds + 16 * mm + 4 * q + e;
                        double xik = (Xi && k < d) ? Xi[k] : 0.0;
                        a = fma(xik, xp[k], a);
                    }
            eta = s == 0 ? a : eta + a;
        }
        double term = 0.0, r = 0.0;
        if (i < m->n) {
            const double y = m->Y[i];
            if (m->kind == ORC_MODEL_LINEAR) {
                double resid = y - eta;                           /* resid = Y - X*vars */
                double z = resid * isn;
                term = -0.5 * (z * z + ORC_LOG2PI) - logsn;       /* resid ~ Normal(0, sn) */
                r = resid * is2n;                                 /* -d/dresid, MCMCDerivRules.jl:57 */
            } else if (m->kind == ORC_MODEL_PROBIT) {
                /* examples/probit_regression.jl:26-40: dot(logcdf(N, X pars), y) + dot(logcdf(N, -X pars), 1 - y),
                   per observation here; d/deta = y exp(A - logcdf(eta)) - (1 - y) exp(A - logcdf(-eta)),
                   A = -(eta^2 + log(2 pi))/2 (the example's grad_log_posterior) */
                const double la = orc_normlogcdf(eta), lb = orc_normlogcdf(-eta);
                term = y * la + (1.0 - y) * lb;
                const double A = (-(eta * eta + ORC_LOG2PI)) / 2.0;
                r = y * orc_exp(A - la) - (1.0 - y) * orc_exp(A - lb);
            } else {
                /* prob = 1/(1+exp(-s X*vars)), Y ~ Bernoulli(prob): term = log(prob) or log(1 - prob), and d/deta
                   of it, the rule dd1 += 1/(p - 1 + y) (MCMCDerivRules.jl:111) times dprob/deta = s t/(1+t)^2, which
                   is s (y - p) for y in {0, 1}; both as functions of u = -w eta, w = s (2y - 1) (orc_logi) */
                const double w = (y >= 0.5) ? sgn : -sgn;
                orc_logi(eta, w, &term, &r);
                /* -Inf where the reference's p rounds to 1 (y = 0) or 0 (y = 1): u = -w eta >= T(y) (glm_layout.hpp
                   logi_bound: RU(53 ln 2); the first double past fdlibm exp's overflow threshold) */
                if (-(w * eta) + ((y >= 0.5) ? -0x1.62e42fefa39f0p+9 : -0x1.25e4f7b2737fbp+5) >= 0.0) logi_oos = 1;
            }
            const int q = (int)(i & 3), rr = (int)((i & 15) >> 2);
            double* lp_ = lik_part[rr / rpw];
            lp_[q] = lp_[q] + term;
        }
        /* G_k = sum_i X[i][k] r_i, fma chain over obs (padded obs: X = 0, r = 0) */
        for (int k = 0; k < dp; ++k) {
            double xik = (Xi && k < d) ? Xi[k] : 0.0;
            G[k] = fma(xik, r, G[k]);
        }
    }
    double lik = 0.0;
    for (int s = 0; s < geo.nw; ++s) {
        const double w = (lik_part[s][0] + lik_part[s][2]) + (lik_part[s][1] + lik_part[s][3]);
        lik = s == 0 ? w : lik + w;
    }
    if (logi_oos) lik = -INFINITY;
    for (int k = 0; k < dp; ++k) {
        double z = (xp[k] - 0.0) / sp;
        t[k] = -0.5 * (z * z + ORC_LOG2PI) - logsp;                /* vars ~ Normal(0, sp) */
    }
    const double prior = orc_glm_sum(t, &geo, d, 0);
    double a = 0.0 + prior;
    int oos = !isfinite(a);
    a = a + lik;
    oos = oos || !isfinite(a);
    if (oos) a = -INFINITY;
    if (g)
        for (int k = 0; k < d; ++k) g[k] = oos ? 0.0 : (0.0 - xp[k]) / s2p + G[k];
    return a;
}

/* ------------------------------------------------------------ models */
/* Returns lp; writes the gradient into g (length d) when g != NULL; tmp: scratch (see orc_scratch). */
/* v ~ Dist(p1, p2) elementwise (MCMCDerivRules.jl:56-104; Distributions.jl parametrisations).  The
   parameter-only constant is computed as the runtime does (glibc log / lgamma), the rest as
   csrc/models.hpp DistDSL. */
static double orc_dist_const(int dist, double p1, double p2) {
    const double kPi = 3.14159265358979323846;
    switch (dist) {
        case 1: return -log(p2);
        case 2: return -log(p2 - p1);
        case 3: return log(p1 / p2);
        case 4: return lgamma(p1 + p2) - lgamma(p1) - lgamma(p2);
        case 5: return lgamma((p1 + 1.0) / 2.0) - lgamma(p1 / 2.0) - 0.5 * log(p1 * kPi);
        case 6: return -log(p1);
        case 7: return -lgamma(p1) - p1 * log(p2);
        case 8: return -log(kPi * p2);
        case 9: return -log(p2) - 0.5 * log(2.0 * kPi);
        case 10: return -log(2.0 * p2);
        default: return NAN;
    }
}

static double orc_dist_logpdf(int dist, double p1, double p2, double c, double v) {
    switch (dist) {
        case 1: { double z = (v - p1) / p2; return -0.5 * (z * z + ORC_LOG2PI) + c; }
        case 2: return (v >= p1 && v <= p2) ? c : -INFINITY;
        case 3: {
            if (v < 0.0) return -INFINITY;
            double lr = orc_log(v / p2);
            return c + (p1 - 1.0) * lr - orc_exp(p1 * lr);
        }
        case 4:
            if (v < 0.0 || v > 1.0) return -INFINITY;
            return (p1 - 1.0) * orc_log(v) + (p2 - 1.0) * orc_log(1.0 - v) + c;
        case 5: return c - ((p1 + 1.0) / 2.0) * orc_log(1.0 + (v * v) / p1);
        case 6: return v < 0.0 ? -INFINITY : c - v / p1;
        case 7: return v < 0.0 ? -INFINITY : (p1 - 1.0) * orc_log(v) - v / p2 + c;
        case 8: { double z = (v - p1) / p2; return c - orc_log(1.0 + z * z); }
        case 9: {
            if (v <= 0.0) return -INFINITY;
            double lv = orc_log(v), e = lv - p1;
            return -(e * e) / (2.0 * p2 * p2) - lv + c;
        }
        case 10: return c - fabs(v - p1) / p2;
        default: return NAN;
    }
}

static double orc_dist_grad(int dist, double p1, double p2, double v) {
    switch (dist) {
        case 1: return (p1 - v) / (p2 * p2);
        case 2: return 0.0;
        case 3: return ((1.0 - orc_exp(p1 * orc_log(v / p2))) * p1 - 1.0) / v;
        case 4: return (p1 - 1.0) / v - (p2 - 1.0) / (1.0 - v);
        case 5: return -(p1 + 1.0) * v / (p1 + v * v);
        case 6: return -1.0 / p1;
        case 7: return -(p2 + v - p1 * p2) / (p2 * v);
        case 8: { double e = v - p1; return 2.0 * (p1 - v) / (p2 * p2 + e * e); }
        case 9: return (p1 - p2 * p2 - orc_log(v)) / (p2 * p2 * v);
        case 10: return (v > p1 ? -1.0 : 1.0) / p2;
        default: return 0.0;
    }
}

static double orc_eval(const orc_model* m, const double* x, double* g, double* tmp, int order) {
    const int d = m->d;
    if (m->kind == ORC_MODEL_OU) {
        /* examples/ornstein.jl:19-30 (models.hpp OUDSL): pars (tau, sigma, mu), series Y[0..n-1].  LLAcc(0.) +
           logpdf(Uniform(0,100), tau) + logpdf(Uniform(0,2), sigma) + logpdf(Uniform(0,20), mu) (-log(b - a) inside,
           -Inf outside: OutOfSupportError), then + sum(logpdf(Normal(0, sigma), resid)) left to right with
           resid_i = (Y[i] - Y[i-1] fac) - mu (1 - fac), fac = exp(-1/tau).  Gradient by reverse mode with the DSL's
           rules (MCMCDerivRules.jl:57-59 Normal dx / dsigma, :62 Uniform dx = 0): dr = (0 - r)/(sigma sigma),
           d tau = (mu G0 - G1)(fac/(tau tau)), d sigma = sum ((r r)/(sigma sigma) - 1)/sigma, d mu = -(G0 (1 - fac)). */
        const double tau = x[0], sigma = x[1], mu = x[2];
        const int insup = tau >= 0.0 && tau <= 100.0 && sigma >= 0.0 && sigma <= 2.0 && mu >= 0.0 && mu <= 20.0;
        double lp = -INFINITY;
        int oos = 1;
        if (insup) {
            const double c0 = ((0.0 + -log(100.0)) + -log(2.0)) + -log(20.0);   /* host glibc, as the runtime */
            const double fac = orc_exp(-1.0 / tau);
            const double c = mu * (1.0 - fac);
            const double logsig = orc_log(sigma);
            double s = 0.0;
            for (int64_t i = 1; i < m->n; ++i) {
                const double z = ((m->Y[i] - m->Y[i - 1] * fac) - c) / sigma;
                s = s + (-0.5 * (z * z + ORC_LOG2PI) - logsig);
            }
            lp = c0 + s;
            oos = !isfinite(lp);
            if (oos) lp = -INFINITY;
        }
        if (g) {
            g[0] = g[1] = g[2] = 0.0;
            if (!oos) {
                const double fac = orc_exp(-1.0 / tau);
                const double c = mu * (1.0 - fac);
                const double s2 = sigma * sigma;
                double g0 = 0.0, g1 = 0.0, gs = 0.0;
                for (int64_t i = 1; i < m->n; ++i) {
                    const double r = (m->Y[i] - m->Y[i - 1] * fac) - c;
                    const double dr = (0.0 - r) / s2;
                    g0 = g0 + dr;
                    g1 = g1 + dr * m->Y[i - 1];
                    gs = gs + ((r * r) / s2 - 1.0) / sigma;
                }
                g[0] = (mu * g0 - g1) * (fac / (tau * tau));
                g[1] = gs;
                g[2] = -(g0 * (1.0 - fac));
            }
        }
        return lp;
    }
    if (m->kind == ORC_MODEL_DIST_OBS) {
        /* benchmarks/benchunits/bare_distribs.jl:13: y = x * v; y ~ Dist(p1, p2), scalar x, data v = Y [n]: the LLAcc
           sum left to right, d/dx = sum_i v_i dlogpdf(x v_i) (left to right) */
        const double c = orc_dist_const(m->dist, m->mu, m->sigma);
        double lp = 0.0, gx = 0.0;
        for (int64_t i = 0; i < m->n; ++i) lp = lp + orc_dist_logpdf(m->dist, m->mu, m->sigma, c, x[0] * m->Y[i]);
        int oos = !isfinite(lp);
        if (oos) lp = -INFINITY;
        if (g) {
            for (int64_t i = 0; i < m->n; ++i) gx = gx + m->Y[i] * orc_dist_grad(m->dist, m->mu, m->sigma, x[0] * m->Y[i]);
            g[0] = oos ? 0.0 : gx;
        }
        return lp;
    }
    if (m->kind == ORC_MODEL_DIST) {
        const double c = orc_dist_const(m->dist, m->mu, m->sigma);
        for (int j = 0; j < d; ++j) tmp[j] = orc_dist_logpdf(m->dist, m->mu, m->sigma, c, x[j]);
        double lp = orc_sum(tmp, m, order);
        int oos = !isfinite(lp);
        if (oos) lp = -INFINITY;                  /* LLAcc: (-Inf, zero(beta)), modelparser.jl:64-72 */
        if (g)
            for (int j = 0; j < d; ++j) g[j] = oos ? 0.0 : orc_dist_grad(m->dist, m->mu, m->sigma, x[j]);
        return lp;
    }
    if (orc_is_glm(m)) return orc_glm_eval(m, x, g, tmp);
    if (m->kind == ORC_MODEL_ISO) {
        /* model(v -> -dot(v,v), grad = v -> -2v)  README.md:60,63; test/test_syntax.jl:40-41 */
        double lp = -orc_dot(x, m, order);
        if (g)
            for (int j = 0; j < d; ++j) g[j] = -2.0 * x[j];
        return lp;
    }
    if (m->kind == ORC_MODEL_NORMAL || m->kind == ORC_MODEL_ABS_NORMAL) {
        /* v ~ Normal(mu, sigma): LLAcc(0.) + sum(logpdf(...)) (AccumulatorDerivRules.jl:10-20,
           modelparser.jl:48-51); gradient rule dx += (mu - x)/(sigma*sigma)*ds (MCMCDerivRules.jl:57).
           ABS_NORMAL: y = abs(x); y ~ Normal(mu, sigma) (README.md:246-251), gradient times sign(x). */
        const int ab = m->kind == ORC_MODEL_ABS_NORMAL;
        const double logsig = orc_log(m->sigma);
        for (int j = 0; j < d; ++j) {
            double z = ((ab ? fabs(x[j]) : x[j]) - m->mu) / m->sigma;
            tmp[j] = -0.5 * (z * z + ORC_LOG2PI) - logsig;
        }
        double lp = orc_sum(tmp, m, order);
        int oos = !isfinite(lp);
        if (oos) lp = -INFINITY;                  /* OutOfSupportError -> (-Inf, zero(beta)), modelparser.jl:64-72 */
        if (g) {
            const double s2 = m->sigma * m->sigma;
            for (int j = 0; j < d; ++j) {
                if (ab) {
                    const double sg = x[j] > 0.0 ? 1.0 : (x[j] < 0.0 ? -1.0 : 0.0);
                    g[j] = oos ? 0.0 : sg * ((m->mu - fabs(x[j])) / s2);
                } else {
                    g[j] = oos ? 0.0 : (m->mu - x[j]) / s2;
                }
            }
        }
        return lp;
    }
    return NAN;
}

/* normals of step `step` for chain `chain`: coordinate j <- block j/4, slot j%4 */
static void orc_normals(uint64_t seed, uint32_t chain, uint32_t step, int d, double* z) {
    for (int b = 0; 4 * b < d; ++b) {
        uint32_t w[4];
        double zz[4];
        orc_block(seed, chain, step, (uint32_t)b, ORC_TAG_NORMAL, w);
        orc_normals4(w, zz);
        for (int e = 0; e < 4 && 4 * b + e < d; ++e) z[4 * b + e] = zz[e];
    }
}

static double orc_accept_uniform(uint64_t seed, uint32_t chain, uint32_t step) {
    uint32_t w[4];
    orc_block(seed, chain, step, 0u, ORC_TAG_ACCEPT, w);
    return orc_uniform52(w[0], w[1]);
}

/* i in r = (burnin+1):thinning:len ?  (SerialMC.jl:35, :49) */
static int orc_kept(int64_t i_loc, int64_t burnin, int64_t thinning, int64_t len, int64_t* kk) {
    if (i_loc <= burnin || i_loc > len) return 0;
    int64_t off = i_loc - burnin - 1;
    if (off % thinning) return 0;
    *kk = off / thinning;
    return 1;
}

/* adapt!(tune, tuner): rate = accepted/proposed; step *= 1/(1+exp(-11*(rate-target))) + 0.5
   (MALA.jl:36-39, HMC.jl:165-169) */
static double orc_tune_factor(int32_t acc, int32_t prop, double target) {
    double rate = (double)acc / (double)prop;
    return 1.0 / (1.0 + orc_exp(-11.0 * (rate - target))) + 0.5;
}

/* `ratio > 0 || ratio > log(rand())`, uniform drawn only when needed (RWM.jl:63, MALA.jl:108) */
static int orc_mh_short_circuit(uint64_t seed, uint32_t chain, uint32_t step, double ratio) {
    if (ratio > 0.0) return 1;
    return ratio > orc_log(orc_accept_uniform(seed, chain, step));
}

/* nl leapfrogs (HMC.jl:93-102) from (x, mom, g); returns the final lp */
static double orc_trajectory(const orc_model* m, double eps, int64_t nl, double* x, double* mom, double* g,
                             double lp, double* tmp, int order) {
    const int d = m->d;
    for (int64_t l = 0; l < nl; ++l) {
        for (int j = 0; j < d; ++j) mom[j] = mom[j] + (0.5 * g[j]) * eps;   /* n.m += 0.5*n.grad*ve */
        for (int j = 0; j < d; ++j) x[j] = x[j] + eps * mom[j];              /* n.pars += ve * n.m   */
        lp = orc_eval(m, x, g, tmp, order);                                   /* calc!(n, ll)         */
        for (int j = 0; j < d; ++j) mom[j] = mom[j] + (0.5 * g[j]) * eps;   /* n.m += 0.5*n.grad*ve */
    }
    return lp;
}

/* RAM scale tuning (RAM.jl:74-78) on the packed factor Lc (element (r, c) at Lc[(r(r+1)/2 + c) * C]).
   The reference sets S = chol(S (I + a z z'/|z|^2) S')'; restated as the rank-1 Cholesky update
   (a >= 0) / downdate (a < 0) of S with sqrt(|a|/|z|^2) u, u = S z, in the kernels' order
   (mcmc.jl_amd/csrc/ram.hpp ram_update). */
static void orc_ram_update(double* Lc, int64_t C, int d, int64_t i, double ratio, double rate, double nz, double* u) {
    const double eta = fmin(1.0, (double)d * orc_exp((-2.0 / 3.0) * orc_log((double)i)));
    const double alpha = eta * (fmin(1.0, orc_exp(ratio)) - rate);
    const double beta = alpha / nz;
    const int up = beta >= 0.0;
    const double sb = sqrt(fabs(beta));
    for (int k = 0; k < d; ++k) u[k] = sb * u[k];
    for (int k = 0; k < d; ++k) {
        double* Lkk = Lc + (size_t)(k * (k + 1) / 2 + k) * C;
        const double lkk = *Lkk;
        const double xk = u[k];
        const double t2 = xk * xk;
        const double l2 = lkk * lkk;
        const double r = sqrt(up ? l2 + t2 : l2 - t2);
        const double cc = r / lkk;
        const double sn = xk / lkk;
        const double ic = 1.0 / cc;
        *Lkk = r;
        for (int q = k + 1; q < d; ++q) {
            double* Lq = Lc + (size_t)(q * (q + 1) / 2 + k) * C;
            const double su = sn * u[q];
            const double l = (up ? *Lq + su : *Lq - su) * ic;
            *Lq = l;
            u[q] = cc * u[q] - sn * l;
        }
    }
}

/* storeLeaps record (HMC.jl:145-150): pars / grads / mom [nkept][cap+1][d][C], lp / H [nkept][cap+1][C],
   nl [nkept][C] */
typedef struct {
    int64_t cap;
    double *pars, *grads, *mom, *lp, *H;
    int32_t* nl;
} orc_leaps;

static void orc_leap_put(const orc_leaps* lv, int64_t kk, int64_t l, int d, int64_t C, int64_t c, const double* x,
                         const double* g, const double* mom, double lp, double H) {
    const size_t base = (size_t)kk * (size_t)(lv->cap + 1) + (size_t)l;
    for (int j = 0; j < d; ++j) {
        lv->pars[(base * d + j) * C + c] = x[j];
        lv->grads[(base * d + j) * C + c] = g[j];
        lv->mom[(base * d + j) * C + c] = mom[j];
    }
    lv->lp[base * C + c] = lp;
    lv->H[base * C + c] = H;
}

/* ------------------------------------------------------------ one chain */
/* `len` steps of SerialMC (SerialMC.jl:47-67) for chain c, sampler loop counter continuing from step0. */
static void orc_chain(const orc_model* m, const orc_sampler* s, uint64_t seed, uint32_t chain, int64_t c,
                      int64_t C, int64_t step0, int64_t burnin, int64_t thinning, int64_t len, orc_state* st,
                      double* samples, double* grads, uint8_t* acc_out, int order, double* buf,
                      const orc_leaps* lv) {
    const int d = m->d;
    double* x = buf;          /* state: pars */
    double* g = x + d;        /* state: grad */
    double* xp = g + d;       /* proposal    */
    double* gp = xp + d;
    double* mom = gp + d;
    double* sc = mom + d;     /* RWM scale = model.scale .* sampler.scale (RWM.jl:52) */
    double* tmp = sc + d;     /* model scratch (orc_scratch) */
    for (int j = 0; j < d; ++j) x[j] = st->x[(size_t)j * C + c];
    for (int j = 0; j < d; ++j) sc[j] = m->scale ? m->scale[j] * s->scale : s->scale;
    double lp = st->lp[c];
    (void)orc_eval(m, x, g, tmp, order);     /* state grad (deterministic recompute of the stored one) */

    const int tuned = s->tuner && (s->kind == ORC_MALA || s->kind == ORC_HMC);
    double h = (s->kind == ORC_MALA && tuned) ? st->t_step[c] : s->drift_step;
    double eps = ((s->kind == ORC_HMC && tuned) || s->kind == ORC_HMCDA) ? st->t_step[c] : s->leap_step;
    int64_t nl_fixed = (s->kind == ORC_HMC && tuned) ? (int64_t)st->t_leaps[c] : s->n_leaps;
    double eps_bar = s->kind == ORC_HMCDA ? st->t_bar[c] : 0.0;
    double h_bar = s->kind == ORC_HMCDA ? st->t_h[c] : 0.0;
    int32_t n_acc = tuned ? st->t_acc[c] : 0;
    int32_t n_prop = tuned ? st->t_prop[c] : 0;
    int64_t n_evals = 0;
    const double mu = orc_log(10.0);          /* HMCDA.jl:92: mu = log(10*leapStep) with leapStep = 1 */
    const int64_t max_leaps = s->max_leaps > 0 ? s->max_leaps : ((int64_t)1 << 20);

    for (int64_t t = 0; t < len; ++t) {
        const int64_t i = step0 + t + 1;      /* the sampler's loop counter (HMC.jl:126 `for i in 1:Inf`) */
        int acc = 0;
        double ram_ratio = 0.0, ram_nz = 0.0;
        double p_da = 0.0;
        if (s->kind == ORC_RWM) {
            /* RWM.jl:58-71 */
            orc_normals(seed, chain, (uint32_t)i, d, mom);
            for (int j = 0; j < d; ++j) xp[j] = x[j] + mom[j] * sc[j];        /* pars + randn(d) .* scale */
            double lpp = orc_eval(m, xp, NULL, tmp, order);
            double ratio = lpp - lp;
            acc = orc_mh_short_circuit(seed, chain, (uint32_t)i, ratio);
            if (acc) {
                memcpy(x, xp, sizeof(double) * d);
                lp = lpp;
            }
        } else if (s->kind == ORC_RAM) {
            /* RAM.jl:58-78 */
            double* Lc = st->ram_L + c;
            orc_normals(seed, chain, (uint32_t)i, d, mom);                    /* rvec = randn(d) */
            double nz = 0.0;                                                  /* dot(rvec, rvec): in order, */
            if (orc_is_glm(m) && d > 32)                                      /* or in the lane order of the */
                nz = orc_dot_lanes(mom, d, d <= 256 ? ORC_ORDER_HALF : 1);    /* wave-per-chain kernels: the */
            else if (order == 0 || order == ORC_ORDER_PAIR || orc_is_glm(m))  /* regression split step (d > 32, */
                for (int j = 0; j < d; ++j) nz = fma(mom[j], mom[j], nz);     /* glm_ram_wave.hip), separable */
            else                                                              /* targets (d > 32) */
                nz = orc_dot(mom, m, order);
            for (int r = 0; r < d; ++r) {                                     /* S * rvec */
                double a = 0.0;
                for (int q = 0; q <= r; ++q) a = fma(Lc[(size_t)(r * (r + 1) / 2 + q) * C], mom[q], a);
                gp[r] = a;
            }
            for (int j = 0; j < d; ++j) xp[j] = x[j] + gp[j];
            double lpp = orc_eval(m, xp, NULL, tmp, order);
            double ratio = lpp - lp;
            acc = orc_mh_short_circuit(seed, chain, (uint32_t)i, ratio);
            if (acc) {
                memcpy(x, xp, sizeof(double) * d);
                lp = lpp;
            }
            ram_ratio = ratio;
            ram_nz = nz;
        } else if (s->kind == ORC_MALA) {
            /* MALA.jl:89-125 */
            if (tuned) n_prop += 1;
            const double half = h / 2.0;
            const double sq = sqrt(h);
            const double twoh = 2.0 * h;
            const double L = orc_log(ORC_TWOPI * h) / 2.0;                   /* log(2*pi*driftStep)/2 */
            orc_normals(seed, chain, (uint32_t)i, d, mom);
            for (int j = 0; j < d; ++j) {
                double pm = x[j] + half * g[j];                               /* parsMean */
                xp[j] = pm + sq * mom[j];                                     /* proposedPars */
                double e = pm - xp[j];
                tmp[j] = (-(e * e)) / twoh - L;
            }
            double qf = orc_sum(tmp, m, order);                               /* probNewGivenOld */
            double lpp = orc_eval(m, xp, gp, tmp, order);                     /* evalallg(proposedPars) */
            for (int j = 0; j < d; ++j) {
                double e = (xp[j] + half * gp[j]) - x[j];
                tmp[j] = (-(e * e)) / twoh - L;
            }
            double qb = orc_sum(tmp, m, order);                               /* probOldGivenNew */
            double ratio = ((lpp + qb) - lp) - qf;
            acc = orc_mh_short_circuit(seed, chain, (uint32_t)i, ratio);
            if (acc) {
                memcpy(x, xp, sizeof(double) * d);
                memcpy(g, gp, sizeof(double) * d);
                lp = lpp;
                if (tuned) n_acc += 1;
            }
        } else {
            /* HMC.jl:126-173 / HMCDA.jl:97-142 */
            const int da = s->kind == ORC_HMCDA;
            if (!da && tuned) n_prop += 1;
            orc_normals(seed, chain, (uint32_t)i, d, mom);                    /* state0.m = randn(model.size) */
            const double H0 = -lp + 0.5 * orc_dot(mom, m, order);             /* update!(state0) */
            memcpy(xp, x, sizeof(double) * d);
            memcpy(gp, g, sizeof(double) * d);
            int64_t nl;
            if (da) {
                double r = orc_round_away(s->len / eps);                      /* round(len/leapStep) */
                nl = r < 1.0 ? 1 : (r > (double)max_leaps ? max_leaps : (int64_t)r);
            } else {
                nl = nl_fixed;
            }
            n_evals += nl;
            int64_t kk_rec = 0;
            double lpl;
            if (lv && orc_kept(i - step0, burnin, thinning, len, &kk_rec)) {
                /* storeLeaps: leapStates[1] = state0, then the state after every leapfrog (HMC.jl:145-150) */
                orc_leap_put(lv, kk_rec, 0, d, C, c, xp, gp, mom, lp, H0);
                lpl = lp;
                for (int64_t l = 1; l <= nl; ++l) {
                    lpl = orc_trajectory(m, eps, 1, xp, mom, gp, lpl, tmp, order);
                    if (l <= lv->cap) orc_leap_put(lv, kk_rec, l, d, C, c, xp, gp, mom, lpl, -lpl + 0.5 * orc_dot(mom, m, order));
                }
                lv->nl[(size_t)kk_rec * C + c] = (int32_t)nl;
            } else {
                lpl = orc_trajectory(m, eps, nl, xp, mom, gp, lp, tmp, order);
            }
            const double H = -lpl + 0.5 * orc_dot(mom, m, order);
            const double u = orc_accept_uniform(seed, chain, (uint32_t)i);
            if (da) {
                p_da = fmin(1.0, orc_exp(H0 - H));                            /* min(1, exp(H0-H)), NaN-ignoring */
                acc = u < p_da;
            } else {
                acc = u < orc_exp(H0 - H);
            }
            if (acc) {
                memcpy(x, xp, sizeof(double) * d);
                memcpy(g, gp, sizeof(double) * d);
                lp = lpl;
                if (!da && tuned) n_acc += 1;
            }
        }
        int64_t kk;
        if (orc_kept(i - step0, burnin, thinning, len, &kk)) {
            if (samples)
                for (int j = 0; j < d; ++j) samples[((size_t)kk * d + j) * C + c] = x[j];
            if (grads && s->kind != ORC_RWM && s->kind != ORC_RAM)
                for (int j = 0; j < d; ++j) grads[((size_t)kk * d + j) * C + c] = g[j];
            if (acc_out) acc_out[(size_t)kk * C + c] = (uint8_t)acc;
        }
        /* adaptation, with the runner's burnin (`i <= runner.burnin`, MALA.jl:116, HMC.jl:167) */
        if (s->kind == ORC_RAM) {
            orc_ram_update(st->ram_L + c, C, d, i, ram_ratio, s->rate, ram_nz, gp);
        } else if (s->kind == ORC_MALA && tuned && i <= burnin && (i % s->adapt_step) == 0) {
            h = h * orc_tune_factor(n_acc, n_prop, s->target_rate);
            n_acc = 0;
            n_prop = 0;
        } else if (s->kind == ORC_HMC && tuned && i <= burnin && (i % s->adapt_step) == 0) {
            eps = eps * orc_tune_factor(n_acc, n_prop, s->target_rate);
            double nlf = ceil(s->target_path / eps);                         /* min(maxStep, ceil(targetPath/leapStep)) */
            if (nlf > (double)s->max_step) nlf = (double)s->max_step;
            if (nlf > (double)max_leaps) nlf = (double)max_leaps;
            nl_fixed = (int64_t)nlf;
            n_acc = 0;
            n_prop = 0;
        } else if (s->kind == ORC_HMCDA) {
            const double di = (double)i;
            if (di < (double)burnin) {                                        /* HMCDA.jl:133-138 */
                double eta = 1.0 / (di + s->t0);
                h_bar = (1.0 - eta) * h_bar + eta * (s->rate - p_da);
                eps = orc_exp(mu - (sqrt(di) * h_bar) / s->shrinkage);
                eta = orc_exp(orc_log(di) * (-s->step));                      /* i^(-step) */
                eps_bar = orc_exp((1.0 - eta) * orc_log(eps_bar) + eta * orc_log(eps));
            } else {
                eps = eps_bar;                                                /* HMCDA.jl:140 */
            }
        }
    }
    for (int j = 0; j < d; ++j) st->x[(size_t)j * C + c] = x[j];
    st->lp[c] = lp;
    if (st->n_evals) st->n_evals[c] += (s->kind == ORC_RWM || s->kind == ORC_MALA || s->kind == ORC_RAM) ? len : n_evals;
    if (tuned || s->kind == ORC_HMCDA) st->t_step[c] = (s->kind == ORC_MALA) ? h : eps;
    if (s->kind == ORC_HMCDA) {
        st->t_bar[c] = eps_bar;
        st->t_h[c] = h_bar;
    }
    if (tuned) {
        if (s->kind == ORC_HMC) st->t_leaps[c] = (int32_t)nl_fixed;
        st->t_acc[c] = n_acc;
        st->t_prop[c] = n_prop;
    }
}

/* ------------------------------------------------------------ exported API (ctypes) */
static size_t orc_scratch(const orc_model* m) {
    size_t n = (size_t)m->d + 16;
    if (orc_is_glm(m)) n = 3 * (size_t)orc_glm_geometry(m).d_pad + 16;
    return n;
}

/* SamplerTask initialisation: lp = eval(x), tuner state defaults.  Returns the number of
   chains whose start is out of support ("Initial values out of model support", RWM.jl:55). */
int64_t orc_init(const orc_model* m, const orc_sampler* s, int64_t C, orc_state* st, int order) {
    const int d = m->d;
    int64_t bad = 0;
    double* buf = (double*)malloc(sizeof(double) * ((size_t)d + orc_scratch(m)));
    double* x = buf;
    double* tmp = buf + d;
    for (int64_t c = 0; c < C; ++c) {
        for (int j = 0; j < d; ++j) x[j] = st->x[(size_t)j * C + c];
        double lp = orc_eval(m, x, NULL, tmp, orc_eval_order(order));
        st->lp[c] = lp;
        if (!isfinite(lp)) bad++;
        const int tuned = s->tuner && (s->kind == ORC_MALA || s->kind == ORC_HMC);
        if (s->kind == ORC_MALA && tuned) st->t_step[c] = s->drift_step;
        if (s->kind == ORC_HMC && tuned) { st->t_step[c] = s->leap_step; st->t_leaps[c] = (int32_t)s->n_leaps; }
        if (s->kind == ORC_HMCDA) { st->t_step[c] = 1.0; st->t_bar[c] = 1.0; st->t_h[c] = 0.0; }
        if (s->kind == ORC_RAM)                   /* S = diag(model.scale .* sampler.scale) (RAM.jl:51,55) */
            for (int r = 0; r < d; ++r)
                for (int q = 0; q <= r; ++q)
                    st->ram_L[(size_t)(r * (r + 1) / 2 + q) * C + c] =
                        q == r ? (m->scale ? m->scale[r] * s->scale : s->scale) : 0.0;
        if (tuned) { st->t_acc[c] = 0; st->t_prop[c] = 0; }
        if (st->n_evals) st->n_evals[c] = 0;
    }
    free(buf);
    return bad;
}

/* run_serialmc over chains [c_begin, c_end) of a batch of C (SerialMC.jl:37-85).
   samples/grads: [nkept][d][C]; acc_out: [nkept][C] bytes.  nthreads > 1 uses OpenMP. */
static void orc_run_impl(const orc_model* m, const orc_sampler* s, uint64_t seed, int64_t chain0, int64_t C,
                         int64_t c_begin, int64_t c_end, int64_t step0, int64_t burnin, int64_t thinning, int64_t len,
                         orc_state* st, double* samples, double* grads, uint8_t* acc_out, int order, int nthreads,
                         const orc_leaps* lv) {
    const int d = m->d;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
    {
        double* buf = (double*)malloc(sizeof(double) * (6 * (size_t)d + orc_scratch(m)));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t c = c_begin; c < c_end; ++c)
            orc_chain(m, s, seed, (uint32_t)(chain0 + c), c, C, step0, burnin, thinning, len, st, samples, grads,
                      acc_out, order, buf, lv);
        free(buf);
    }
    (void)nthreads;
}

void orc_run(const orc_model* m, const orc_sampler* s, uint64_t seed, int64_t chain0, int64_t C,
             int64_t c_begin, int64_t c_end, int64_t step0, int64_t burnin, int64_t thinning, int64_t len,
             orc_state* st, double* samples, double* grads, uint8_t* acc_out, int order, int nthreads) {
    orc_run_impl(m, s, seed, chain0, C, c_begin, c_end, step0, burnin, thinning, len, st, samples, grads, acc_out,
                 order, nthreads, NULL);
}

/* orc_run with the storeLeaps record of every kept HMC / HMCDA step (buffers as mcmc_chains_store_leaps) */
void orc_run_leaps(const orc_model* m, const orc_sampler* s, uint64_t seed, int64_t chain0, int64_t C,
                   int64_t step0, int64_t burnin, int64_t thinning, int64_t len, orc_state* st, double* samples,
                   double* grads, uint8_t* acc_out, int order, int64_t cap, double* lpars, double* lgrads,
                   double* lmom, double* llp, double* lH, int32_t* lnl) {
    orc_leaps lv = {cap, lpars, lgrads, lmom, llp, lH, lnl};
    orc_run_impl(m, s, seed, chain0, C, 0, C, step0, burnin, thinning, len, st, samples, grads, acc_out, order, 1,
                 &lv);
}

/* model.eval / evalallg on a batch x[d][C] */
void orc_eval_batch(const orc_model* m, int64_t C, const double* xs, double* lp, double* grad, int order) {
    const int d = m->d;
    double* buf = (double*)malloc(sizeof(double) * (2 * (size_t)d + orc_scratch(m)));
    for (int64_t c = 0; c < C; ++c) {
        for (int j = 0; j < d; ++j) buf[j] = xs[(size_t)j * C + c];
        lp[c] = orc_eval(m, buf, buf + d, buf + 2 * d, order);
        if (grad)
            for (int j = 0; j < d; ++j) grad[(size_t)j * C + c] = buf[d + j];
    }
    free(buf);
}

/* detmath probes (same op codes as mcmc_debug_detmath) */
void orc_detmath(int op, int64_t n, const double* x, const double* y, double* out) {
    for (int64_t i = 0; i < n; ++i) {
        double a = x[i], r = 0.0, sn, cs;
        switch (op) {
            case 0: r = orc_log(a); break;
            case 1: r = orc_exp(a); break;
            case 2: orc_sincos2pi(a, &sn, &cs); r = sn; break;
            case 3: orc_sincos2pi(a, &sn, &cs); r = cs; break;
            case 4: r = sqrt(a); break;
            case 5: r = a / y[i]; break;
            case 6: {
                uint64_t packed = (uint64_t)a;
                uint32_t ctr[4] = {(uint32_t)packed, (uint32_t)y[i], (uint32_t)(packed >> 32), ORC_TAG_NORMAL};
                uint32_t key[2] = {0u, 0u}, w[4];
                double z[4];
                orc_philox4x32_10(ctr, key, w);
                orc_normals4(w, z);
                for (int k = 0; k < 4; ++k) out[4 * i + k] = z[k];
                continue;
            }
            case 7: r = orc_round_away(a); break;
            case 9: r = orc_bm_log_u32((uint32_t)(uint64_t)a); break;
            case 10: orc_sincos2pi_u32((uint32_t)(uint64_t)a, &sn, &cs); r = sn; break;
            case 11: orc_sincos2pi_u32((uint32_t)(uint64_t)a, &sn, &cs); r = cs; break;
            case 12: r = sqrt(a); break;     /* device: sqrt_pos_normal (guard-free IEEE sequence) */
            case 13: r = orc_exp_tab(a); break;
            case 14: r = orc_log_tab(a); break;
            case 15: r = a > orc_log(y[i]) ? 1.0 : 0.0; break;    /* RWM.jl:63's test; device: gt_det_log */
            case 16: r = -2.0 * orc_bm_log_u32((uint32_t)(uint64_t)a); break;   /* device: bm_rad2_u32 */
            case 17: r = orc_bm_radius_u32((uint32_t)(uint64_t)a); break;       /* device: bm_radius_u32 */
            case 18: r = orc_erfc(a); break;
            case 19: r = orc_log1p(a); break;
            case 20: r = orc_normlogcdf(a); break;
            case 21: r = orc_bm_radius_u32((uint32_t)(uint64_t)a); break;       /* device: the LDS-table path */
            case 22: { double tm, rv; orc_logi(a, y[i], &tm, &rv); r = tm; break; }   /* logistic term (eta, w) */
            case 23: { double tm, rv; orc_logi(a, y[i], &tm, &rv); r = rv; break; }   /* ... and its weight */
            case 8: {
                uint32_t ctr[4] = {(uint32_t)(uint64_t)a, 0u, 0u, ORC_TAG_ACCEPT};
                uint32_t key[2] = {0u, 0u}, w[4];
                orc_philox4x32_10(ctr, key, w);
                r = orc_uniform52(w[0], w[1]);
            } break;
            default: r = 0.0;
        }
        out[i] = r;
    }
}

void orc_philox(int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    for (int64_t i = 0; i < n; ++i) orc_philox4x32_10(ctr + 4 * i, key + 2 * i, out + 4 * i);
}

/* ------------------------------------------------------------ output analysis
 * Effective sample size of every (parameter j, chain c) series of samples [n][d][C]
 * (ess.jl:6-10): n * var_iid / var_vtype with var_iid = var(x)/n (var.jl:7-8), and
 * vtype 1 = Geyer IMSE (var.jl:45-75), 2 = IPSE (var.jl:95-117), 3 = batch means (var.jl:20-27).
 * Autocovariances as StatsBase acf(x, lags, correlation=false): sum_t z_t z_{t+k} / n.
 * Sums left to right; sums of products (ss and the lag sums) accumulate with fma(z_t, z_{t+k}, s) -- the
 * order and rounding kernels/stats.hip uses. */
static double orc_ess_one(const double* x, size_t stride, int64_t n, int vtype, int64_t maxlag, int64_t bl,
                          double* var_out) {
    const double nd = (double)n;
    double sum = 0.0;
    for (int64_t t = 0; t < n; ++t) sum = sum + x[(size_t)t * stride];
    const double mean = sum / nd;
    double ss = 0.0;                          /* sums of products accumulate with fma (kernels/stats.hip) */
    for (int64_t t = 0; t < n; ++t) {
        const double z = x[(size_t)t * stride] - mean;
        ss = fma(z, z, ss);
    }
    const double var_iid = (ss / (nd - 1.0)) / nd;
    double var_v;
    if (vtype == 3) {
        const int64_t nb = n / bl;
        double bsum = 0.0;
        for (int64_t b = 0; b < nb; ++b) {
            double s = 0.0;
            for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + x[(size_t)t * stride];
            bsum = bsum + s / (double)bl;
        }
        const double bmean = bsum / (double)nb;
        double bss = 0.0;
        for (int64_t b = 0; b < nb; ++b) {
            double s = 0.0;
            for (int64_t t = b * bl; t < (b + 1) * bl; ++t) s = s + x[(size_t)t * stride];
            const double e = s / (double)bl - bmean;
            bss = bss + e * e;
        }
        var_v = ((double)bl * (bss / (double)(nb - 1))) / (double)(nb * bl);
    } else {
        const int64_t k = (maxlag - 1) >= 0 ? (maxlag - 1) / 2 : -1;    /* floor((maxlag-1)/2) */
        const double acv0 = ss / nd;
        double gsum = 0.0, prev = 0.0;
        for (int64_t j = 0; j <= k; ++j) {
            double acv[2];
            for (int h = 0; h < 2; ++h) {
                const int64_t lag = 2 * j + h;
                if (lag == 0) {
                    acv[h] = acv0;
                    continue;
                }
                double s = 0.0;
                for (int64_t t = 0; t + lag < n; ++t)
                    s = fma(x[(size_t)t * stride] - mean, x[(size_t)(t + lag) * stride] - mean, s);
                acv[h] = s / nd;
            }
            double g = acv[0] + acv[1];
            if (g <= 0.0) break;                                       /* m = j */
            if (vtype == 1 && j > 0 && g > prev) g = prev;             /* initial monotone sequence */
            prev = g;
            gsum = gsum + g;
        }
        var_v = (-acv0 + 2.0 * gsum) / nd;
    }
    if (var_out) *var_out = var_v;
    return (nd * var_iid) / var_v;
}

void orc_ess(const double* samples, int64_t n, int64_t d, int64_t C, int vtype, int64_t maxlag, int64_t batchlen,
             double* ess, double* var) {
    if (maxlag <= 0) maxlag = n - 1;
#pragma omp parallel for schedule(static)
    for (int64_t o = 0; o < d * C; ++o) {
        const int64_t j = o / C, c = o % C;
        ess[o] = orc_ess_one(samples + (size_t)j * C + c, (size_t)d * C, n, vtype, maxlag, batchlen,
                             var ? var + o : NULL);
    }
}

/* ------------------------------------------------------------ SeqMC population runner
 * run_seqmc (SeqMC.jl:43-122): particle n is chain n of every target.  Per outer step i and target t:
 * reset (state <- particle, lp <- eval; MCMC.reset, RWM.jl:49), one sampler step, logW += lp(reset) -
 * logtarget, logtarget <- lp after the step; resample multinomially when var(exp(logW)) < trigger.
 * The weight reductions follow kernels/seqmc.hip exactly: 256 chunks of ceil(N/256) particles summed
 * left to right, the chunk sums added left to right; cp[n] = (exclusive chunk prefix + running chunk
 * sum) / total; the resampling uniform is Philox (particle n, i, t, tag 2) under `seed`. */
#define ORC_SEQ_T 256
#define ORC_TAG_RESAMPLE 2u

void orc_seqmc(const orc_model* const* models, const orc_sampler* const* samplers, const uint64_t* seeds,
               orc_state* const* states, int64_t* steps_done, int ntargets, int64_t N, const double* particles,
               int64_t steps, int64_t burnin, double trigger, uint64_t seed, int order, double* samples,
               double* weights, int32_t* resampled) {
    const int d = models[0]->d;
    size_t sc = 0;
    for (int t = 0; t < ntargets; ++t) {
        size_t s1 = orc_scratch(models[t]);
        if (s1 > sc) sc = s1;
    }
    double* pars = (double*)malloc(sizeof(double) * (size_t)d * N);
    double* pars2 = (double*)malloc(sizeof(double) * (size_t)d * N);
    double* logW = (double*)calloc((size_t)N, sizeof(double));
    double* lt = (double*)calloc((size_t)N, sizeof(double));
    double* lt2 = (double*)malloc(sizeof(double) * N);
    double* ll0 = (double*)malloc(sizeof(double) * N);
    double* cp = (double*)malloc(sizeof(double) * N);
    double* xv = (double*)malloc(sizeof(double) * ((size_t)d + sc));
    double* tmp = xv + d;
    memcpy(pars, particles, sizeof(double) * (size_t)d * N);
    const int64_t chunk = (N + ORC_SEQ_T - 1) / ORC_SEQ_T;
    for (int64_t i = 1; i <= steps; ++i) {
        for (int t = 0; t < ntargets; ++t) {
            const orc_model* m = models[t];
            orc_state* st = states[t];
            for (int64_t n = 0; n < N; ++n) {                       /* MCMC.reset(t, pars[n]) */
                for (int j = 0; j < d; ++j) {
                    st->x[(size_t)j * N + n] = pars[(size_t)j * N + n];
                    xv[j] = pars[(size_t)j * N + n];
                }
                st->lp[n] = orc_eval(m, xv, NULL, tmp, orc_eval_order(order));
                ll0[n] = st->lp[n];
            }
            orc_run(m, samplers[t], seeds[t], 0, N, 0, N, steps_done[t], 0, 1, 1, st, NULL, NULL, NULL, order, 1);
            steps_done[t] += 1;
            memcpy(pars, st->x, sizeof(double) * (size_t)d * N);      /* pars[n] = sample.ppars */
            for (int64_t n = 0; n < N; ++n) {
                logW[n] = logW[n] + (ll0[n] - lt[n]);
                lt[n] = st->lp[n];
            }
            /* var(W) and cumsum(W)/sum(W) in the kernel's chunked order */
            double part[ORC_SEQ_T], qpart[ORC_SEQ_T];
            for (int k = 0; k < ORC_SEQ_T; ++k) {
                int64_t b = (int64_t)k * chunk, e = b + chunk < N ? b + chunk : N;
                double s = 0.0;
                for (int64_t n = b; n < e; ++n) s = s + orc_exp(logW[n]);
                part[k] = s;
            }
            double total = 0.0;
            for (int k = 0; k < ORC_SEQ_T; ++k) total = total + part[k];
            const double mean = total / (double)N;
            for (int k = 0; k < ORC_SEQ_T; ++k) {
                int64_t b = (int64_t)k * chunk, e = b + chunk < N ? b + chunk : N;
                double q = 0.0;
                for (int64_t n = b; n < e; ++n) {
                    double dv = orc_exp(logW[n]) - mean;
                    q = q + dv * dv;
                }
                qpart[k] = q;
            }
            double ss = 0.0;
            for (int k = 0; k < ORC_SEQ_T; ++k) ss = ss + qpart[k];
            const int flag = (ss / (double)(N - 1)) < trigger;
            if (resampled) resampled[(size_t)(i - 1) * ntargets + t] = flag;
            double run = 0.0;
            for (int k = 0; k < ORC_SEQ_T; ++k) {
                int64_t b = (int64_t)k * chunk, e = b + chunk < N ? b + chunk : N;
                double pre = run;
                for (int64_t n = b; n < e; ++n) {
                    pre = pre + orc_exp(logW[n]);
                    cp[n] = pre / total;
                }
                run = run + part[k];
            }
            if (flag) {
                for (int64_t n = 0; n < N; ++n) {
                    uint32_t w[4];
                    orc_block(seed, (uint32_t)n, (uint32_t)i, (uint32_t)t, ORC_TAG_RESAMPLE, w);
                    const double u = orc_uniform52(w[0], w[1]);
                    int64_t lo = 0, hi = N - 1;
                    while (lo < hi) {
                        int64_t mid = lo + (hi - lo) / 2;
                        if (cp[mid] >= u) hi = mid;
                        else lo = mid + 1;
                    }
                    for (int j = 0; j < d; ++j) pars2[(size_t)j * N + n] = pars[(size_t)j * N + lo];
                    lt2[n] = lt[lo];
                }
                for (int64_t n = 0; n < N; ++n) logW[n] = 0.0;
                memcpy(pars, pars2, sizeof(double) * (size_t)d * N);
                memcpy(lt, lt2, sizeof(double) * N);
            }
        }
        for (int64_t n = 0; n < N; ++n) lt[n] = 0.0;                 /* logtarget = zeros(npart) */
        if (i > burnin) {
            const size_t row = (size_t)(i - burnin - 1);
            if (samples) memcpy(samples + row * (size_t)d * N, pars, sizeof(double) * (size_t)d * N);
            if (weights)
                for (int64_t n = 0; n < N; ++n) weights[row * N + n] = orc_exp(logW[n]);
        }
    }
    free(pars); free(pars2); free(logW); free(lt); free(lt2); free(ll0); free(cp); free(xv);
}
