// models.hpp -- separable log-targets of the model catalogue, device side.
//
// The reference evaluates user closures (likmodel.jl:21,25) or DSL-generated
// code (modelparser.jl:39-104).  Across the C ABI the model is a catalogue
// entry; each entry restates the arithmetic of its reference definition:
//
//   IsoDot     model(v -> -dot(v,v), grad = v -> -2v)   README.md:60,63;
//              test/test_syntax.jl:40-41.  A function model: no LLAcc rule,
//              the closure's value is used as is (likmodel.jl:100-143).
//   NormalDSL  :(v ~ Normal(mu, sigma)), gradient=true  README.md:67-72.
//              lp = LLAcc(0.) + sum(logpdf(Normal(mu,sigma), v)) and a
//              non-finite running sum throws OutOfSupportError, which the
//              generated function turns into (-Inf, zero(beta))
//              (AccumulatorDerivRules.jl:14-16, modelparser.jl:64-72).
//              Gradient rule dx += (mu - x)/(sigma*sigma) * ds (MCMCDerivRules.jl:57).
//   AbsNormalDSL :(y = abs(x); y ~ Normal(mu, sigma))   README.md:246-251 (the SeqMC example):
//              lp = LLAcc(0.) + sum(logpdf(Normal(mu,sigma), |v|)).  Gradient: the Normal rule
//              times d|v|/dv = sign(v) (ReverseDiffSource's rule for abs is not vendored: that
//              factor is "parity unpinned"; the README example runs RWM, which needs no gradient).
//
// Summation: the reference sums with BLAS ddot / Julia `sum`; the build fixes
// the order so that the oracle can restate it exactly: lane-per-chain kernels
// sum left to right over j; wave-per-chain kernels sum each lane's coordinates
// in order and then combine the 64 lane partials by an xor butterfly
// (DESIGN.md §4).  Accumulation is `acc = fma(v, v, acc)` for the dot product
// and `acc = acc + term` for logpdf sums.
#pragma once
#include "common.hpp"
#include "detmath.hpp"

namespace mcmc {

constexpr double kLog2Pi = 0x1.d67f1c864beb5p+0;   // log(2*pi) rounded
constexpr double kTwoPi = 0x1.921fb54442d18p+2;    // 2*pi rounded (Julia 2*pi)

struct IsoDot {
    static constexpr const char* kName = "IsoDot";
    static constexpr bool kLLAcc = false;
    // 0.5 * grad(v) = 0.5 * (-2 v) is -v exactly while |v| < 2^1023 (samplers.hpp trajectory_halfneg)
    static constexpr bool kHalfGradNeg = true;
    __device__ explicit IsoDot(const ModelArgs&) {}
    __device__ __forceinline__ void acc(double& a, double v) const { a = __builtin_fma(v, v, a); }
    __device__ __forceinline__ double finish(double a) const { return -a; }
    __device__ __forceinline__ double grad(double v) const { return -2.0 * v; }
};

struct NormalDSL {
    static constexpr const char* kName = "NormalDSL";
    static constexpr bool kLLAcc = true;
    static constexpr bool kHalfGradNeg = false;
    double mu, sigma, logsig, s2;
    __device__ explicit NormalDSL(const ModelArgs& m) : mu(m.mu), sigma(m.sigma) {
        logsig = det_log(sigma);
        s2 = sigma * sigma;
    }
    __device__ __forceinline__ void acc(double& a, double v) const {
        const double z = (v - mu) / sigma;
        a = a + (-0.5 * (z * z + kLog2Pi) - logsig);
    }
    __device__ __forceinline__ double finish(double a) const { return a; }
    __device__ __forceinline__ double grad(double v) const { return (mu - v) / s2; }
};

struct AbsNormalDSL {
    static constexpr const char* kName = "AbsNormalDSL";
    static constexpr bool kLLAcc = true;
    static constexpr bool kHalfGradNeg = false;
    double mu, sigma, logsig, s2;
    __device__ explicit AbsNormalDSL(const ModelArgs& m) : mu(m.mu), sigma(m.sigma) {
        logsig = det_log(sigma);
        s2 = sigma * sigma;
    }
    __device__ __forceinline__ void acc(double& a, double v) const {
        const double z = (__builtin_fabs(v) - mu) / sigma;
        a = a + (-0.5 * (z * z + kLog2Pi) - logsig);
    }
    __device__ __forceinline__ double finish(double a) const { return a; }
    __device__ __forceinline__ double grad(double v) const {
        const double sg = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0);
        return sg * ((mu - __builtin_fabs(v)) / s2);
    }
};

// v ~ Dist(p1, p2) elementwise: logpdf and the x-derivative rules of MCMCDerivRules.jl:56-104
// (Distributions.jl parametrisations: Weibull(shape, scale), Beta(alpha, beta), TDist(df),
// Exponential(scale), Gamma(shape, scale), Cauchy(location, scale), LogNormal(meanlog, sdlog),
// Laplace(location, scale), Uniform(a, b)).  Outside the support the term is -Inf, which the LLAcc rule
// turns into (-Inf, zero gradient).  `c` holds the parameter-only part (lgamma / log terms), computed on
// the host (restated by oracle/oracle.c orc_dist_const).  The distribution is uniform over a launch:
// the switch is a scalar branch.
struct DistDSL {
    static constexpr const char* kName = "DistDSL";
    static constexpr bool kLLAcc = true;
    static constexpr bool kHalfGradNeg = false;
    int32_t dist;
    double p1, p2, c;
    __device__ explicit DistDSL(const ModelArgs& m) : dist(m.dist), p1(m.mu), p2(m.sigma), c(m.dconst) {
    }
    __device__ __forceinline__ double logpdf(double v) const {
        const double ninf = -__builtin_inf();
        switch (dist) {
            case DK_NORMAL: { const double z = (v - p1) / p2; return -0.5 * (z * z + kLog2Pi) + c; }
            case DK_UNIFORM: return (v >= p1 && v <= p2) ? c : ninf;
            case DK_WEIBULL: {
                if (v < 0.0) return ninf;
                const double lr = det_log(v / p2);
                return c + (p1 - 1.0) * lr - det_exp(p1 * lr);
            }
            case DK_BETA:
                if (v < 0.0 || v > 1.0) return ninf;
                return (p1 - 1.0) * det_log(v) + (p2 - 1.0) * det_log(1.0 - v) + c;
            case DK_TDIST: return c - ((p1 + 1.0) / 2.0) * det_log(1.0 + (v * v) / p1);
            case DK_EXPONENTIAL: return v < 0.0 ? ninf : c - v / p1;
            case DK_GAMMA: return v < 0.0 ? ninf : (p1 - 1.0) * det_log(v) - v / p2 + c;
            case DK_CAUCHY: { const double z = (v - p1) / p2; return c - det_log(1.0 + z * z); }
            case DK_LOGNORMAL: {
                if (v <= 0.0) return ninf;
                const double lv = det_log(v), e = lv - p1;
                return -(e * e) / (2.0 * p2 * p2) - lv + c;
            }
            case DK_LAPLACE: return c - __builtin_fabs(v - p1) / p2;
            default: return bits2d(0x7ff8000000000000ull);
        }
    }
    __device__ __forceinline__ void acc(double& a, double v) const { a = a + logpdf(v); }
    __device__ __forceinline__ double finish(double a) const { return a; }
    __device__ __forceinline__ double grad(double v) const {
        switch (dist) {
            case DK_NORMAL: return (p1 - v) / (p2 * p2);                                       // :57
            case DK_UNIFORM: return 0.0;                                                       // :62
            case DK_WEIBULL: return ((1.0 - det_exp(p1 * det_log(v / p2))) * p1 - 1.0) / v;   // :69
            case DK_BETA: return (p1 - 1.0) / v - (p2 - 1.0) / (1.0 - v);                      // :74
            case DK_TDIST: return -(p1 + 1.0) * v / (p1 + v * v);                              // :79
            case DK_EXPONENTIAL: return -1.0 / p1;                                             // :83
            case DK_GAMMA: return -(p2 + v - p1 * p2) / (p2 * v);                              // :88
            case DK_CAUCHY: { const double e = v - p1; return 2.0 * (p1 - v) / (p2 * p2 + e * e); }   // :93
            case DK_LOGNORMAL: return (p1 - p2 * p2 - det_log(v)) / (p2 * p2 * v);             // :98
            case DK_LAPLACE: return (v > p1 ? -1.0 : 1.0) / p2;                                // :103
            default: return 0.0;
        }
    }
};

// The DSL block `y = x * v; y ~ Dist(p1, p2)` of the reference's bare_distribs benchmark unit
// (benchmarks/benchunits/bare_distribs.jl:13): a scalar parameter x (d = 1) scaling a data vector v of n entries,
// log-target sum_i logpdf(D, x v_i) (LLAcc: left to right), d/dx = sum_i v_i dlogpdf(D, x v_i) (the reverse rule of
// y = x * v).  The data is read by every lane at the same address (a broadcast from L1 / L2).
struct DistObsDSL {
    static constexpr const char* kName = "DistObsDSL";
    static constexpr bool kLLAcc = true;
    static constexpr bool kHalfGradNeg = false;
    DistDSL D;
    const double* v;
    int64_t n;
    __device__ explicit DistObsDSL(const ModelArgs& m) : D(m), v(m.Y), n(m.n) {}
    __device__ __forceinline__ void acc(double& a, double x) const {
        for (int64_t i = 0; i < n; ++i) a = a + D.logpdf(x * v[i]);
    }
    __device__ __forceinline__ double finish(double a) const { return a; }
    __device__ __forceinline__ double grad(double x) const {
        double g = 0.0;
        for (int64_t i = 0; i < n; ++i) g = g + v[i] * D.grad(x * v[i]);
        return g;
    }
};

// LLAcc rule: a non-finite total means out of support -> (-Inf, 0).
template <class M>
__device__ __forceinline__ double llacc_finish(const M& m, double a, bool& oos) {
    double lp = m.finish(a);
    oos = false;
    if (M::kLLAcc) {
        oos = !(lp - lp == 0.0);      // !isfinite(lp)
        if (oos) lp = -__builtin_inf();
    }
    return lp;
}

}  // namespace mcmc
