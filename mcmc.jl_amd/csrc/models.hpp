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
#include <type_traits>
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

// The Ornstein-Uhlenbeck model of examples/ornstein.jl:19-30 -- a joint (non-separable) target over
// v = (tau, sigma, mu) and a series y[0..n-1]:
//     tau ~ Uniform(0, 100); sigma ~ Uniform(0, 2); mu ~ Uniform(0, 20)
//     fac = exp(-1/tau); resid = y[2:end] - y[1:end-1] * fac - mu * (1 - fac); resid ~ Normal(0, sigma)
// LLAcc order: ((0 + logpdf(U, tau)) + logpdf(U, sigma)) + logpdf(U, mu) is the host constant c0 (-log(b - a) each,
// glibc log), then + sum(logpdf(Normal(0, sigma), resid)) summed left to right; an out-of-support prior is -Inf
// (AccumulatorDerivRules.jl:12-20).  Gradient: reverse mode through the expression with the DSL's rules
// (MCMCDerivRules.jl:57-59 Normal dx / dsigma, :62 Uniform dx = 0):
//     dr_i = (0 - r_i) / (sigma sigma);  G0 = sum dr_i;  G1 = sum dr_i y_i;  Gs = sum ((r_i r_i) / (sigma sigma) - 1) / sigma
//     d tau = (mu G0 - G1) (fac / (tau tau));  d sigma = Gs;  d mu = -(G0 (1 - fac))
// Joint models run lane per chain only (the runtime refuses other widths); the series is read by every lane at the
// same address (a broadcast).  oracle.c ORC_MODEL_OU is the twin.
struct OUDSL {
    static constexpr const char* kName = "OUDSL";
    static constexpr bool kLLAcc = true;
    static constexpr bool kHalfGradNeg = false;
    static constexpr bool kJoint = true;
    const double* y;
    int64_t n;
    double c0;
    __device__ explicit OUDSL(const ModelArgs& m) : y(m.Y), n(m.n), c0(m.dconst) {}
    __device__ __forceinline__ static bool in_support(double tau, double sigma, double mu) {
        return tau >= 0.0 && tau <= 100.0 && sigma >= 0.0 && sigma <= 2.0 && mu >= 0.0 && mu <= 20.0;
    }
    template <int NC>
    __device__ __forceinline__ double joint_lp(const double (&v)[NC], bool& oos) const {
        oos = true;
        if constexpr (NC < 3) return -__builtin_inf();   // never run: the runtime refuses d != 3 (lpc_rwm_spec<1|2>)
        const double tau = v[0], sigma = v[1 < NC ? 1 : 0], mu = v[2 < NC ? 2 : 0];
        if (!in_support(tau, sigma, mu)) return -__builtin_inf();
        const double fac = det_exp(-1.0 / tau);
        const double c = mu * (1.0 - fac);
        const double logsig = det_log(sigma);
        double s = 0.0;
        double y0 = y[0];
        for (int64_t i = 1; i < n; ++i) {
            const double y1 = y[i];
            const double z = ((y1 - y0 * fac) - c) / sigma;
            s = s + (-0.5 * (z * z + kLog2Pi) - logsig);
            y0 = y1;
        }
        const double lp = c0 + s;
        oos = !(lp - lp == 0.0);
        return oos ? -__builtin_inf() : lp;
    }
    template <int NC>
    __device__ __forceinline__ void joint_grad(const double (&v)[NC], double (&g)[NC]) const {
        static_assert(NC >= 3, "the OU model has 3 parameters");
        const double tau = v[0], sigma = v[1], mu = v[2];
        const double fac = det_exp(-1.0 / tau);
        const double c = mu * (1.0 - fac);
        const double s2 = sigma * sigma;
        double g0 = 0.0, g1 = 0.0, gs = 0.0;
        double y0 = y[0];
        for (int64_t i = 1; i < n; ++i) {
            const double y1 = y[i];
            const double r = (y1 - y0 * fac) - c;
            const double dr = (0.0 - r) / s2;
            g0 = g0 + dr;
            g1 = g1 + dr * y0;
            gs = gs + ((r * r) / s2 - 1.0) / sigma;
            y0 = y1;
        }
#pragma unroll
        for (int k = 0; k < NC; ++k) g[k] = 0.0;
        g[0] = (mu * g0 - g1) * (fac / (tau * tau));
        g[1] = gs;
        g[2] = -(g0 * (1.0 - fac));
    }
    // the per-coordinate interface of separable models is never used for a joint model
    __device__ __forceinline__ void acc(double&, double) const {}
    __device__ __forceinline__ double finish(double a) const { return a; }
    __device__ __forceinline__ double grad(double) const { return 0.0; }
};

template <class M, class = void>
struct is_joint : std::false_type {};
template <class M>
struct is_joint<M, std::void_t<decltype(M::kJoint)>> : std::bool_constant<M::kJoint> {};

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
