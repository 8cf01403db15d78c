// lpc.hip -- lane-per-chain fused step kernels for separable targets (d <= 32).
//
// One thread owns one chain; 64 consecutive chains form a wave, so every state
// access x[j][c] is a coalesced 512-byte wave access and the accept mask of a
// wave is one __ballot word.  The chain's parameter vector stays in VGPRs for
// all `nsteps` steps of a launch (the SerialMC loop, SerialMC.jl:47-67, runs
// inside the kernel); HBM sees the state once per launch, the kept samples and
// the accept bits.  With nsteps == 1 the same kernel is the classic one-launch-
// per-step streaming kernel (16d + 16 B of state traffic per chain-step).
//
// Per step (reference file:line for each sampler):
//   RWM    RWM.jl:58-71      x' = x + randn .* scale; accept iff r > 0 || r > log(rand())
//   MALA   MALA.jl:89-125    Langevin proposal, forward/backward densities, EmpMCTuner
//   HMC    HMC.jl:252-299    L leapfrogs (HMC.jl:219-228), accept iff rand() < exp(H0 - H)
//   HMCDA  HMCDA.jl:97-142   nLeaps = max(1, round(len/eps)), p = min(1, exp(H0-H)),
//                            dual averaging while i < burnin
// Random stream: normals of step i for chain c come from Philox blocks
// (c, i, b, TAG_NORMAL), b = 0..ceil(d/4)-1, coordinate j <- block j/4, slot j%4;
// the accept uniform from block (c, i, 0, TAG_ACCEPT).
#include "../common.hpp"
#include "../detmath.hpp"
#include "../models.hpp"
#include "../host/kernels_api.hpp"

namespace mcmc {

constexpr int kLpcBlock = 256;

template <int NB>
__device__ __forceinline__ void gen_normals(const Stream& rs, uint32_t chain, uint32_t step, double (&z)[4 * NB]) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const u32x4 w = rs.block(chain, step, (uint32_t)b, TAG_NORMAL);
        normals4(w, z[4 * b], z[4 * b + 1], z[4 * b + 2], z[4 * b + 3]);
    }
}

template <int NB, class M>
__device__ __forceinline__ double eval_lp(const M& model, const double (&v)[4 * NB], int d, bool& oos) {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j)
        if (j < d) model.acc(a, v[j]);
    return llacc_finish(model, a, oos);
}

__device__ __forceinline__ bool mh_accept_short_circuit(const Stream& rs, uint32_t chain, uint32_t step, double ratio) {
    // RWM.jl:63 / MALA.jl:108: ratio > 0 || ratio > log(rand()); the uniform is drawn only if needed.
    bool acc = ratio > 0.0;
    if (!acc) {
        const u32x4 w = rs.block(chain, step, 0u, TAG_ACCEPT);
        acc = ratio > det_log(uniform53(w.x, w.y));
    }
    return acc;
}

// tuner adaptation factor (MALA.jl:36-39, HMC.jl:165-169)
__device__ __forceinline__ double tune_factor(int32_t acc, int32_t prop, double target) {
    const double rate = (double)acc / (double)prop;
    return 1.0 / (1.0 + det_exp(-11.0 * (rate - target))) + 0.5;
}

template <int NB>
__device__ __forceinline__ void store_kept(const StepArgs& s, int64_t c, bool live, int64_t kk,
                                           const double (&v)[4 * NB], double* base) {
    if (base == nullptr || !live) return;
    double* p = base + (size_t)kk * (size_t)s.d * (size_t)s.C + (size_t)c;
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j)
        if (j < s.d) p[(size_t)j * (size_t)s.C] = v[j];
}

__device__ __forceinline__ void store_bits(const StepArgs& s, int64_t c, int64_t kk, bool acc_live) {
    const uint64_t mask = __ballot(acc_live);
    if ((threadIdx.x & 63) == 0 && s.acc_bits != nullptr) {
        const int64_t w = c >> 6;
        if (w < s.nw) s.acc_bits[(size_t)kk * (size_t)s.nw + (size_t)w] = mask;
    }
}

// ------------------------------------------------------------------ RWM
template <int NB, class M>
__global__ __launch_bounds__(kLpcBlock) void lpc_rwm(LpcArgs a) {
    const StepArgs& s = a.s;
    const int64_t c = (int64_t)blockIdx.x * kLpcBlock + threadIdx.x;
    const bool live = c < s.C;
    const int64_t cc = live ? c : 0;
    const int d = s.d;
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)c;

    double x[4 * NB], sc[4 * NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j) {
        x[j] = (j < d) ? a.st.x[(size_t)j * s.ld + cc] : 0.0;
        sc[j] = (j < d) ? s.scale[j] : 0.0;
    }
    double lp = a.st.lp[cc];

    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        double xp[4 * NB];
        gen_normals<NB>(rs, chain, (uint32_t)i, xp);            // xp <- z
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) xp[j] = x[j] + xp[j] * sc[j];
        bool oos;
        const double lpp = eval_lp<NB>(model, xp, d, oos);
        const double ratio = lpp - lp;
        const bool acc = mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
#pragma unroll
            for (int j = 0; j < 4 * NB; ++j) x[j] = xp[j];
            lp = lpp;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            store_kept<NB>(s, c, live, kk, x, s.samples);
            store_bits(s, c, kk, acc && live);
        }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j)
            if (j < d) a.st.x[(size_t)j * s.ld + c] = x[j];
        a.st.lp[c] = lp;
    }
}

// ------------------------------------------------------------------ MALA
template <int NB, class M>
__global__ __launch_bounds__(kLpcBlock) void lpc_mala(LpcArgs a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const int64_t c = (int64_t)blockIdx.x * kLpcBlock + threadIdx.x;
    const bool live = c < s.C;
    const int64_t cc = live ? c : 0;
    const int d = s.d;
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)c;

    double x[4 * NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j) x[j] = (j < d) ? a.st.x[(size_t)j * s.ld + cc] : 0.0;
    double lp = a.st.lp[cc];
    double h = sa.tuner ? a.st.t_step[cc] : sa.drift_step;
    int32_t n_acc = sa.tuner ? a.st.t_acc[cc] : 0;
    int32_t n_prop = sa.tuner ? a.st.t_prop[cc] : 0;

    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (sa.tuner) n_prop += 1;
        const double half = h / 2.0;
        const double sq = __builtin_sqrt(h);
        const double twoh = 2.0 * h;
        const double L = det_log(kTwoPi * h) / 2.0;
        double xp[4 * NB];
        gen_normals<NB>(rs, chain, (uint32_t)i, xp);
        double qf = 0.0;
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) {
            const double pm = x[j] + half * model.grad(x[j]);       // parsMean (MALA.jl:98)
            xp[j] = pm + sq * xp[j];                                // MALA.jl:100
            const double e = pm - xp[j];
            if (j < d) qf = qf + ((-(e * e)) / twoh - L);           // MALA.jl:103
        }
        bool oos;
        const double lpp = eval_lp<NB>(model, xp, d, oos);
        double qb = 0.0;
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) {
            const double gp = oos ? 0.0 : model.grad(xp[j]);
            const double e = (xp[j] + half * gp) - x[j];           // MALA.jl:104-105
            if (j < d) qb = qb + ((-(e * e)) / twoh - L);
        }
        const double ratio = ((lpp + qb) - lp) - qf;                // MALA.jl:107
        const bool acc = mh_accept_short_circuit(rs, chain, (uint32_t)i, ratio);
        if (acc) {
#pragma unroll
            for (int j = 0; j < 4 * NB; ++j) x[j] = xp[j];
            lp = lpp;
            if (sa.tuner) n_acc += 1;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            store_kept<NB>(s, c, live, kk, x, s.samples);
            if (s.grads != nullptr) {
                double g[4 * NB];
#pragma unroll
                for (int j = 0; j < 4 * NB; ++j) g[j] = model.grad(x[j]);
                store_kept<NB>(s, c, live, kk, g, s.grads);
            }
            store_bits(s, c, kk, acc && live);
        }
        if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // MALA.jl:116-118
            h = h * tune_factor(n_acc, n_prop, sa.target_rate);
            n_acc = 0;
            n_prop = 0;
        }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j)
            if (j < d) a.st.x[(size_t)j * s.ld + c] = x[j];
        a.st.lp[c] = lp;
        if (sa.tuner) {
            a.st.t_step[c] = h;
            a.st.t_acc[c] = n_acc;
            a.st.t_prop[c] = n_prop;
        }
    }
}

// ------------------------------------------------------------------ HMC / HMCDA
// One trajectory of nl leapfrogs from (x0, m) (HMC.jl:219-228, 262-277).
// Returns the final log-target; x, m hold the end point.
template <int NB, class M>
__device__ __forceinline__ double trajectory(const M& model, int d, double eps, int64_t nl,
                                             double (&x)[4 * NB], double (&m)[4 * NB], bool& oos_end) {
    bool oos = false;                                               // start point is in support
    double lpl = 0.0;
    for (int64_t l = 0; l < nl; ++l) {
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) {
            const double g = oos ? 0.0 : model.grad(x[j]);
            m[j] = m[j] + (0.5 * g) * eps;                          // n.m += 0.5*n.grad*ve
            x[j] = x[j] + eps * m[j];                               // n.pars += ve * n.m
        }
        lpl = eval_lp<NB>(model, x, d, oos);                        // calc!(n, ll)
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) {
            const double g = oos ? 0.0 : model.grad(x[j]);
            m[j] = m[j] + (0.5 * g) * eps;
        }
    }
    oos_end = oos;
    return lpl;
}

template <int NB>
__device__ __forceinline__ double half_dot(const double (&m)[4 * NB], int d) {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j)
        if (j < d) a = __builtin_fma(m[j], m[j], a);
    return 0.5 * a;
}

template <int NB, class M, bool DA>
__global__ __launch_bounds__(kLpcBlock) void lpc_hmc(LpcArgs a) {
    const StepArgs& s = a.s;
    const SamplerArgs& sa = a.sa;
    const int64_t c = (int64_t)blockIdx.x * kLpcBlock + threadIdx.x;
    const bool live = c < s.C;
    const int64_t cc = live ? c : 0;
    const int d = s.d;
    const M model(a.m);
    const Stream rs{s.key0, s.key1};
    const uint32_t chain = s.chain0 + (uint32_t)c;
    const int64_t max_leaps = sa.max_leaps;

    double x0[4 * NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j) x0[j] = (j < d) ? a.st.x[(size_t)j * s.ld + cc] : 0.0;
    double lp = a.st.lp[cc];
    // HMC: (nLeaps, leapStep), tuned or fixed.  HMCDA: leapStep, dualLeapStep, dualH.
    double eps = (DA || sa.tuner) ? a.st.t_step[cc] : sa.leap_step;
    int64_t nl_fixed = (!DA && sa.tuner) ? (int64_t)a.st.t_leaps[cc] : sa.n_leaps;
    double eps_bar = DA ? a.st.t_bar[cc] : 0.0;
    double h_bar = DA ? a.st.t_h[cc] : 0.0;
    int32_t n_acc = (!DA && sa.tuner) ? a.st.t_acc[cc] : 0;
    int32_t n_prop = (!DA && sa.tuner) ? a.st.t_prop[cc] : 0;
    const double mu = DA ? det_log(10.0) : 0.0;                       // log(10*leapStep0), leapStep0 = 1

    for (int t = 0; t < s.nsteps; ++t) {
        const int64_t i = s.step_begin + t;
        if (!DA && sa.tuner) n_prop += 1;
        double m[4 * NB], x[4 * NB];
        gen_normals<NB>(rs, chain, (uint32_t)i, m);                 // state0.m = randn(model.size)
        const double H0 = -lp + half_dot<NB>(m, d);                 // update!(state0)
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j) x[j] = x0[j];
        int64_t nl;
        if (DA) {
            const double r = round_away(sa.len / eps);              // HMCDA.jl:104
            nl = r < 1.0 ? 1 : (r > (double)max_leaps ? max_leaps : (int64_t)r);
        } else {
            nl = nl_fixed;
        }
        bool oos;
        const double lpl = trajectory<NB>(model, d, eps, nl, x, m, oos);
        const double H = -lpl + half_dot<NB>(m, d);
        const u32x4 w = rs.block(chain, (uint32_t)i, 0u, TAG_ACCEPT);
        const double u = uniform53(w.x, w.y);
        bool acc;
        double p = 0.0;
        if (DA) {
            p = __builtin_fmin(1.0, det_exp(H0 - H));              // HMCDA.jl:120 (Julia 0.2 min: NaN-ignoring)
            acc = u < p;
        } else {
            acc = u < det_exp(H0 - H);                              // HMC.jl:280
        }
        if (acc) {
#pragma unroll
            for (int j = 0; j < 4 * NB; ++j) x0[j] = x[j];
            lp = lpl;
            if (!DA && sa.tuner) n_acc += 1;
        }
        int64_t kk;
        if (kept_index(i - s.run_step0, s.burnin, s.thinning, s.len, &kk)) {
            store_kept<NB>(s, c, live, kk, x0, s.samples);
            if (s.grads != nullptr) {
                double g[4 * NB];
#pragma unroll
                for (int j = 0; j < 4 * NB; ++j) g[j] = model.grad(x0[j]);
                store_kept<NB>(s, c, live, kk, g, s.grads);
            }
            store_bits(s, c, kk, acc && live);
        }
        if (DA) {
            const double di = (double)i;
            if (di < (double)s.tuner_burnin) {                      // HMCDA.jl:133-138
                double eta = 1.0 / (di + sa.t0);
                h_bar = (1.0 - eta) * h_bar + eta * (sa.rate - p);
                eps = det_exp(mu - (__builtin_sqrt(di) * h_bar) / sa.shrinkage);
                eta = det_exp(det_log(di) * (-sa.step));            // i^(-step)
                eps_bar = det_exp((1.0 - eta) * det_log(eps_bar) + eta * det_log(eps));
            } else {
                eps = eps_bar;                                      // HMCDA.jl:140
            }
        } else if (sa.tuner && i <= s.tuner_burnin && (i % sa.adapt_step) == 0) {   // HMC.jl:293-295
            eps = eps * tune_factor(n_acc, n_prop, sa.target_rate);
            double nlf = __builtin_ceil(sa.target_path / eps);
            if (nlf > (double)sa.max_step) nlf = (double)sa.max_step;
            if (nlf > (double)max_leaps) nlf = (double)max_leaps;
            nl_fixed = (int64_t)nlf;
            n_acc = 0;
            n_prop = 0;
        }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j)
            if (j < d) a.st.x[(size_t)j * s.ld + c] = x0[j];
        a.st.lp[c] = lp;
        if (DA || sa.tuner) a.st.t_step[c] = eps;
        if (DA) {
            a.st.t_bar[c] = eps_bar;
            a.st.t_h[c] = h_bar;
        } else if (sa.tuner) {
            a.st.t_leaps[c] = (int32_t)nl_fixed;
            a.st.t_acc[c] = n_acc;
            a.st.t_prop[c] = n_prop;
        }
    }
}

// ------------------------------------------------------------------ init / eval
// x <- init (or given), lp <- model.eval(x); flags chains whose start is out of support
// (RWM.jl:54-55 "Initial values out of model support, try other values").
template <int NB, class M>
__global__ __launch_bounds__(kLpcBlock) void lpc_eval(LpcArgs a, const double* xin, int64_t ldin,
                                                     double* lp_out, double* g_out, int32_t check) {
    const StepArgs& s = a.s;
    const int64_t c = (int64_t)blockIdx.x * kLpcBlock + threadIdx.x;
    if (c >= s.C) return;
    const int d = s.d;
    const M model(a.m);
    double x[4 * NB];
#pragma unroll
    for (int j = 0; j < 4 * NB; ++j) x[j] = (j < d) ? xin[(size_t)j * ldin + c] : 0.0;
    bool oos;
    const double lp = eval_lp<NB>(model, x, d, oos);
    lp_out[c] = lp;
    if (g_out != nullptr) {
#pragma unroll
        for (int j = 0; j < 4 * NB; ++j)
            if (j < d) g_out[(size_t)j * ldin + c] = oos ? 0.0 : model.grad(x[j]);
    }
    if (check && !(lp - lp == 0.0)) atomicOr(s.err, 1);
}

// ------------------------------------------------------------------ dispatch
template <int NB, class M>
static hipError_t launch_lpc_model(const LpcArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kLpcBlock - 1) / kLpcBlock));
    switch (a.sa.kind) {
        case SK_RWM: lpc_rwm<NB, M><<<grid, kLpcBlock, 0, st>>>(a); break;
        case SK_MALA: lpc_mala<NB, M><<<grid, kLpcBlock, 0, st>>>(a); break;
        case SK_HMC: lpc_hmc<NB, M, false><<<grid, kLpcBlock, 0, st>>>(a); break;
        case SK_HMCDA: lpc_hmc<NB, M, true><<<grid, kLpcBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int NB>
static hipError_t launch_lpc_nb(const LpcArgs& a, hipStream_t st) {
    if (a.m.kind == MK_ISO) return launch_lpc_model<NB, IsoDot>(a, st);
    if (a.m.kind == MK_NORMAL) return launch_lpc_model<NB, NormalDSL>(a, st);
    return hipErrorInvalidValue;
}

template <int NB, class M>
static hipError_t launch_eval_model(const LpcArgs& a, const double* xin, int64_t ldin, double* lp, double* g,
                                    int check, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kLpcBlock - 1) / kLpcBlock));
    lpc_eval<NB, M><<<grid, kLpcBlock, 0, st>>>(a, xin, ldin, lp, g, check);
    return hipGetLastError();
}

template <int NB>
static hipError_t launch_eval_nb(const LpcArgs& a, const double* xin, int64_t ldin, double* lp, double* g, int check,
                                 hipStream_t st) {
    if (a.m.kind == MK_ISO) return launch_eval_model<NB, IsoDot>(a, xin, ldin, lp, g, check, st);
    if (a.m.kind == MK_NORMAL) return launch_eval_model<NB, NormalDSL>(a, xin, ldin, lp, g, check, st);
    return hipErrorInvalidValue;
}

static int lpc_nb_for(int d) {
    if (d <= 4) return 1;
    if (d <= 8) return 2;
    if (d <= 16) return 4;
    if (d <= 32) return 8;
    return 0;
}

}  // namespace mcmc

// Host-visible entry points used by the runtime (C++ linkage inside the library).
hipError_t mcmc_launch_lpc_step(const mcmc::LpcArgs& a, hipStream_t st) {
    switch (mcmc::lpc_nb_for(a.s.d)) {
        case 1: return mcmc::launch_lpc_nb<1>(a, st);
        case 2: return mcmc::launch_lpc_nb<2>(a, st);
        case 4: return mcmc::launch_lpc_nb<4>(a, st);
        case 8: return mcmc::launch_lpc_nb<8>(a, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_lpc_eval(const mcmc::LpcArgs& a, const double* xin, int64_t ldin, double* lp, double* g,
                                int check, hipStream_t st) {
    switch (mcmc::lpc_nb_for(a.s.d)) {
        case 1: return mcmc::launch_eval_nb<1>(a, xin, ldin, lp, g, check, st);
        case 2: return mcmc::launch_eval_nb<2>(a, xin, ldin, lp, g, check, st);
        case 4: return mcmc::launch_eval_nb<4>(a, xin, ldin, lp, g, check, st);
        case 8: return mcmc::launch_eval_nb<8>(a, xin, ldin, lp, g, check, st);
        default: return hipErrorInvalidValue;
    }
}

int mcmc_lpc_max_d() { return 32; }
