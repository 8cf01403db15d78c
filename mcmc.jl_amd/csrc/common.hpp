// common.hpp -- kernel argument blocks shared by the host runtime and the HIP kernels.
#pragma once
#include <stdint.h>

namespace mcmc {

enum ModelKind : int32_t {
    MK_ISO = 1, MK_NORMAL = 2, MK_LOGISTIC = 3, MK_LINEAR = 4, MK_ABS_NORMAL = 5, MK_DIST = 6, MK_PROBIT = 7,
    MK_DIST_OBS = 8, MK_OU = 9
};
// MK_DIST: v ~ Dist(p1, p2) elementwise (MCMCDerivRules.jl:56-104, the DSL's continuous distributions)
enum DistKind : int32_t {
    DK_NORMAL = 1, DK_UNIFORM = 2, DK_WEIBULL = 3, DK_BETA = 4, DK_TDIST = 5, DK_EXPONENTIAL = 6, DK_GAMMA = 7,
    DK_CAUCHY = 8, DK_LOGNORMAL = 9, DK_LAPLACE = 10
};
enum SamplerKind : int32_t { SK_RWM = 1, SK_MALA = 2, SK_HMC = 3, SK_HMCDA = 4, SK_RAM = 5 };

// Model parameters as the kernels see them (device pointers).
struct ModelArgs {
    int32_t kind;
    int32_t d;
    double mu, sigma;           // NORMAL_DSL, ABS_NORMAL_DSL; DIST: the two parameters p1, p2
    int32_t dist;               // DIST: DistKind
    double dconst;              // DIST: host-computed constant of the logpdf (lgamma terms etc.)
    double prior_sigma;         // regression prior
    double noise_sigma;         // LINEAR
    double link_sign;           // LOGISTIC
    int64_t n;                  // observations
    int64_t n_pad;              // observations padded to the MFMA tile
    const double* X;            // regression: the staged-tile image of X and Y (glm_layout.hpp)
    const double* Y;            // [n_pad]
    const double* init;         // [d]
};

// Sampler constants (uniform across chains).
struct SamplerArgs {
    int32_t kind;
    int32_t tuner;              // EmpMCTuner on/off
    double scale;               // RWM
    double drift_step;          // MALA
    int64_t n_leaps;            // HMC
    double leap_step;           // HMC
    double rate, len, shrinkage, t0, step;  // HMCDA
    int64_t adapt_step, max_step;
    double target_path, target_rate;
    int64_t max_leaps;
};

// Per-chain sampler state (SoA, length ld).  Which arrays are live depends on the sampler.
struct ChainState {
    double* x;                  // [d][ld]  (lane-per-chain layout)   or [C][d] (wave-per-chain layout)
    double* lp;                 // [ld]
    double* g;                  // [d][ld] gradient at x (regression models only; separable models recompute)
    double* t_step;             // MALA driftStep | HMC leapStep | HMCDA leapStep
    double* t_bar;              // HMCDA dualLeapStep
    double* t_h;                // HMCDA dualH
    int32_t* t_leaps;           // HMC tuned nLeaps
    int32_t* t_acc;             // tuner accepted counter
    int32_t* t_prop;            // tuner proposed counter
    double* mom;                // regression HMC / HMCDA on d-slices (d > 128): the momentum parked in HBM across each
                                //   evaluation [d_pad][ld] (glm.hip glm_hmc), so the MFMA loop keeps its registers
    double* ram_L;              // RAM: jump factor S, two halves of packed padded rows [dpad(dpad+1)/2][ram_ld]
    int64_t ram_ld;             // RAM: lane-per-chain: chain stride of ram_L (a multiple of 256); wave-per-chain:
                                //      doubles per chain (ram.hpp wave layout)
    int64_t ram_hs;             // RAM: doubles from the first half of ram_L to the second
};

// One launch of the fused step kernel.
struct StepArgs {
    int64_t C;                  // local chains
    int64_t ld;                 // leading dimension of state arrays (>= C, multiple of 64)
    int32_t d;
    uint32_t chain0;            // global id of local chain 0
    uint32_t key0, key1;        // seed
    int64_t step_begin;         // global (sampler) step index of the first step of this launch, 1-based
    int32_t nsteps;             // steps in this launch
    int64_t run_step0;          // global step index preceding the run's first step (i_loc = i - run_step0)
    int64_t burnin, thinning, len;   // runner range (run-local)
    int64_t tuner_burnin;       // runner.burnin as seen by the sampler loop (global i)
    const double* scale;        // [d] model.scale .* sampler.scale (RWM) or model.scale
    double scale1;              // the common value when every scale[j] is equal (scale_uniform)
    int32_t scale_uniform;
    double* samples;            // [nkept][d][C]  (NULL: not stored)
    double* grads;              // [nkept][d][C]  (NULL: not stored)
    uint64_t* acc_bits;         // [nkept][nw]
    int64_t nw;                 // words per kept step = ceil(C/64)
    int32_t* err;               // device error word
    unsigned long long* n_evals;  // running count of log-target evaluations over all chains (NULL: off)
    const int32_t* order;       // regression HMC / HMCDA: chain slot -> local chain (NULL: identity), so that a
                                // 16-chain MFMA tile holds chains of similar trajectory length
};

// storeLeaps record of one kept step (HMC.jl:145-150): device pointers already offset to that step;
// pars / grads / mom [cap+1][d][C], lp / H [cap+1][C], nl [C]
struct LeapRec {
    int64_t cap;
    double* pars;
    double* grads;
    double* mom;
    double* lp;
    double* H;
    int32_t* nl;
};

__host__ __device__ inline bool kept_index(int64_t i_loc, int64_t burnin, int64_t thinning, int64_t len,
                                           int64_t* kk) {
    if (i_loc <= burnin || i_loc > len) return false;
    const int64_t off = i_loc - burnin - 1;
    if (off % thinning != 0) return false;
    *kk = off / thinning;
    return true;
}

}  // namespace mcmc
