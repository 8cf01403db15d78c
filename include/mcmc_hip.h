/*
 * mcmc_hip.h -- C ABI of the MI355X (gfx950) many-chain MCMC inner loop.
 *
 * Drop-in boundary for MCMC.jl's model x sampler x runner hot path
 * (reference: /root/reference, Julia 0.2).  Plain C types only: int32/int64,
 * double*, uint64_t*; no torch, no C++ in the signatures.  A Julia host binds
 * these with `ccall` (INTEGRATION.md shows the binding); the in-tree host is
 * Python/ctypes (mcmc.jl_amd/mcmchip).
 *
 *   reference interface                              replaced by
 *   -----------------------------------------------  -------------------------------------------
 *   model(f; init, grad, scale)      mcmcmodels.jl:27-33,   mcmc_model_create (catalogue kind, init,
 *     MCMCLikelihoodModel ctor        likmodel.jl:100-143    scale, data X/Y)
 *   RWM / MALA / HMC / HMCDA ctors   RWM.jl:24-36,          mcmc_sampler_cfg (validated like the
 *                                    MALA.jl:50-62,         reference @asserts: mcmc_sampler_validate)
 *                                    HMC.jl:53-74,
 *                                    HMCDA.jl:24-43
 *   EmpMCTuner                       samplers.jl:32-50      mcmc_sampler_cfg.tuner_*
 *   SerialMC(steps,burnin,thinning)  SerialMC.jl:12-35      mcmc_runner_cfg
 *   m * s * r -> MCMCTask (spinTask) MCMC.jl:87-98,         mcmc_chains_create (a batch of C
 *                                    samplers.jl:53          independent MCMCTasks: one per chain)
 *   run(t::MCMCTask) / run_serialmc  runners.jl:7-11,45,    mcmc_run_serialmc
 *                                    SerialMC.jl:37-85
 *   run(c::MCMCChain) (continue)     runners.jl:14          mcmc_run_serialmc again on the same chains
 *   resume(c; steps)                 SerialMC.jl:93-97      a new batch (mcmc_chains_create) on fresh global
 *                                                           chain ids + mcmc_run_serialmc
 *   MCMCChain fields                 MCMC.jl:58-80          mcmc_outputs (samples, gradients,
 *                                                           accept bits, runtime)
 *   acceptance(chain)                summary.jl:6-15        computed by the host from accept bits
 *
 * Errors: every call returns an int status (MCMC_OK = 0) and sets a
 * thread-local message readable with mcmc_last_error(); the reference's
 * @assert texts are reproduced verbatim where one exists.
 *
 * Threading: one host thread drives a context; calls on one context are not
 * re-entrant; distinct contexts are independent and may be driven from
 * different host threads at once (also on one GPU).  mcmc_group_* drives
 * several GPUs from one host thread (library worker threads per device).  Ownership: the caller owns
 * every output buffer; the library owns device state inside ctx/model/chains
 * and never keeps a caller pointer after a call returns.
 */
#ifndef MCMC_HIP_H
#define MCMC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCMC_ABI_VERSION 1

/* status codes */
enum {
    MCMC_OK = 0,
    MCMC_E_INVALID_ARG = 1,          /* a reference @assert failed, or a NULL/size error            */
    MCMC_E_INIT_OUT_OF_SUPPORT = 2,  /* "Initial values out of model support, try other values"    */
    MCMC_E_NEEDS_GRADIENT = 3,       /* "<S> sampler requires model with gradient function"         */
    MCMC_E_HIP = 4,                  /* a HIP runtime call failed                                   */
    MCMC_E_OOM = 5,                  /* device allocation failed                                    */
    MCMC_E_UNSUPPORTED = 6           /* model x sampler x size combination not built                */
};

/* model catalogue (Julia closures cannot cross a C ABI) */
enum {
    MCMC_MODEL_ISO_NORMAL_DOT = 1,   /* model(v -> -dot(v,v), grad = v -> -2v)   README.md:60,63      */
    MCMC_MODEL_NORMAL_DSL = 2,       /* model(:(v ~ Normal(mu, sigma)), gradient=true)  README.md:67-72 */
    MCMC_MODEL_LOGISTIC = 3,         /* examples/logistic_regression.jl:16-22 (DSL, gradient=true)   */
    MCMC_MODEL_LINEAR = 4,           /* examples/linear_regression.jl:14-20  (DSL, gradient=true)    */
    MCMC_MODEL_ABS_NORMAL_DSL = 5,   /* model(:(y = abs(x); y ~ Normal(mu, sigma)))  README.md:246-251 */
    MCMC_MODEL_DIST_DSL = 6,         /* model(:(v ~ Dist(p1, p2))): dist = MCMC_DIST_*, p1 = mu, p2 = sigma */
    MCMC_MODEL_PROBIT = 7,           /* examples/probit_regression.jl:18-40: log-prior MvNormal(0, prior_sigma^2 I)
                                        + dot(logcdf(N, X pars), Y) + dot(logcdf(N, -X pars), 1 - Y), Y 0.0 / 1.0 */
    MCMC_MODEL_DIST_OBS = 8,         /* model(:(y = x * v; y ~ Dist(p1, p2))), benchmarks/benchunits/bare_distribs.jl:13:
                                        scalar x (d = 1), data v = Y [n]; dist / mu / sigma as MCMC_MODEL_DIST_DSL */
    MCMC_MODEL_OU = 9                /* examples/ornstein.jl:19-30: pars (tau, sigma, mu) (d = 3), the series x = Y [n],
                                        n >= 2: tau ~ Uniform(0,100), sigma ~ Uniform(0,2), mu ~ Uniform(0,20),
                                        resid = x[2:end] - x[1:end-1] exp(-1/tau) - mu (1 - exp(-1/tau)) ~ Normal(0, sigma) */
};

/* distributions of MCMC_MODEL_DIST_DSL: the DSL's continuous logpdf rules, MCMCDerivRules.jl:56-104
   (Distributions.jl parametrisations) */
enum {
    MCMC_DIST_NORMAL = 1,       /* Normal(mu, sigma)          */
    MCMC_DIST_UNIFORM = 2,      /* Uniform(a, b)              */
    MCMC_DIST_WEIBULL = 3,      /* Weibull(shape, scale)      */
    MCMC_DIST_BETA = 4,         /* Beta(alpha, beta)          */
    MCMC_DIST_TDIST = 5,        /* TDist(df)     (p2 unused)  */
    MCMC_DIST_EXPONENTIAL = 6,  /* Exponential(scale)         */
    MCMC_DIST_GAMMA = 7,        /* Gamma(shape, scale)        */
    MCMC_DIST_CAUCHY = 8,       /* Cauchy(location, scale)    */
    MCMC_DIST_LOGNORMAL = 9,    /* LogNormal(meanlog, sdlog)  */
    MCMC_DIST_LAPLACE = 10      /* Laplace(location, scale)   */
};

/* samplers */
enum { MCMC_RWM = 1, MCMC_MALA = 2, MCMC_HMC = 3, MCMC_HMCDA = 4, MCMC_RAM = 5 };

typedef struct mcmc_ctx mcmc_ctx;
typedef struct mcmc_model mcmc_model;
typedef struct mcmc_chains mcmc_chains;

typedef struct {
    int32_t kind;            /* MCMC_MODEL_*                                                     */
    int32_t has_gradient;    /* 0: eval only (hasgradient(model) == false, mcmcmodels.jl:19)      */
    int64_t d;               /* parameter vector size (model.size)                               */
    const double* init;      /* [d]  model.init                                                  */
    const double* scale;     /* [d]  model.scale (NULL -> ones)                                   */
    double mu, sigma;        /* NORMAL_DSL, ABS_NORMAL_DSL: Normal(mu, sigma)                     */
    double prior_sigma;      /* LOGISTIC/LINEAR: vars ~ Normal(0, prior_sigma)                    */
    double noise_sigma;      /* LINEAR: resid ~ Normal(0, noise_sigma)                             */
    double link_sign;        /* LOGISTIC: +1 -> prob = 1/(1+exp(-X*vars)) (example),
                                          -1 -> prob = 1/(1+exp(+X*vars)) (test/test_syntax.jl:13) */
    int64_t n;               /* observations                                                      */
    const double* X;         /* [n][d] row-major covariates                                        */
    const double* Y;         /* [n] responses (LOGISTIC: 0.0 / 1.0)                                */
    int32_t dist;            /* DIST_DSL: MCMC_DIST_* (parameters in mu, sigma)                     */
} mcmc_model_desc;

typedef struct {
    int32_t kind;            /* MCMC_RWM | MCMC_MALA | MCMC_HMC | MCMC_HMCDA | MCMC_RAM           */
    double scale;            /* RWM, RAM: scale (RWM.jl:25, RAM.jl:23)                             */
    double drift_step;       /* MALA: driftStep (MALA.jl:51)                                       */
    int64_t n_leaps;         /* HMC: nLeaps (HMC.jl:54)                                            */
    double leap_step;        /* HMC: leapStep (HMC.jl:55)                                          */
    double rate, len, shrinkage, t0, step;   /* HMCDA (HMCDA.jl:25-29); rate: RAM target rate (RAM.jl:24) */
    int32_t tuner;           /* 0: nothing; 1: EmpiricalMCMCTuner (MALA, HMC)                      */
    int64_t adapt_step, max_step;            /* EmpMCTuner (samplers.jl:33-37)                      */
    double target_path, target_rate;
    int64_t max_leaps;       /* HMCDA/HMC-tuner safety cap on leapfrogs per step (0 -> 1<<20)      */
} mcmc_sampler_cfg;

typedef struct {
    int64_t burnin;          /* SerialMC.burnin                                                    */
    int64_t thinning;        /* SerialMC.thinning                                                  */
    int64_t len;             /* SerialMC.len: steps consumed per run                              */
} mcmc_runner_cfg;

/* Output buffers.  Any pointer may be NULL (not wanted).  Layouts:
 *   samples, gradients : [nkept][d][nchains]   (MCMCChain.samples / .gradients, per chain c:
 *                                              samples[j][:, c] is row j of its DataFrame)
 *   accept_bits        : [nkept][ceil(nchains/64)]  bit (c % 64) of word c/64 = diagnostics["accept"][j]
 *   final_x            : [d][nchains]          state after the run
 *   final_lp           : [nchains]
 * nkept = length((burnin+1):thinning:len).  on_device != 0 means every pointer is a
 * device pointer on the context's GPU (e.g. torch tensors): nothing crosses PCIe. */
typedef struct {
    double* samples;
    double* gradients;
    uint64_t* accept_bits;
    double* final_x;
    double* final_lp;
    int32_t on_device;
    double runtime_s;        /* out: wall time of the step loop (MCMCChain.runTime, SerialMC.jl:38,84) */
    double kernel_ms;        /* out: device time of the step kernels (HIP events)                     */
    int64_t nkept;           /* out */
} mcmc_outputs;

/* ---- library ---- */
const char* mcmc_last_error(void);
int mcmc_abi_version(void);
int mcmc_device_count(int* count);

/* ---- context: one GPU, one stream ---- */
int mcmc_ctx_create(int device, mcmc_ctx** out);
int mcmc_ctx_destroy(mcmc_ctx* ctx);
int mcmc_ctx_synchronize(mcmc_ctx* ctx);

/* ---- model: uploads init/scale/X/Y once (model data is replicated per GPU) ---- */
int mcmc_model_create(mcmc_ctx* ctx, const mcmc_model_desc* desc, mcmc_model** out);
int mcmc_model_destroy(mcmc_model* model);
/* evaluate log-target (and gradient) of `nchains` parameter vectors x[d][nchains] on the device
 * (model.eval / model.evalallg, likmodel.jl:21,25); host pointers. grad may be NULL. */
int mcmc_model_eval(mcmc_model* model, int64_t nchains, const double* x, double* lp, double* grad);

/* ---- sampler config validation (the reference constructors' @asserts) ---- */
int mcmc_sampler_validate(const mcmc_sampler_cfg* cfg);
int mcmc_runner_validate(const mcmc_runner_cfg* cfg);

/* ---- chains: C independent MCMCTasks of one (model, sampler) on one GPU ----
 * chain_offset = global id of local chain 0 (multi-GPU sharding): the random
 * stream is keyed by (seed, global chain, global step), so results do not
 * depend on the number of GPUs.  init_x: optional per-chain start [d][nchains]
 * (NULL -> every chain starts at model.init, RWM.jl:53).  Sizes built: d <= 16384 for the separable
 * models, d <= 1024 for the regression models; RAM d <= 1024 (separable and regression), else
 * MCMC_E_UNSUPPORTED. */
int mcmc_chains_create(mcmc_model* model, const mcmc_sampler_cfg* sampler, int64_t nchains,
                       int64_t chain_offset, uint64_t seed, const double* init_x, mcmc_chains** out);
int mcmc_chains_destroy(mcmc_chains* chains);
/* restart from model.init (resume(), SerialMC.jl:93-97): step counter back to 0. */
int mcmc_chains_reset(mcmc_chains* chains);
/* MCMC.reset(t, x) (src/MCMC.jl:39; the samplers' task-local :reset hooks, RWM.jl:49, MALA.jl:75-80, HMC.jl:114-116,
 * HMCDA.jl:82-83, RAM.jl:47): every chain's position := x (host [d][nchains]) and its log-target (and gradient)
 * re-evaluated there; lp (may be NULL) receives the log-targets [nchains].  The step counter, tuner state and RAM
 * factor are kept.  Used by SeqMC-style drivers (SeqMC.jl:68-69) that move particles between tasks. */
int mcmc_chains_set_state(mcmc_chains* chains, const double* x, double* lp);
/* chains [first, first + count) of src as a new, independent batch (same model, sampler and seed; global chain ids
 * src's + first) holding a copy of their whole state and step counter, so that running it continues exactly those
 * chains whatever src does next.  No reference counterpart beyond run(c::MCMCChain) = run(c.task) (runners.jl:14):
 * after one batched run of an Array{MCMCTask}, each returned chain's task continues its own chain. */
int mcmc_chains_fork(mcmc_chains* src, int64_t first, int64_t count, mcmc_chains** out);
/* steps consumed so far (the sampler's own loop counter i). */
int mcmc_chains_steps_done(mcmc_chains* chains, int64_t* steps);
/* per-chain adaptive state after the last run, [nchains] each (any may be NULL): step = the current step size
 * (MALA driftStep under EmpiricalMALATune, HMC leapStep under EmpiricalHMCTune, HMCDA leapStep, HMCDA.jl:136,140);
 * step_bar = HMCDA's dual-averaged dualLeapStep (HMCDA.jl:138); nleaps = the tuned HMC nLeaps (HMC.jl:42).
 * A quantity the sampler does not adapt reads NaN (steps) or 0 (nleaps). */
int mcmc_chains_tuner_state(mcmc_chains* chains, double* step, double* step_bar, int32_t* nleaps);
/* log-target evaluations (with gradient for MALA/HMC/HMCDA) summed over all chains since
 * create/reset: steps x C for RWM/MALA, the leapfrog count for HMC/HMCDA (HMC.jl:93-102),
 * whose trajectory length varies per chain under HMCDA / EmpMCTuner. */
int mcmc_chains_evals(mcmc_chains* chains, int64_t* evals);
/* RAM: the current jump factor S of every chain (RAM.jl:55, :78), lower triangle packed by rows:
 * element (r, c), c <= r, of chain k at S[(r(r+1)/2 + c) * nchains + k]; host buffer of
 * d(d+1)/2 * nchains doubles.  MCMC_E_INVALID_ARG for other samplers. */
int mcmc_chains_ram_factor(mcmc_chains* chains, double* S);
/* steps fused per kernel launch (0 = whole run in one launch, the default). */
int mcmc_chains_set_steps_per_launch(mcmc_chains* chains, int64_t steps_per_launch);
/* The burnin the samplers' adaptation sees, apart from the kept range of mcmc_run_serialmc.  The reference's
 * tuners read the task's own runner: EmpiricalMALATune / EmpiricalHMCTune adapt while i <= runner.burnin
 * (MALA.jl:116, HMC.jl:167) and HMCDA dual-averages while i < runner.burnin (HMCDA.jl:133-141), i the sampler's
 * step counter.  A host that keeps every step of a run and applies the kept range itself (a Julia Task producing
 * one MCMCSample per consume, in chunks: julia/mcmc_jl_hook.jl) sets the task runner's burnin here.  -1 (the
 * default): each run's own runner->burnin.  Copied by mcmc_chains_fork. */
int mcmc_chains_set_tuner_burnin(mcmc_chains* chains, int64_t burnin);
/* store gradients of kept samples for gradient samplers (default 1, SerialMC.jl:51-53) */
int mcmc_chains_set_store_gradients(mcmc_chains* chains, int32_t store);
/* pre-size the library's own output buffers for runs keeping up to nkept steps (staging of the
 * wave-per-chain layout; device copies when on_device == 0), so that mcmc_run_serialmc allocates
 * nothing (no reference counterpart: the Julia runner grows its DataFrame per run, SerialMC.jl:39-42). */
int mcmc_chains_reserve_outputs(mcmc_chains* chains, int64_t nkept, int32_t on_device);
/* kernel launches a run of len steps takes (steps per launch as set, capped by kernels that fuse a
 * bounded number of steps); for timing per launch. */
int mcmc_chains_launches(mcmc_chains* chains, int64_t len, int64_t* launches);
/* the step kernel instance the last mcmc_run_serialmc launched, e.g. "lpc_rwm<8, true, IsoDot, true>"
 * (the template instance rocprofv3 names, without the namespace), NUL-terminated into buf[cap];
 * "" before the first run.  No reference counterpart: lets tests and benchmarks check which
 * specialisation ran. */
int mcmc_chains_step_kernel(mcmc_chains* chains, char* buf, int64_t cap);

/* storeLeaps (HMC.jl:145-150, HMCDA.jl:110-117; HMC and HMCDA only).  The next mcmc_run_serialmc records, for
 * every kept step, the states of its trajectory -- leap 0 = state0 after update!, leap l = the state after
 * the l-th leapfrog, l <= min(nLeaps, cap) -- into host buffers: pars, grads, mom [nkept][cap+1][d][C];
 * lp, H [nkept][cap+1][C] (NaN past nLeaps); nleaps [nkept][C] (the full nLeaps, also when above cap).
 * That run takes one step per launch.  pars == NULL switches it off; one run consumes the registration. */
int mcmc_chains_store_leaps(mcmc_chains* chains, int64_t cap, double* pars, double* grads, double* mom, double* lp,
                            double* H, int32_t* nleaps);

/* run_serialmc: consume runner->len steps, keep (burnin+1):thinning:len. */
int mcmc_run_serialmc(mcmc_chains* chains, const mcmc_runner_cfg* runner, mcmc_outputs* out);

/* ---- one node's GPUs driven by one host thread (SURVEY.md §8(b),(e)) ----
 * Replaces the reference's only parallel path, prun -> pmap of independent tasks over worker processes
 * (src/runners/runners.jl:35-42, examples/parallel_serialmc.jl:1-8): one batch of nchains chains is split
 * into contiguous blocks of whole 64-chain groups, block g on devices[g] (mcmc_group_plan).  Every block
 * keys its random streams by global chain id (chain_offset + its first chain), so the results are
 * bit-identical to one context running all chains, for any device list.  A run launches every block's step
 * loop concurrently (one library worker thread per block, each with its own context and stream; no
 * collective inside the step loop), then gathers each block's outputs device -> host straight into the
 * caller's [nkept][d][nchains] buffers (a strided copy per GPU over that GPU's own host link: the end
 * gather of MCMCChain assembly, timed apart).  A device may be listed more than once (several blocks on one
 * GPU).  Outputs of a group run are host buffers (on_device must be 0). */
typedef struct mcmc_group mcmc_group;
typedef struct mcmc_group_chains mcmc_group_chains;
int mcmc_group_create(const int32_t* devices, int32_t ndevices, mcmc_group** out);
int mcmc_group_destroy(mcmc_group* group);     /* after every mcmc_group_chains of it is destroyed */
int mcmc_group_size(mcmc_group* group, int32_t* ndevices);
/* the block of every device: block g = chains [first[g], first[g] + count[g]); blocks of ceil(nchains /
 * nblocks) rounded up to a multiple of 64 chains, so trailing blocks may be short or empty (count 0).
 * Host-only arithmetic (no device needed). */
int mcmc_group_plan(int64_t nchains, int32_t nblocks, int64_t* first, int64_t* count);
/* model (replicated: uploaded once per device), sampler and chains on every device; init_x: optional
 * [d][nchains] host array (NULL -> model.init) */
int mcmc_group_chains_create(mcmc_group* group, const mcmc_model_desc* model, const mcmc_sampler_cfg* sampler,
                             int64_t nchains, int64_t chain_offset, uint64_t seed, const double* init_x,
                             mcmc_group_chains** out);
int mcmc_group_chains_destroy(mcmc_group_chains* gc);
int mcmc_group_chains_reset(mcmc_group_chains* gc);                       /* resume(): every block */
int mcmc_group_chains_steps_done(mcmc_group_chains* gc, int64_t* steps);
int mcmc_group_chains_set_steps_per_launch(mcmc_group_chains* gc, int64_t steps_per_launch);
/* block g's chains (NULL when the block is empty) and its first chain / chain count; the block's
 * mcmc_chains may be queried (evals, step kernel, RAM factor) but not run or destroyed on its own */
int mcmc_group_chains_block(mcmc_group_chains* gc, int32_t g, mcmc_chains** chains, int64_t* first,
                            int64_t* count);
/* run_serialmc on every block concurrently; out holds host buffers for all nchains chains (mcmc_outputs
 * layout); out->runtime_s / kernel_ms: the slowest block's step loop; gather_s (may be NULL): the slowest
 * block's device -> host gather of its outputs.  Output buffers that are not already page-locked are
 * registered (hipHostRegister, portable) for the duration of the call, so the gather is direct DMA; callers
 * that run repeatedly into the same buffers can pin them once themselves.  If any block fails, the error
 * names the block and device, and these chains refuse further runs (and steps_done) until
 * mcmc_group_chains_reset: the blocks may then be at different steps. */
int mcmc_group_run_serialmc(mcmc_group_chains* gc, const mcmc_runner_cfg* runner, mcmc_outputs* out,
                            double* gather_s);
/* the last mcmc_group_run_serialmc's page-locking of the caller's output buffers (hipHostRegister before,
 * hipHostUnregister after; 0 when they were pinned already), in seconds.  It is not part of gather_s, which
 * times the copies alone: a caller that runs once into fresh pageable buffers pays both. */
int mcmc_group_last_pin_s(const mcmc_group_chains* gc, double* pin_s);
/* test hook: the next mcmc_group_run_serialmc fails block `block` before it starts (the others run) */
int mcmc_debug_group_inject_failure(mcmc_group_chains* gc, int32_t block);

/* ---- SeqMC population runner (src/runners/SeqMC.jl:21-122) ----
 * targets[t] (t < ntargets) are chain batches of one context, equal d, each with nchains == npart:
 * particle n is chain n of every target.  Per outer step i = 1..steps and target t: every particle is
 * reset into target t (state = particle, lp = eval: MCMC.reset, MCMC.jl:39) and advanced one step of
 * its sampler; logW += lp_t(reset) - logtarget; logtarget = lp after the step; when var(exp(logW)) <
 * trigger the particles are resampled multinomially from cumsum(W)/sum(W) (one Philox uniform of
 * (particle, i, t, tag 2) under `seed`) and logW = 0.  After each outer step logtarget = 0, and for
 * i > burnin the particles and exp(logW) are stored.
 *   particles : [d][npart] start values (SeqMC.jl:43 `particles`)
 *   samples   : [steps-burnin][d][npart]   (row i-burnin-1: the particles after outer step i)
 *   weights   : [steps-burnin][npart]      (diagnostics["weigths"])
 *   resampled : [steps][ntargets] int32 flags, or NULL
 * on_device != 0: particles/samples/weights/resampled are device pointers on the context's GPU. */
typedef struct {
    int64_t steps;           /* SeqMC.steps   (SeqMC.jl:24)                                          */
    int64_t burnin;          /* SeqMC.burnin                                                          */
    double trigger;          /* SeqMC.trigger: resample when var(W) < trigger                        */
} mcmc_seqmc_cfg;
int mcmc_seqmc_validate(const mcmc_seqmc_cfg* cfg);
int mcmc_run_seqmc(mcmc_chains* const* targets, int32_t ntargets, int64_t npart, const double* particles,
                   const mcmc_seqmc_cfg* cfg, uint64_t seed, int32_t on_device, double* samples, double* weights,
                   int32_t* resampled, double* runtime_s);

/* ---- output analysis (src/stats/ess.jl:6-10, var.jl:7-117) ----
 * Effective sample size n * var_iid / var_vtype of every (parameter j, chain c) series of
 * samples [nkept][d][nchains] (the mcmc_outputs layout).  vtype: MCMC_VAR_IMSE (Geyer initial
 * monotone sequence), MCMC_VAR_IPSE (initial positive sequence), MCMC_VAR_BM (batch means of
 * `batchlen`).  maxlag <= 0 -> nkept - 1.  Outputs ess[j][c] and optionally var[j][c] (the vtype
 * variance of the mean).  on_device != 0: every pointer is device memory on ctx's GPU. */
enum { MCMC_VAR_IMSE = 1, MCMC_VAR_IPSE = 2, MCMC_VAR_BM = 3 };
int mcmc_stats_ess(mcmc_ctx* ctx, const double* samples, int64_t nkept, int64_t d, int64_t nchains, int32_t vtype,
                   int64_t maxlag, int64_t batchlen, int32_t on_device, double* ess, double* var);

/* ---- diagnostics used by the parity tests: evaluate the build's deterministic
 *      math on the device.  op: 0 log, 1 exp, 2 sin2pi, 3 cos2pi,
 *      4 sqrt, 5 div(x, y), 6 normals (x = block counters), 7 Julia-0.2 round,
 *      8 accept uniform, 9 Box-Muller radius log, 10/11 Box-Muller angle sin/cos,
 *      12 guard-free sqrt of the Box-Muller radius, 13/14 det_exp_tab / det_log_tab, 15 the screened accept test,
 *      16 the Box-Muller radius^2 -2 log u (bm_rad2_u32, bitwise -2 x op 9), 17 the Box-Muller radius
 *      sqrt(-2 log u) (bm_radius_u32, the segment polynomials), 22 / 23 the logistic Bernoulli term / its
 *      eta-derivative weight of (eta = x, w = y) (det_logi). ---- */
int mcmc_debug_detmath(mcmc_ctx* ctx, int op, int64_t n, const double* x, const double* y, double* out);
int mcmc_debug_philox(mcmc_ctx* ctx, int64_t n, const uint32_t* ctr /*[n][4]*/, const uint32_t* key /*[n][2]*/,
                      uint32_t* out /*[n][4]*/);
/* nk chained v_mfma_f64_16x16x4_f64: D = A[16][4nk] * B[4nk][16] + C[16][16] (row-major, host pointers);
   pins the fp64 MFMA accumulation order the regression kernels rely on. */
int mcmc_debug_mfma_f64(mcmc_ctx* ctx, int nk, const double* A, const double* B, const double* C, double* D);
/* The chain order the last run of `chains` launched with (regression HMC / HMCDA run their chains
   sorted by trajectory length, slot -> local chain): *used = 1 and order[0..C) filled, or *used = 0 (identity). */
int mcmc_debug_chains_order(mcmc_chains* chains, int32_t* used, int32_t* order);

#ifdef __cplusplus
}
#endif
#endif
