// runtime.cpp -- host runtime behind the C ABI (include/mcmc_hip.h).
//
// Owns device contexts, model uploads, per-chain state and the SerialMC step
// loop.  Everything numeric runs in the HIP kernels; the host validates
// arguments (the reference's @asserts), plans launches and moves buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/mcmc_hip.h"
#include "../glm_layout.hpp"
#include "../common.hpp"
#include "internal.hpp"
#include "kernels_api.hpp"

using namespace mcmc;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            return fail(e_ == hipErrorOutOfMemory ? MCMC_E_OOM : MCMC_E_HIP,                   \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                    \
        }                                                                                      \
    } while (0)

extern "C" const char* mcmc_last_error(void) { return g_err.c_str(); }
int mcmc_set_error(int code, const std::string& msg) { return fail(code, msg); }

// the step kernel instance the last launch function on this thread dispatched (kernels_api.hpp)
#include <cstdarg>
static thread_local char g_step_kernel[160];
void mcmc_note_step_kernel(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_step_kernel, sizeof g_step_kernel, fmt, ap);
    va_end(ap);
}
const char* mcmc_last_step_kernel() { return g_step_kernel; }
extern "C" int mcmc_abi_version(void) { return MCMC_ABI_VERSION; }
extern "C" int mcmc_device_count(int* count) {
    if (!count) return fail(MCMC_E_INVALID_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return MCMC_OK;
}

// ------------------------------------------------------------------ objects
struct mcmc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int32_t* d_err = nullptr;
    // a second stream for launch sequences that split a batch in two halves whose kernels bind on different resources
    // (RAM on regression targets: the MFMA eval of one half beside the HBM-bound factor update of the other)
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

struct mcmc_model {
    mcmc_ctx* ctx = nullptr;
    ModelArgs args{};
    int has_gradient = 0;
    std::vector<double> init, scale;
    double* d_init = nullptr;
    double* d_scale = nullptr;
    double* d_X = nullptr;
    double* d_Y = nullptr;
    int chains_alive = 0;            // chains created on this model and not yet destroyed
    bool released = false;           // mcmc_model_destroy called: free when the last chains go
};

enum Layout { LAYOUT_LPC = 0, LAYOUT_WPC = 1, LAYOUT_GLM = 2 };

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct mcmc_chains {
    mcmc_model* model = nullptr;
    mcmc_sampler_cfg cfg{};          // the sampler configuration it was created with (mcmc_chains_fork)
    SamplerArgs sa{};
    int64_t C = 0, ld = 0, offset = 0;
    uint64_t seed = 0;
    Layout layout = LAYOUT_LPC;
    ChainState st{};
    double* d_scale_eff = nullptr;   // model.scale .* sampler.scale (RWM.jl:52)
    std::vector<double> h_scale_eff; // its host copy
    int ram_dpad = 0;                // RAM: padded factor width
    bool ram_wave = false;           // RAM: the factor in the wave-per-chain layout (separable d > 32, regression d > 32)
    bool glm_ram_wave = false;       // RAM on a regression target with d > 32: the split step (glm_ram_wave.hip)
    double *ram_u = nullptr, *ram_nz = nullptr, *xprop = nullptr, *lpp = nullptr;   // ... its buffers
    double scale1 = 0.0;             // its common value when all coordinates agree
    int32_t scale_uniform = 0;
    double* d_init_x = nullptr;      // optional per-chain start, [d][C]
    unsigned long long* d_evals = nullptr;   // log-target evaluations since create/reset (all chains)
    int64_t h_evals = 0;             // ... of the samplers with one evaluation per chain-step, counted here
    int64_t steps_done = 0;
    int64_t spl = 0;                 // steps per launch (0: whole run)
    int store_grads = 1;
    int64_t tuner_burnin = -1;       // the tuners' burnin (mcmc_chains_set_tuner_burnin); -1: the run's runner burnin
    DevBuf out_samples, out_grads, out_bits, out_tmp, stage_samples, stage_grads;
    DevBuf order_buf;                // regression HMC / HMCDA: chain slot -> chain (StepArgs.order)
    std::vector<int32_t> h_order;
    bool last_order = false;         // the last run launched with order_buf (mcmc_debug_chains_order)
    // storeLeaps (HMC.jl:145-150): host buffers the next run fills (h_lpars == NULL: off), device staging
    int64_t leap_cap = 0;
    double *h_lpars = nullptr, *h_lgrads = nullptr, *h_lmom = nullptr, *h_llp = nullptr, *h_lH = nullptr;
    int32_t* h_lnl = nullptr;
    DevBuf leap_buf;
    std::string step_kernel;         // the step kernel instance the last run launched
};

// Transfers are ordered on the context's (non-blocking) stream, after every kernel queued there,
// and waited for before the host buffer is released.
static hipError_t h2d(mcmc_ctx* ctx, void* dst, const void* src, size_t bytes) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
}
static hipError_t d2h(mcmc_ctx* ctx, void* dst, const void* src, size_t bytes) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
}
static hipError_t dzero(mcmc_ctx* ctx, void* dst, size_t bytes) {
    return hipMemsetAsync(dst, 0, bytes, ctx->stream);
}

static int set_device(mcmc_ctx* ctx) {
    HIP_TRY(hipSetDevice(ctx->device));
    return MCMC_OK;
}

template <class T>
static int dmalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) return MCMC_OK;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(MCMC_E_OOM, std::string("hipMalloc(") + std::to_string(count * sizeof(T)) + " B): " +
                                    hipGetErrorString(e));
    }
    return MCMC_OK;
}

static void dfree(void* p) {
    if (p) (void)hipFree(p);
}

static int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return MCMC_OK;
    dfree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    if (bytes == 0) return MCMC_OK;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        b.p = nullptr;
        return fail(MCMC_E_OOM, std::string("hipMalloc(") + std::to_string(bytes) + " B) for outputs: " +
                                    hipGetErrorString(e));
    }
    b.bytes = bytes;
    return MCMC_OK;
}

// ------------------------------------------------------------------ context
extern "C" int mcmc_ctx_create(int device, mcmc_ctx** out) {
    if (!out) return fail(MCMC_E_INVALID_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(MCMC_E_HIP, "no HIP device available");
    if (device < 0 || device >= n) return fail(MCMC_E_INVALID_ARG, "device ordinal out of range");
    auto* c = new mcmc_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_err, sizeof(int32_t));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e != hipSuccess) {
        delete c;
        return fail(MCMC_E_HIP, std::string("context creation: ") + hipGetErrorString(e));
    }
    *out = c;
    return MCMC_OK;
}

extern "C" int mcmc_ctx_destroy(mcmc_ctx* ctx) {
    if (!ctx) return MCMC_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    dfree(ctx->d_err);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return MCMC_OK;
}

extern "C" int mcmc_ctx_synchronize(mcmc_ctx* ctx) {
    if (!ctx) return fail(MCMC_E_INVALID_ARG, "ctx is NULL");
    if (int r = set_device(ctx)) return r;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MCMC_OK;
}

// ------------------------------------------------------------------ validation

extern "C" int mcmc_sampler_validate(const mcmc_sampler_cfg* s) {
    if (!s) return fail(MCMC_E_INVALID_ARG, "sampler cfg is NULL");
    switch (s->kind) {
        case MCMC_RWM:
            if (!(s->scale > 0)) return fail(MCMC_E_INVALID_ARG, "scale should be > 0");               // RWM.jl:29
            if (s->tuner) return fail(MCMC_E_UNSUPPORTED, "RWM has no tuner in the reference (RWMTuner is abstract)");
            break;
        case MCMC_MALA:
            if (!(s->drift_step > 0)) return fail(MCMC_E_INVALID_ARG, "MALA drift step should be > 0"); // MALA.jl:55
            break;
        case MCMC_HMC:
            if (!(s->n_leaps > 0)) return fail(MCMC_E_INVALID_ARG, "inner steps should be > 0");        // HMC.jl:60
            if (!(s->leap_step > 0)) return fail(MCMC_E_INVALID_ARG, "inner steps scaling should be > 0"); // HMC.jl:61
            break;
        case MCMC_RAM: {
            if (!(s->scale > 0)) return fail(MCMC_E_INVALID_ARG, "scale should be > 0");               // RAM.jl:27
            if (!(s->rate > 0.0 && s->rate < 1.0)) {
                char buf[160];
                snprintf(buf, sizeof buf, "target acceptance rate (%g) should be between 0 and 1", s->rate);
                return fail(MCMC_E_INVALID_ARG, buf);                                                    // RAM.jl:28
            }
            if (s->tuner) return fail(MCMC_E_UNSUPPORTED, "RAM takes no tuner");
            break;
        }
        case MCMC_HMCDA: {
            char buf[160];
            if (!(0.0 < s->rate && s->rate < 1.0)) {
                snprintf(buf, sizeof buf, "Target acceptance rate (%g) should be between 0 and 1", s->rate);
                return fail(MCMC_E_INVALID_ARG, buf);                                                    // HMCDA.jl:33
            }
            if (!(s->len > 0)) {
                snprintf(buf, sizeof buf, "len parameter of HMCDA sampler (%g) must be non-negative", s->len);
                return fail(MCMC_E_INVALID_ARG, buf);                                                    // HMCDA.jl:34
            }
            if (!(s->shrinkage > 0)) {
                snprintf(buf, sizeof buf, "shrinkage parameter of HMCDA sampler (%g) must be positive", s->shrinkage);
                return fail(MCMC_E_INVALID_ARG, buf);                                                    // HMCDA.jl:35
            }
            if (!(s->t0 >= 0)) {
                snprintf(buf, sizeof buf, "t0 parameter of HMCDA sampler (%g) must be non-negative", s->t0);
                return fail(MCMC_E_INVALID_ARG, buf);                                                    // HMCDA.jl:36
            }
            if (s->tuner) return fail(MCMC_E_UNSUPPORTED, "HMCDA takes no tuner");
            break;
        }
        default:
            return fail(MCMC_E_UNSUPPORTED, "unknown sampler kind");
    }
    if (s->tuner) {
        char buf[160];
        if (!(s->adapt_step > 0)) {
            snprintf(buf, sizeof buf, "Adaptation step size (%lld) should be > 0", (long long)s->adapt_step);
            return fail(MCMC_E_INVALID_ARG, buf);                                                        // samplers.jl:40
        }
        if (!(s->max_step > 0)) {
            snprintf(buf, sizeof buf, "Adaptation step size (%lld) should be > 0", (long long)s->max_step);
            return fail(MCMC_E_INVALID_ARG, buf);                                                        // samplers.jl:41
        }
        if (!(0.0 < s->target_rate && s->target_rate < 1.0)) {
            snprintf(buf, sizeof buf, "Target acceptance rate (%g) should be between 0 and 1", s->target_rate);
            return fail(MCMC_E_INVALID_ARG, buf);                                                        // samplers.jl:42
        }
    }
    if (s->max_leaps < 0) return fail(MCMC_E_INVALID_ARG, "max_leaps should be >= 0");
    return MCMC_OK;
}

extern "C" int mcmc_runner_validate(const mcmc_runner_cfg* r) {
    if (!r) return fail(MCMC_E_INVALID_ARG, "runner cfg is NULL");
    char buf[160];
    if (!(r->burnin >= 0)) {
        snprintf(buf, sizeof buf, "Burnin rounds (%lld) should be >= 0", (long long)r->burnin);
        return fail(MCMC_E_INVALID_ARG, buf);                                                            // SerialMC.jl:25
    }
    if (!(r->len > r->burnin)) {
        snprintf(buf, sizeof buf, "Total MCMC length (%lld) should be > to burnin (%lld)", (long long)r->len,
                 (long long)r->burnin);
        return fail(MCMC_E_INVALID_ARG, buf);                                                            // SerialMC.jl:26
    }
    if (!(r->thinning >= 1)) {
        snprintf(buf, sizeof buf, "Thinning (%lld) should be >= 1", (long long)r->thinning);
        return fail(MCMC_E_INVALID_ARG, buf);                                                            // SerialMC.jl:27
    }
    if (r->len > 0x7fffffffLL) return fail(MCMC_E_INVALID_ARG, "len exceeds the 2^31 step counter");
    return MCMC_OK;
}

static int64_t nkept_of(const mcmc_runner_cfg& r) {
    if (r.len <= r.burnin) return 0;
    return (r.len - r.burnin - 1) / r.thinning + 1;
}

// ------------------------------------------------------------------ model
extern "C" int mcmc_model_create(mcmc_ctx* ctx, const mcmc_model_desc* desc, mcmc_model** out) {
    if (!ctx || !desc || !out) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (int r = set_device(ctx)) return r;
    const int64_t d = desc->d;
    if (d <= 0) return fail(MCMC_E_INVALID_ARG, "model size d should be > 0");
    if (!desc->init) return fail(MCMC_E_INVALID_ARG, "model init is NULL");
    auto* m = new mcmc_model();
    m->ctx = ctx;
    m->init.assign(desc->init, desc->init + d);
    m->scale.assign((size_t)d, 1.0);
    if (desc->scale) m->scale.assign(desc->scale, desc->scale + d);
    m->has_gradient = desc->has_gradient;
    ModelArgs& a = m->args;
    a.kind = desc->kind;
    a.d = (int32_t)d;
    a.mu = desc->mu;
    a.sigma = desc->sigma;
    a.prior_sigma = desc->prior_sigma;
    a.noise_sigma = desc->noise_sigma;
    a.link_sign = desc->link_sign;
    a.n = 0;
    a.n_pad = 0;
    auto bail = [&](int code) {
        mcmc_model_destroy(m);
        return code;
    };
    switch (desc->kind) {
        case MCMC_MODEL_ISO_NORMAL_DOT:
            break;
        case MCMC_MODEL_NORMAL_DSL:
            if (!(desc->sigma > 0)) return bail(fail(MCMC_E_INVALID_ARG, "Normal sigma should be > 0"));
            break;
        case MCMC_MODEL_ABS_NORMAL_DSL:
            if (!(desc->sigma > 0)) return bail(fail(MCMC_E_INVALID_ARG, "Normal sigma should be > 0"));
            break;
        case MCMC_MODEL_DIST_OBS:
            if (d != 1) return bail(fail(MCMC_E_INVALID_ARG, "y = x * v needs a scalar parameter x (d = 1)"));
            if (desc->n <= 0 || !desc->Y) return bail(fail(MCMC_E_INVALID_ARG, "y = x * v needs the data v (n > 0, Y)"));
            [[fallthrough]];
        case MCMC_MODEL_DIST_DSL: {
            const double p1 = desc->mu, p2 = desc->sigma;
            const double kPi = 3.14159265358979323846;
            double c = 0.0;
            bool ok = true;
            switch (desc->dist) {
                case MCMC_DIST_NORMAL: ok = p2 > 0; c = -std::log(p2); break;
                case MCMC_DIST_UNIFORM: ok = p1 < p2; c = -std::log(p2 - p1); break;
                case MCMC_DIST_WEIBULL: ok = p1 > 0 && p2 > 0; c = std::log(p1 / p2); break;
                case MCMC_DIST_BETA: ok = p1 > 0 && p2 > 0; c = std::lgamma(p1 + p2) - std::lgamma(p1) - std::lgamma(p2); break;
                case MCMC_DIST_TDIST:
                    ok = p1 > 0;
                    c = std::lgamma((p1 + 1.0) / 2.0) - std::lgamma(p1 / 2.0) - 0.5 * std::log(p1 * kPi);
                    break;
                case MCMC_DIST_EXPONENTIAL: ok = p1 > 0; c = -std::log(p1); break;
                case MCMC_DIST_GAMMA: ok = p1 > 0 && p2 > 0; c = -std::lgamma(p1) - p1 * std::log(p2); break;
                case MCMC_DIST_CAUCHY: ok = p2 > 0; c = -std::log(kPi * p2); break;
                case MCMC_DIST_LOGNORMAL: ok = p2 > 0; c = -std::log(p2) - 0.5 * std::log(2.0 * kPi); break;
                case MCMC_DIST_LAPLACE: ok = p2 > 0; c = -std::log(2.0 * p2); break;
                default: return bail(fail(MCMC_E_UNSUPPORTED, "unknown distribution"));
            }
            if (!ok) return bail(fail(MCMC_E_INVALID_ARG, "invalid distribution parameters"));
            a.dist = desc->dist;
            a.dconst = c;
            if (desc->kind == MCMC_MODEL_DIST_OBS) {                    // the data v, read by every chain
                if (int r = dmalloc(&m->d_Y, (size_t)desc->n)) return bail(r);
                if (h2d(ctx, m->d_Y, desc->Y, (size_t)desc->n * 8) != hipSuccess)
                    return bail(fail(MCMC_E_HIP, "model data upload failed"));
                a.n = desc->n;
                a.Y = m->d_Y;
            }
            break;
        }
        case MCMC_MODEL_OU: {
            // examples/ornstein.jl:19-30; the prior part of the LLAcc sum, ((0 + logpdf(Uniform(0, 100), tau)) +
            // logpdf(Uniform(0, 2), sigma)) + logpdf(Uniform(0, 20), mu) inside the support, -log(b - a) each
            if (d != 3) return bail(fail(MCMC_E_INVALID_ARG, "the Ornstein-Uhlenbeck model has 3 parameters (tau, sigma, mu)"));
            if (desc->n < 2 || !desc->Y) return bail(fail(MCMC_E_INVALID_ARG, "the Ornstein-Uhlenbeck model needs a series of n >= 2 values (Y)"));
            a.dconst = ((0.0 + -std::log(100.0)) + -std::log(2.0)) + -std::log(20.0);
            if (int r = dmalloc(&m->d_Y, (size_t)desc->n)) return bail(r);
            if (h2d(ctx, m->d_Y, desc->Y, (size_t)desc->n * 8) != hipSuccess)
                return bail(fail(MCMC_E_HIP, "model data upload failed"));
            a.n = desc->n;
            a.Y = m->d_Y;
            break;
        }
        case MCMC_MODEL_LOGISTIC:
        case MCMC_MODEL_PROBIT:
        case MCMC_MODEL_LINEAR: {
            if (d > mcmc_glm_max_d()) return bail(fail(MCMC_E_UNSUPPORTED, "regression models support d <= 1024"));
            if (desc->n <= 0 || !desc->X || !desc->Y) return bail(fail(MCMC_E_INVALID_ARG, "regression needs n > 0, X, Y"));
            if (!(desc->prior_sigma > 0)) return bail(fail(MCMC_E_INVALID_ARG, "prior sigma should be > 0"));
            if (desc->kind == MCMC_MODEL_LINEAR && !(desc->noise_sigma > 0))
                return bail(fail(MCMC_E_INVALID_ARG, "noise sigma should be > 0"));
            if (desc->kind == MCMC_MODEL_LOGISTIC && !(desc->link_sign == 1.0 || desc->link_sign == -1.0))
                return bail(fail(MCMC_E_INVALID_ARG, "link_sign must be +1 or -1"));
            if (desc->kind == MCMC_MODEL_LOGISTIC || desc->kind == MCMC_MODEL_PROBIT)
                for (int64_t i = 0; i < desc->n; ++i)
                    if (!(desc->Y[i] == 0.0 || desc->Y[i] == 1.0))
                        return bail(fail(MCMC_E_INVALID_ARG, desc->kind == MCMC_MODEL_LOGISTIC
                                                                 ? "logistic responses must be 0 or 1 (Bernoulli)"
                                                                 : "probit responses must be 0 or 1"));
            // the kernels' staged-tile image of X and Y (glm_layout.hpp: 16-row tiles in the LDS layout, Y inside
            // each tile, zero padding), plus Y [n_pad] on its own
            const int64_t n_pad = (desc->n + 15) / 16 * 16;
            std::vector<double> Xp(mcmc_glm_image_doubles((int)d, desc->n)), Yp((size_t)n_pad, 0.0);
            for (int64_t i = 0; i < desc->n * (int64_t)d; ++i)
                if (!std::isfinite(desc->X[i])) return bail(fail(MCMC_E_INVALID_ARG, "X must be finite"));
            for (int64_t i = 0; i < desc->n; ++i)
                if (!std::isfinite(desc->Y[i])) return bail(fail(MCMC_E_INVALID_ARG, "Y must be finite"));
            // The logistic / probit terms clamp |eta| into their tables (det_logi, the normal log-cdf twins), so a
            // NaN eta would not reach LLAcc's non-finite rule as it does in the reference (a NaN term makes the sum
            // NaN and the point out of support, modelparser.jl:64-72).  eta is NaN only when X vars overflows with
            // mixed signs: every partial sum of row i is bounded by |vars|_inf |X_i|_1, and a vars whose prior term
            // is finite has |vars|_inf < sqrt(DBL_MAX) prior_sigma.  Data for which that product can reach 2^1022
            // (rows with L1 norm ~1e154 / prior_sigma) are refused here instead of clamped in the kernels.
            if (desc->kind == MCMC_MODEL_LOGISTIC || desc->kind == MCMC_MODEL_PROBIT) {
                double l1max = 0.0;
                for (int64_t i = 0; i < desc->n; ++i) {
                    double l1 = 0.0;
                    for (int k = 0; k < d; ++k) l1 += std::fabs(desc->X[i * (int64_t)d + k]);
                    l1max = std::max(l1max, l1);
                }
                if (!(l1max * (std::sqrt(DBL_MAX) * desc->prior_sigma) < 0x1p1022))
                    return bail(fail(MCMC_E_UNSUPPORTED, "covariates too large: X * vars can overflow to NaN at a "
                                                         "parameter vector of finite prior density"));
            }
            // the logistic model's tile columns hold w = s (2y - 1) (s the link sign) instead of y and the bounds
            // -T(y) where the reference's p rounds to 1 or 0 (detmath.hpp det_logi, logi_bound)
            std::vector<double> Yw, Bw;
            if (desc->kind == MCMC_MODEL_LOGISTIC) {
                Yw.resize((size_t)desc->n);
                Bw.resize((size_t)desc->n);
                for (int64_t i = 0; i < desc->n; ++i) {
                    Yw[(size_t)i] = desc->Y[i] == 1.0 ? desc->link_sign : -desc->link_sign;
                    Bw[(size_t)i] = mcmc::logi_bound(desc->Y[i]);
                }
            }
            mcmc_glm_pack_image((int)d, desc->n, desc->X, Yw.empty() ? desc->Y : Yw.data(),
                                Bw.empty() ? nullptr : Bw.data(), Xp.data());
            for (int64_t i = 0; i < desc->n; ++i) Yp[(size_t)i] = desc->Y[i];
            if (int r = dmalloc(&m->d_X, Xp.size())) return bail(r);
            if (int r = dmalloc(&m->d_Y, Yp.size())) return bail(r);
            if (h2d(ctx, m->d_X, Xp.data(), Xp.size() * 8) != hipSuccess ||
                h2d(ctx, m->d_Y, Yp.data(), Yp.size() * 8) != hipSuccess)
                return bail(fail(MCMC_E_HIP, "model data upload failed"));
            a.n = desc->n;
            a.n_pad = n_pad;
            a.X = m->d_X;
            a.Y = m->d_Y;
            break;
        }
        default:
            return bail(fail(MCMC_E_UNSUPPORTED, "unknown model kind"));
    }
    if (d > 0x7fffffff) return bail(fail(MCMC_E_INVALID_ARG, "d too large"));
    if (int r = dmalloc(&m->d_init, (size_t)d)) return bail(r);
    if (int r = dmalloc(&m->d_scale, (size_t)d)) return bail(r);
    a.init = m->d_init;
    hipError_t e = h2d(ctx, m->d_init, m->init.data(), (size_t)d * 8);
    if (e == hipSuccess) e = h2d(ctx, m->d_scale, m->scale.data(), (size_t)d * 8);
    if (e != hipSuccess) return bail(fail(MCMC_E_HIP, std::string("model upload: ") + hipGetErrorString(e)));
    // likmodel.jl:54  @assert isfinite(f(i)) "Initial values out of model support, try other values"
    double lp = 0;
    if (int r = mcmc_model_eval(m, 1, m->init.data(), &lp, nullptr)) return bail(r);
    if (!std::isfinite(lp))
        return bail(fail(MCMC_E_INIT_OUT_OF_SUPPORT, "Initial values out of model support, try other values"));
    *out = m;
    return MCMC_OK;
}

static void model_free(mcmc_model* m) {
    (void)hipSetDevice(m->ctx->device);
    dfree(m->d_init);
    dfree(m->d_scale);
    dfree(m->d_X);
    dfree(m->d_Y);
    delete m;
}

// A model outlives its chains: destroying it while chains still use it (garbage-collected hosts
// finalize in any order) only marks it; the last mcmc_chains_destroy frees it.
extern "C" int mcmc_model_destroy(mcmc_model* m) {
    if (!m) return MCMC_OK;
    m->released = true;
    if (m->chains_alive == 0) model_free(m);
    return MCMC_OK;
}

// the lane / wave-per-chain kernel families (the joint OU target runs there too, at its fixed d = 3)
static bool model_is_separable(const mcmc_model* m) {
    return m->args.kind == MK_ISO || m->args.kind == MK_NORMAL || m->args.kind == MK_ABS_NORMAL ||
           m->args.kind == MK_DIST || m->args.kind == MK_DIST_OBS || m->args.kind == MK_OU;
}
static bool model_is_glm(const mcmc_model* m) {
    return m->args.kind == MK_LOGISTIC || m->args.kind == MK_LINEAR || m->args.kind == MK_PROBIT;
}

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// RAM jump factor (ram.hpp): packed lower-triangular rows padded to the kernel's width + a trash row,
// two halves
static size_t ram_nrows(int d) { return (size_t)d * (size_t)(d + 1) / 2; }
// first element of column k in the wave layout's column-major packing (ram.hpp ram_wave_colstart)
static int64_t wave_colstart(int64_t k, int64_t d) { return k * d - k * (k - 1) / 2; }

// State layout of a chain batch: lane-per-chain [d][ld] for d <= 32, wave-per-chain [C][ld] above.
static Layout layout_for(const mcmc_model* m) {
    if (model_is_glm(m)) return LAYOUT_GLM;
    return m->args.d <= mcmc_lpc_max_d() ? LAYOUT_LPC : LAYOUT_WPC;
}
static int64_t ld_for(Layout L, int64_t C, int d) { return L == LAYOUT_WPC ? round_up(d, 4) : round_up(C, 64); }

static KernelArgs base_args(const mcmc_model* m, int64_t C, int64_t ld) {
    KernelArgs a{};
    a.m = m->args;
    a.s.C = C;
    a.s.ld = ld;
    a.s.d = m->args.d;
    a.s.err = m->ctx->d_err;
    a.s.thinning = 1;
    return a;
}

static hipError_t launch_eval(Layout L, const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                              hipStream_t st) {
    if (L == LAYOUT_GLM) return mcmc_launch_glm_eval(a, xin, lp, g, check, st);
    return L == LAYOUT_LPC ? mcmc_launch_lpc_eval(a, xin, lp, g, check, st)
                           : mcmc_launch_wpc_eval(a, xin, lp, g, check, st);
}
static hipError_t launch_record(Layout L, const KernelArgs& a, const LeapRec& r, hipStream_t st) {
    if (L == LAYOUT_GLM) return mcmc_launch_glm_record(a, r, st);
    return L == LAYOUT_LPC ? mcmc_launch_lpc_record(a, r, st) : mcmc_launch_wpc_record(a, r, st);
}
static hipError_t launch_step(Layout L, const KernelArgs& a, hipStream_t st) {
    if (L == LAYOUT_GLM) return mcmc_launch_glm_step(a, st);
    return L == LAYOUT_LPC ? mcmc_launch_lpc_step(a, st) : mcmc_launch_wpc_step(a, st);
}

// [d][C] (stride ldc) <-> state layout
static hipError_t cols_to_state(Layout L, double* state, int64_t ld, const double* cols, int64_t ldc, int d, int64_t C,
                                hipStream_t st) {
    if (L != LAYOUT_WPC) return mcmc_copy_cols(state, ld, cols, ldc, d, C, st);
    // [d][C] -> [C][ld]: transpose of a d x C matrix
    hipError_t e = hipMemsetAsync(state, 0, (size_t)C * ld * 8, st);
    if (e != hipSuccess) return e;
    return mcmc_transpose(state, ld, cols, ldc, 1, d, C, st);
}
static hipError_t state_to_cols(Layout L, double* cols, int64_t ldc, const double* state, int64_t ld, int d, int64_t C,
                                hipStream_t st) {
    if (L != LAYOUT_WPC) return mcmc_copy_cols(cols, ldc, state, ld, d, C, st);
    return mcmc_transpose(cols, ldc, state, ld, 1, C, d, st);
}

extern "C" int mcmc_model_eval(mcmc_model* m, int64_t nchains, const double* x, double* lp, double* grad) {
    if (!m || !x || !lp) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    if (nchains <= 0) return fail(MCMC_E_INVALID_ARG, "nchains should be > 0");
    mcmc_ctx* ctx = m->ctx;
    if (int r = set_device(ctx)) return r;
    const int d = m->args.d;
    if (model_is_separable(m) && d > mcmc_wpc_max_d()) return fail(MCMC_E_UNSUPPORTED, "d > 16384 is not built");
    const Layout L = layout_for(m);
    const int64_t ld = ld_for(L, nchains, d);
    const size_t nst = L != LAYOUT_WPC ? (size_t)d * ld : (size_t)nchains * ld;
    double *dcols = nullptr, *dx = nullptr, *dlp = nullptr, *dg = nullptr;
    hipStream_t st = ctx->stream;
    int rc = MCMC_OK;
    do {
        if ((rc = dmalloc(&dcols, (size_t)d * nchains))) break;
        if ((rc = dmalloc(&dx, nst))) break;
        if ((rc = dmalloc(&dlp, (size_t)nchains))) break;
        if (grad && (rc = dmalloc(&dg, nst))) break;
        hipError_t e = hipMemcpyAsync(dcols, x, (size_t)d * nchains * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = cols_to_state(L, dx, ld, dcols, nchains, d, nchains, st);
        KernelArgs a = base_args(m, nchains, ld);
        if (e == hipSuccess) e = launch_eval(L, a, dx, dlp, dg, 0, st);
        if (e == hipSuccess && grad) e = state_to_cols(L, dcols, nchains, dg, ld, d, nchains, st);
        if (e == hipSuccess) e = hipMemcpyAsync(lp, dlp, (size_t)nchains * 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && grad)
            e = hipMemcpyAsync(grad, dcols, (size_t)d * nchains * 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("model eval: ") + hipGetErrorString(e));
    } while (0);
    (void)hipStreamSynchronize(st);
    dfree(dcols);
    dfree(dx);
    dfree(dlp);
    dfree(dg);
    return rc;
}

// ------------------------------------------------------------------ chains
static void free_state(mcmc_chains* c) {
    ChainState& s = c->st;
    dfree(s.x); dfree(s.lp); dfree(s.g); dfree(s.t_step); dfree(s.t_bar); dfree(s.t_h);
    dfree(s.t_leaps); dfree(s.t_acc); dfree(s.t_prop); dfree(s.ram_L); dfree(s.mom);
    s = ChainState{};
}

// the step kernels of one launch; RAM on a regression target with d > 32 is a sequence of kernels per step
static hipError_t launch_chain_step(const mcmc_chains* c, const KernelArgs& a, hipStream_t st) {
    if (c->glm_ram_wave) {
        const mcmc_ctx* ctx = c->model->ctx;
        return mcmc_launch_glm_ram_wave(a, c->ram_u, c->ram_nz, c->xprop, c->lpp, st,
                                        st == ctx->stream ? ctx->stream2 : nullptr, ctx->ev_fork, ctx->ev_join);
    }
    return launch_step(c->layout, a, st);
}

// RWM, MALA and RAM evaluate the log-target once per chain-step, so a launch of n steps adds C n evaluations:
// counted on the host.  The step kernels count only where the count is data-dependent (HMC / HMCDA trajectories):
// one device-scope atomic per wave on a single address serialises at the memory side (32 768 of them per 2^20-chain
// launch of the pair kernel, ~10 ns apart) and held a short launch's tail for hundreds of microseconds.
static bool evals_on_host(const mcmc_chains* c) {
    return c->sa.kind == SK_RWM || c->sa.kind == SK_MALA || c->sa.kind == SK_RAM;
}

// Regression HMC / HMCDA: the chains' order for the next run, longest trajectory first.  A 16-chain MFMA tile runs
// its leapfrog loop to the longest trajectory among its chains (glm_hmc's glm_max), and an HMCDA chain's length
// round(len / leapStep) follows its own adapted leapStep (config 5: 240 to 384 leapfrogs a step), so tiles of
// arbitrary chains idle on ~10% of their leapfrogs; sorted, a tile's chains take (nearly) the same number, and the
// longest tiles are dispatched first.  Bitwise neutral: a tile's MFMA columns are independent chains, and every
// chain-indexed access goes through the permutation (glm.hip glm_pos).  The key is the state the run starts from:
// the current leapStep (HMCDA; smaller is longer, NaN last) or the tuned nLeaps (HMC).
static int glm_trajectory_order(mcmc_chains* c, hipStream_t st) {
    mcmc_ctx* ctx = c->model->ctx;
    const int64_t C = c->C;
    if (int rc = ensure(c->order_buf, (size_t)C * sizeof(int32_t))) return rc;
    std::vector<double> key((size_t)C);
    if (c->sa.kind == SK_HMCDA) {
        HIP_TRY(d2h(ctx, key.data(), c->st.t_step, (size_t)C * sizeof(double)));
    } else {
        std::vector<int32_t> nl((size_t)C);
        HIP_TRY(d2h(ctx, nl.data(), c->st.t_leaps, (size_t)C * sizeof(int32_t)));
        for (int64_t i = 0; i < C; ++i) key[(size_t)i] = -(double)nl[(size_t)i];
    }
    c->h_order.resize((size_t)C);
    for (int64_t i = 0; i < C; ++i) c->h_order[(size_t)i] = (int32_t)i;
    std::stable_sort(c->h_order.begin(), c->h_order.end(), [&](int32_t a, int32_t b) {
        const double ka = key[(size_t)a], kb = key[(size_t)b];
        const bool na = std::isnan(ka), nb = std::isnan(kb);
        return na != nb ? nb : (!na && ka < kb);
    });
    // two tiles a workgroup (d-sliced, 128 < d <= 512): the longest tile shares its workgroup with the shortest, the
    // second longest with the second shortest, ...: the workgroup runs its longer tile's trajectory, and once the
    // shorter tile's chains have all finished it stops computing (glm_hmc, GLM_TILE_SKIP), so the long tiles -- the
    // dispatch's end -- run their tails with the SIMDs to themselves.  Whole 32-chain workgroups only.
    static const bool pair_off = [] {                  // MCMCHIP_TILE_PAIR=0: sorted neighbours share (A/B)
        const char* e = std::getenv("MCMCHIP_TILE_PAIR");
        return e != nullptr && e[0] == '0';
    }();
    if (!pair_off && mcmc_glm_tiles_per_wg(c->model->args.d) == 2 && C % 32 == 0) {
        const int64_t nt = C / 16;
        std::vector<int32_t> paired((size_t)C);
        for (int64_t w = 0; w < nt / 2; ++w)
            for (int h = 0; h < 2; ++h) {
                const int64_t src = h == 0 ? w : nt - 1 - w;             // sorted tile
                for (int k = 0; k < 16; ++k)
                    paired[(size_t)((2 * w + h) * 16 + k)] = c->h_order[(size_t)(src * 16 + k)];
            }
        c->h_order.swap(paired);
    }
    HIP_TRY(hipMemcpyAsync(c->order_buf.p, c->h_order.data(), (size_t)C * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MCMC_OK;
}

// Put every chain at its start and reset the sampler's state (SamplerTask initialisation).
static int init_state(mcmc_chains* c) {
    mcmc_model* m = c->model;
    mcmc_ctx* ctx = m->ctx;
    const int d = m->args.d;
    const SamplerArgs& sa = c->sa;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipMemsetAsync(ctx->d_err, 0, sizeof(int32_t), st));
    HIP_TRY(hipMemsetAsync(c->d_evals, 0, sizeof(unsigned long long), st));
    c->h_evals = 0;
    if (c->d_init_x) {
        HIP_TRY(cols_to_state(c->layout, c->st.x, c->ld, c->d_init_x, c->C, d, c->C, st));
    } else if (c->layout == LAYOUT_WPC) {       // chain-major [C][ld]
        HIP_TRY(mcmc_broadcast_rows(c->st.x, c->ld, m->d_init, d, c->C, st));
    } else {                                    // coordinate-major [d][ld] (LPC, GLM)
        HIP_TRY(mcmc_broadcast_cols(c->st.x, c->ld, m->d_init, d, c->C, st));
    }
    KernelArgs a = base_args(m, c->C, c->ld);
    HIP_TRY(launch_eval(c->layout, a, c->st.x, c->st.lp, c->st.g, 1, st));
    if (sa.kind == SK_MALA && sa.tuner) HIP_TRY(mcmc_fill_f64(c->st.t_step, c->C, sa.drift_step, st));
    if (sa.kind == SK_HMC && sa.tuner) {
        HIP_TRY(mcmc_fill_f64(c->st.t_step, c->C, sa.leap_step, st));
        HIP_TRY(mcmc_fill_i32(c->st.t_leaps, c->C, (int32_t)sa.n_leaps, st));
    }
    if (sa.kind == SK_HMCDA) {
        // initializeHMCDAStep returns 1 for every chain: state0.H is still NaN when it runs
        // (HMC.jl:88 ctor, HMCDA.jl:86-92), so p = NaN, a = -1 and the while loop never runs.
        HIP_TRY(mcmc_fill_f64(c->st.t_step, c->C, 1.0, st));
        HIP_TRY(mcmc_fill_f64(c->st.t_bar, c->C, 1.0, st));     // dualLeapStep = 1.
        HIP_TRY(mcmc_fill_f64(c->st.t_h, c->C, 0.0, st));       // dualH = 0.
    }
    if (sa.kind == SK_RAM) {
        // S = diag(model.scale .* sampler.scale) (RAM.jl:51,55) in half 0: packed rows in 64-chain tiles
        // (ram.hpp), diagonal (r, r) at row r(r+1)/2 + r of every tile; the padding block d..dpad-1 is the identity
        const int64_t rl = c->st.ram_ld;
        HIP_TRY(hipMemsetAsync(c->st.ram_L, 0, 2 * (size_t)c->st.ram_hs * 8, st));
        if (c->ram_wave) {                                 // diagonal (k, k) at colstart(k) of every chain block
            for (int k = 0; k < d; ++k)
                HIP_TRY(mcmc_fill_f64_strided(c->st.ram_L + wave_colstart(k, d), c->st.ram_hs / rl, 1, rl,
                                              c->h_scale_eff[k], st));
        } else {
            const int64_t tile = (int64_t)(ram_nrows(c->ram_dpad) + 1) * 64;
            for (int r = 0; r < c->ram_dpad; ++r)
                HIP_TRY(mcmc_fill_f64_strided(c->st.ram_L + (size_t)(r * (r + 1) / 2 + r) * 64, rl / 64, 64, tile,
                                              r < d ? c->h_scale_eff[r] : 1.0, st));
        }
    }
    if (sa.tuner) {
        HIP_TRY(mcmc_fill_i32(c->st.t_acc, c->C, 0, st));
        HIP_TRY(mcmc_fill_i32(c->st.t_prop, c->C, 0, st));
    }
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, ctx->d_err, sizeof err, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (err) return fail(MCMC_E_INIT_OUT_OF_SUPPORT, "Initial values out of model support, try other values");
    c->steps_done = 0;
    return MCMC_OK;
}

extern "C" int mcmc_chains_create(mcmc_model* m, const mcmc_sampler_cfg* s, int64_t nchains, int64_t chain_offset,
                                  uint64_t seed, const double* init_x, mcmc_chains** out) {
    if (!m || !s || !out) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (int r = mcmc_sampler_validate(s)) return r;
    if (nchains <= 0) return fail(MCMC_E_INVALID_ARG, "nchains should be > 0");
    if (chain_offset < 0 || chain_offset + nchains > (int64_t)0x100000000LL)
        return fail(MCMC_E_INVALID_ARG, "global chain ids must fit in 32 bits");
    if (s->kind == MCMC_RAM && m->args.d > mcmc_wpc_ram_max_d())
        return fail(MCMC_E_UNSUPPORTED, "RAM is built for d <= " + std::to_string(mcmc_wpc_ram_max_d()) +
                                        " (the d x d jump factor of every chain is kept in HBM)");
    if (s->kind != MCMC_RWM && s->kind != MCMC_RAM && !m->has_gradient) {
        const char* nm = s->kind == MCMC_MALA ? "MALA" : s->kind == MCMC_HMC ? "HMC" : "HMCDA";
        return fail(MCMC_E_NEEDS_GRADIENT, std::string(nm) + " sampler requires model with gradient function");
    }
    mcmc_ctx* ctx = m->ctx;
    if (int r = set_device(ctx)) return r;
    const int d = m->args.d;
    if (model_is_separable(m) && d > mcmc_wpc_max_d())
        return fail(MCMC_E_UNSUPPORTED, "separable targets support d <= 16384");
    auto* c = new mcmc_chains();
    c->model = m;
    m->chains_alive += 1;
    c->C = nchains;
    c->layout = layout_for(m);
    c->ld = ld_for(c->layout, nchains, d);
    c->offset = chain_offset;
    c->seed = seed;
    c->cfg = *s;
    SamplerArgs& sa = c->sa;
    sa.kind = s->kind;
    sa.tuner = s->tuner;
    sa.scale = s->scale;
    sa.drift_step = s->drift_step;
    sa.n_leaps = s->n_leaps;
    sa.leap_step = s->leap_step;
    sa.rate = s->rate;
    sa.len = s->len;
    sa.shrinkage = s->shrinkage;
    sa.t0 = s->t0;
    sa.step = s->step;
    sa.adapt_step = s->adapt_step;
    sa.max_step = s->max_step;
    sa.target_path = s->target_path;
    sa.target_rate = s->target_rate;
    sa.max_leaps = s->max_leaps > 0 ? s->max_leaps : (int64_t)1 << 20;
    auto bail = [&](int code) {
        mcmc_chains_destroy(c);
        return code;
    };
    const size_t nst = c->layout != LAYOUT_WPC ? (size_t)d * c->ld : (size_t)nchains * c->ld;
    const size_t nc = (size_t)round_up(nchains, 64);
    if (int r = dmalloc(&c->st.x, nst)) return bail(r);
    if (c->layout == LAYOUT_GLM)                 // gradient at the state (regression targets are not separable)
        if (int r = dmalloc(&c->st.g, nst)) return bail(r);
    if (c->layout == LAYOUT_GLM && d > 128 && (sa.kind == SK_HMC || sa.kind == SK_HMCDA))   // d-sliced: momentum
        if (int r = dmalloc(&c->st.mom, (size_t)mcmc_glm_d_pad(d) * c->ld)) return bail(r);      // parking (glm_hmc)
    if (int r = dmalloc(&c->st.lp, nc)) return bail(r);
    const bool tuned = sa.tuner && (sa.kind == SK_MALA || sa.kind == SK_HMC);
    if (tuned || sa.kind == SK_HMCDA)
        if (int r = dmalloc(&c->st.t_step, nc)) return bail(r);
    if (sa.kind == SK_HMCDA) {
        if (int r = dmalloc(&c->st.t_bar, nc)) return bail(r);
        if (int r = dmalloc(&c->st.t_h, nc)) return bail(r);
    }
    if (tuned) {
        if (sa.kind == SK_HMC)
            if (int r = dmalloc(&c->st.t_leaps, nc)) return bail(r);
        if (int r = dmalloc(&c->st.t_acc, nc)) return bail(r);
        if (int r = dmalloc(&c->st.t_prop, nc)) return bail(r);
    }
    // scale = model.scale .* sampler.scale (RWM.jl:52); other samplers do not use it.
    std::vector<double> se(m->scale);
    if (sa.kind == SK_RWM || sa.kind == SK_RAM)                       // RAM.jl:51
        for (auto& v : se) v = v * sa.scale;
    c->h_scale_eff = se;
    if (sa.kind == SK_RAM) {
        // padded width: the lane-per-chain kernel's NC = 4 ceil(d/4), the regression kernel's DF = d_pad
        c->ram_wave = c->layout == LAYOUT_WPC || (c->layout == LAYOUT_GLM && d > 32);
        c->glm_ram_wave = c->layout == LAYOUT_GLM && d > 32;
        if (c->ram_wave) {
            // wave-per-chain: [half][chain][column-major packed factor] (ram.hpp wave layout), one block per chain of
            // every launched wave (8 chains per workgroup when two chains share a wave)
            c->ram_dpad = d;
            c->st.ram_ld = round_up((int64_t)ram_nrows(d), 8);
            c->st.ram_hs = round_up(nchains, 8) * c->st.ram_ld;
        } else {
            c->ram_dpad = c->layout == LAYOUT_GLM ? mcmc_glm_d_pad(d) : (int)round_up(d, 4);
            c->st.ram_ld = round_up(nchains, 256);
            c->st.ram_hs = (int64_t)(ram_nrows(c->ram_dpad) + 1) * c->st.ram_ld;
        }
        if (int r = dmalloc(&c->st.ram_L, 2 * (size_t)c->st.ram_hs)) return bail(r);
        if (c->glm_ram_wave) {
            if (int r = dmalloc(&c->ram_u, (size_t)nchains * (size_t)mcmc_glm_ram_wave_ustride(d))) return bail(r);
            if (int r = dmalloc(&c->ram_nz, (size_t)nchains)) return bail(r);
            if (int r = dmalloc(&c->xprop, nst)) return bail(r);
            if (int r = dmalloc(&c->lpp, nc)) return bail(r);
        }
    }
    c->scale1 = se.empty() ? 0.0 : se[0];
    c->scale_uniform = 1;
    for (double v : se)
        if (!(v == c->scale1)) c->scale_uniform = 0;   // bitwise-equal products only (NaN never)
    if (int r = dmalloc(&c->d_scale_eff, (size_t)round_up(d, 256))) return bail(r);
    if (int r = dmalloc(&c->d_evals, 1)) return bail(r);
    if (dzero(ctx, c->d_scale_eff, (size_t)round_up(d, 256) * 8) != hipSuccess ||
        h2d(ctx, c->d_scale_eff, se.data(), (size_t)d * 8) != hipSuccess)
        return bail(fail(MCMC_E_HIP, "scale upload failed"));
    if (init_x) {
        if (int r = dmalloc(&c->d_init_x, (size_t)d * nchains)) return bail(r);
        if (h2d(ctx, c->d_init_x, init_x, (size_t)d * nchains * 8) != hipSuccess)
            return bail(fail(MCMC_E_HIP, "init_x upload failed"));
    }
    if (int r = init_state(c)) return bail(r);
    *out = c;
    return MCMC_OK;
}

extern "C" int mcmc_chains_destroy(mcmc_chains* c) {
    if (!c) return MCMC_OK;
    (void)hipSetDevice(c->model->ctx->device);
    (void)hipStreamSynchronize(c->model->ctx->stream);
    free_state(c);
    dfree(c->d_scale_eff);
    dfree(c->d_init_x);
    dfree(c->d_evals);
    dfree(c->out_samples.p);
    dfree(c->order_buf.p);
    dfree(c->out_grads.p);
    dfree(c->out_bits.p);
    dfree(c->out_tmp.p);
    dfree(c->stage_samples.p);
    dfree(c->stage_grads.p);
    dfree(c->ram_u);
    dfree(c->ram_nz);
    dfree(c->xprop);
    dfree(c->lpp);
    mcmc_model* m = c->model;
    delete c;
    if (--m->chains_alive == 0 && m->released) model_free(m);
    return MCMC_OK;
}

extern "C" int mcmc_chains_reset(mcmc_chains* c) {
    if (!c) return fail(MCMC_E_INVALID_ARG, "chains is NULL");
    if (int r = set_device(c->model->ctx)) return r;
    return init_state(c);
}

// MCMC.reset(t, x) (MCMC.jl:39): the task-local :reset hook of every sampler (RWM.jl:49, MALA.jl:75-80,
// HMC.jl:114-116, HMCDA.jl:82-83, RAM.jl:47) sets pars = x and re-evaluates the log-target (and gradient) there; the
// step counter, the tuners' state and RAM's factor are left as they are.  x: host [d][C]; lp (may be NULL): host [C],
// the log-targets at x.  A point out of support is accepted (the reference's hook does not assert): its log-target
// is -Inf and the next proposal's ratio decides.
extern "C" int mcmc_chains_set_state(mcmc_chains* c, const double* x, double* lp) {
    if (!c || !x) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    mcmc_model* m = c->model;
    mcmc_ctx* ctx = m->ctx;
    if (int r = set_device(ctx)) return r;
    const int d = m->args.d;
    const int64_t C = c->C;
    hipStream_t st = ctx->stream;
    double* dcols = nullptr;
    if (int r = dmalloc(&dcols, (size_t)d * C)) return r;
    hipError_t e = hipMemcpyAsync(dcols, x, (size_t)d * C * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = cols_to_state(c->layout, c->st.x, c->ld, dcols, C, d, C, st);
    KernelArgs a = base_args(m, C, c->ld);
    if (e == hipSuccess) e = launch_eval(c->layout, a, c->st.x, c->st.lp, c->st.g, 0, st);
    if (e == hipSuccess && lp) e = hipMemcpyAsync(lp, c->st.lp, (size_t)C * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipStreamSynchronize(st);
    dfree(dcols);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("set_state: ") + hipGetErrorString(e));
    c->h_evals += C;                                    // model.eval(pars) once per chain
    return MCMC_OK;
}

// chains [first, first + count) of src as an independent batch: the same model, sampler and seed, global chain ids
// src's + first, and a copy of their whole state -- position, log-target, gradient, the tuners' per-chain state, RAM's
// factor and the step counter -- so running the new batch continues exactly those chains (their random streams are
// keyed by (seed, global chain, global step)), whatever src does afterwards.  Evaluation counts restart at 0.  Used
// for run(t::Array{MCMCTask}) on GPU tasks: one batched launch, then every returned MCMCChain's task continues its own
// chain (runners.jl:14).
extern "C" int mcmc_chains_fork(mcmc_chains* src, int64_t first, int64_t count, mcmc_chains** out) {
    if (!src || !out) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (first < 0 || count <= 0 || first + count > src->C)
        return fail(MCMC_E_INVALID_ARG, "fork: chains [" + std::to_string(first) + ", " + std::to_string(first + count) +
                                            ") are not inside the batch of " + std::to_string(src->C));
    mcmc_model* m = src->model;
    mcmc_ctx* ctx = m->ctx;
    if (int r = set_device(ctx)) return r;
    hipStream_t st = ctx->stream;
    HIP_TRY(hipStreamSynchronize(st));
    const int d = m->args.d;
    std::vector<double> init;
    if (src->d_init_x) {                                   // the forked chains' own starts (resume restarts there)
        init.resize((size_t)d * count);
        HIP_TRY(hipMemcpy2DAsync(init.data(), (size_t)count * 8, src->d_init_x + first, (size_t)src->C * 8,
                                 (size_t)count * 8, (size_t)d, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    mcmc_chains* c = nullptr;
    if (int r = mcmc_chains_create(m, &src->cfg, count, src->offset + first, src->seed,
                                   init.empty() ? nullptr : init.data(), &c))
        return r;
    auto bail = [&](hipError_t e) {
        mcmc_chains_destroy(c);
        return fail(MCMC_E_HIP, std::string("fork: ") + hipGetErrorString(e));
    };
    auto cols = [&](double* dst, const double* from) -> hipError_t {       // per-coordinate rows or per-chain rows
        if (!dst || !from) return hipSuccess;
        if (c->layout == LAYOUT_WPC)
            return hipMemcpyAsync(dst, from + (size_t)first * src->ld, (size_t)count * c->ld * 8,
                                  hipMemcpyDeviceToDevice, st);
        return hipMemcpy2DAsync(dst, (size_t)c->ld * 8, from + first, (size_t)src->ld * 8, (size_t)count * 8,
                                (size_t)d, hipMemcpyDeviceToDevice, st);
    };
    auto vec = [&](void* dst, const void* from, size_t esz) -> hipError_t {
        if (!dst || !from) return hipSuccess;
        return hipMemcpyAsync(dst, (const char*)from + (size_t)first * esz, (size_t)count * esz,
                              hipMemcpyDeviceToDevice, st);
    };
    hipError_t e = cols(c->st.x, src->st.x);
    if (e == hipSuccess) e = cols(c->st.g, src->st.g);
    if (e == hipSuccess) e = vec(c->st.lp, src->st.lp, 8);
    if (e == hipSuccess) e = vec(c->st.t_step, src->st.t_step, 8);
    if (e == hipSuccess) e = vec(c->st.t_bar, src->st.t_bar, 8);
    if (e == hipSuccess) e = vec(c->st.t_h, src->st.t_h, 8);
    if (e == hipSuccess) e = vec(c->st.t_leaps, src->st.t_leaps, 4);
    if (e == hipSuccess) e = vec(c->st.t_acc, src->st.t_acc, 4);
    if (e == hipSuccess) e = vec(c->st.t_prop, src->st.t_prop, 4);
    if (e != hipSuccess) return bail(e);
    if (src->st.ram_L) {
        // the factor written last sits in half (steps_done & 1) of both batches (the step counter is copied)
        const size_t half = (size_t)(src->steps_done & 1);
        const double* sh = src->st.ram_L + half * (size_t)src->st.ram_hs;
        double* dh = c->st.ram_L + half * (size_t)c->st.ram_hs;
        if (c->ram_wave) {                                 // [chain][ram_ld]
            e = hipMemcpyAsync(dh, sh + (size_t)first * src->st.ram_ld, (size_t)count * c->st.ram_ld * 8,
                               hipMemcpyDeviceToDevice, st);
        } else {                                           // [64-chain tile][row][64]: re-tile on the host
            const size_t tile = (ram_nrows(src->ram_dpad) + 1) * 64;
            std::vector<double> hs(((size_t)src->C + 63) / 64 * tile), hd(((size_t)count + 63) / 64 * tile, 0.0);
            e = hipMemcpyAsync(hs.data(), sh, hs.size() * 8, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipMemcpyAsync(hd.data(), dh, hd.size() * 8, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e == hipSuccess) {
                for (int64_t k = 0; k < count; ++k) {
                    const size_t a = (size_t)(first + k), b = (size_t)k;
                    for (size_t r = 0; r + 1 < tile / 64; ++r) hd[(b >> 6) * tile + r * 64 + (b & 63)] =
                                                                   hs[(a >> 6) * tile + r * 64 + (a & 63)];
                }
                e = hipMemcpyAsync(dh, hd.data(), hd.size() * 8, hipMemcpyHostToDevice, st);
            }
        }
        if (e != hipSuccess) return bail(e);
    }
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return bail(e);
    c->steps_done = src->steps_done;
    c->spl = src->spl;
    c->store_grads = src->store_grads;
    c->tuner_burnin = src->tuner_burnin;
    *out = c;
    return MCMC_OK;
}

extern "C" int mcmc_debug_chains_order(mcmc_chains* c, int32_t* used, int32_t* order) {
    if (!c || !used) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    *used = c->last_order ? 1 : 0;
    if (c->last_order && order) std::copy(c->h_order.begin(), c->h_order.end(), order);
    return MCMC_OK;
}

extern "C" int mcmc_chains_evals(mcmc_chains* c, int64_t* evals) {
    if (!c || !evals) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    mcmc_ctx* ctx = c->model->ctx;
    if (int r = set_device(ctx)) return r;
    unsigned long long v = 0;
    HIP_TRY(d2h(ctx, &v, c->d_evals, sizeof v));
    *evals = (int64_t)v + c->h_evals;
    return MCMC_OK;
}

extern "C" int mcmc_chains_ram_factor(mcmc_chains* c, double* S) {
    if (!c || !S) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    if (c->sa.kind != SK_RAM) return fail(MCMC_E_INVALID_ARG, "chains do not run the RAM sampler");
    mcmc_ctx* ctx = c->model->ctx;
    if (int r = set_device(ctx)) return r;
    const size_t rows = ram_nrows(c->model->args.d);          // the leading rows of the padded packing
    const size_t rl = (size_t)c->st.ram_ld;
    const double* cur = c->st.ram_L + (size_t)(c->steps_done & 1) * (size_t)c->st.ram_hs;   // written last
    if (c->ram_wave) {                                         // [chain][column-major packed] -> [row][chain]
        const int64_t d = c->model->args.d;
        std::vector<double> h((size_t)c->C * rl);
        HIP_TRY(hipMemcpyAsync(h.data(), cur, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        for (int64_t r = 0; r < d; ++r)
            for (int64_t q = 0; q <= r; ++q)
                for (size_t ch = 0; ch < (size_t)c->C; ++ch)
                    S[(size_t)(r * (r + 1) / 2 + q) * (size_t)c->C + ch] = h[ch * rl + (size_t)(wave_colstart(q, d) + r - q)];
        return MCMC_OK;
    }
    const size_t tile = (ram_nrows(c->ram_dpad) + 1) * 64;    // one 64-chain tile of a half (ram.hpp)
    const size_t ntiles = ((size_t)c->C + 63) / 64;
    std::vector<double> h(ntiles * tile);
    HIP_TRY(hipMemcpyAsync(h.data(), cur, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (size_t r = 0; r < rows; ++r)                          // [tile][row][64] -> [row][chain]
        for (size_t ch = 0; ch < (size_t)c->C; ++ch) S[r * (size_t)c->C + ch] = h[(ch >> 6) * tile + r * 64 + (ch & 63)];
    return MCMC_OK;
}

// per-chain adaptive state: the step size (MALA driftStep, HMC leapStep, HMCDA leapStep), HMCDA's dual-averaged
// step (dualLeapStep, HMCDA.jl:139) and the tuned HMC nLeaps; a buffer the sampler does not keep is filled with
// NaN (step, step_bar) or 0 (nleaps)
extern "C" int mcmc_chains_tuner_state(mcmc_chains* c, double* step, double* step_bar, int32_t* nleaps) {
    if (!c) return fail(MCMC_E_INVALID_ARG, "chains is NULL");
    mcmc_ctx* ctx = c->model->ctx;
    if (int r = set_device(ctx)) return r;
    const size_t C = (size_t)c->C;
    auto get = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
        return e == hipSuccess ? hipStreamSynchronize(ctx->stream) : e;
    };
    if (step) {
        if (c->st.t_step) HIP_TRY(get(step, c->st.t_step, C * 8));
        else std::fill(step, step + C, __builtin_nan(""));
    }
    if (step_bar) {
        if (c->st.t_bar) HIP_TRY(get(step_bar, c->st.t_bar, C * 8));
        else std::fill(step_bar, step_bar + C, __builtin_nan(""));
    }
    if (nleaps) {
        if (c->st.t_leaps) HIP_TRY(get(nleaps, c->st.t_leaps, C * 4));
        else std::fill(nleaps, nleaps + C, 0);
    }
    return MCMC_OK;
}

extern "C" int mcmc_chains_steps_done(mcmc_chains* c, int64_t* steps) {
    if (!c || !steps) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    *steps = c->steps_done;
    return MCMC_OK;
}

extern "C" int mcmc_chains_step_kernel(mcmc_chains* c, char* buf, int64_t cap) {
    if (!c || !buf || cap < 1) return fail(MCMC_E_INVALID_ARG, "bad argument");
    std::snprintf(buf, (size_t)cap, "%s", c->step_kernel.c_str());
    return MCMC_OK;
}

extern "C" int mcmc_chains_set_steps_per_launch(mcmc_chains* c, int64_t spl) {
    if (!c || spl < 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    c->spl = spl;
    return MCMC_OK;
}

extern "C" int mcmc_chains_set_tuner_burnin(mcmc_chains* c, int64_t burnin) {
    if (!c) return fail(MCMC_E_INVALID_ARG, "chains is NULL");
    if (burnin < -1) return fail(MCMC_E_INVALID_ARG, "tuner burnin must be >= 0, or -1 (the runner's burnin)");
    c->tuner_burnin = burnin;
    return MCMC_OK;
}

extern "C" int mcmc_chains_set_store_gradients(mcmc_chains* c, int32_t store) {
    if (!c) return fail(MCMC_E_INVALID_ARG, "chains is NULL");
    c->store_grads = store ? 1 : 0;
    return MCMC_OK;
}

// steps fused per launch for a run of len steps: the user's setting (0: the whole run), capped by the
// kernels that fuse a bounded number of steps (the single-slice regression MALA kernel: one)
static int64_t launch_steps(const mcmc_chains* c, int64_t len) {
    int64_t spl = c->spl > 0 ? c->spl : len;
    if (c->layout == LAYOUT_GLM) {
        const int64_t kmax = mcmc_glm_steps_per_launch(c->model->args.d, c->model->args.n, c->sa.kind);
        if (kmax > 0 && spl > kmax) spl = kmax;
    }
    return spl < 1 ? 1 : spl;
}

extern "C" int mcmc_chains_launches(mcmc_chains* c, int64_t len, int64_t* launches) {
    if (!c || !launches || len < 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    const int64_t spl = launch_steps(c, len);
    *launches = len == 0 ? 0 : (len + spl - 1) / spl;
    return MCMC_OK;
}

// Pre-size the library-owned output buffers of a run keeping nkept steps (the wave-per-chain staging
// rows, and the device copies used when the caller's buffers are on the host), so that the run itself
// allocates nothing.  Buffers only grow; they are freed with the chains.
extern "C" int mcmc_chains_reserve_outputs(mcmc_chains* c, int64_t nkept, int32_t on_device) {
    if (!c || nkept < 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    if (int rc = set_device(c->model->ctx)) return rc;
    const size_t d = (size_t)c->model->args.d, C = (size_t)c->C, nk = (size_t)nkept;
    const bool grads = c->sa.kind != SK_RWM && c->sa.kind != SK_RAM && c->store_grads;
    if (c->layout == LAYOUT_WPC) {
        const size_t nstage = nk * C * (size_t)c->ld;
        if (int rc = ensure(c->stage_samples, nstage * 8)) return rc;
        if (grads)
            if (int rc = ensure(c->stage_grads, nstage * 8)) return rc;
    }
    if (!on_device) {
        if (int rc = ensure(c->out_samples, nk * d * C * 8)) return rc;
        if (grads)
            if (int rc = ensure(c->out_grads, nk * d * C * 8)) return rc;
        if (int rc = ensure(c->out_bits, nk * ((C + 63) / 64) * 8)) return rc;
    }
    return MCMC_OK;
}

extern "C" int mcmc_chains_store_leaps(mcmc_chains* c, int64_t cap, double* pars, double* grads, double* mom,
                                       double* lp, double* H, int32_t* nleaps) {
    if (!c) return fail(MCMC_E_INVALID_ARG, "NULL chains");
    if (pars == nullptr) {
        c->h_lpars = nullptr;
        c->leap_cap = 0;
        return MCMC_OK;
    }
    if (c->sa.kind != SK_HMC && c->sa.kind != SK_HMCDA)
        return fail(MCMC_E_INVALID_ARG, "storeLeaps needs an HMC or HMCDA sampler");
    if (cap < 0 || !grads || !mom || !lp || !H || !nleaps) return fail(MCMC_E_INVALID_ARG, "bad storeLeaps buffers");
    c->leap_cap = cap;
    c->h_lpars = pars;
    c->h_lgrads = grads;
    c->h_lmom = mom;
    c->h_llp = lp;
    c->h_lH = H;
    c->h_lnl = nleaps;
    return MCMC_OK;
}

// ------------------------------------------------------------------ run
// device -> host copy of `rows` rows of `width` bytes from a packed device array into a host array whose
// rows are `dpitch` bytes apart (dpitch == width: one contiguous copy)
static hipError_t d2h_rows(mcmc_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t width, size_t rows) {
    hipError_t e = dpitch == width
                       ? hipMemcpyAsync(dst, src, width * rows, hipMemcpyDeviceToHost, ctx->stream)
                       : hipMemcpy2DAsync(dst, dpitch, src, width, width, rows, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
}

extern "C" int mcmc_run_serialmc(mcmc_chains* c, const mcmc_runner_cfg* r, mcmc_outputs* out) {
    return mcmc_run_serialmc_ld(c, r, out, c ? c->C : 0, nullptr);
}

// run_serialmc with host outputs laid out for a larger chain batch this one is a block of (mcmc_group.cpp):
// samples/gradients/final_x rows are ldc chains apart, accept-bit rows ceil(ldc/64) words apart; the caller
// has offset every pointer to this block's first chain (a multiple of 64 when ldc != C).  copy_s: the
// device -> host time of the outputs.
int mcmc_run_serialmc_ld(mcmc_chains* c, const mcmc_runner_cfg* r, mcmc_outputs* out, int64_t ldc, double* copy_s) {
    if (!c || !r) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    if (ldc < c->C) return fail(MCMC_E_INVALID_ARG, "output leading dimension below the chain count");
    if (out && out->on_device && ldc != c->C)
        return fail(MCMC_E_INVALID_ARG, "strided outputs are host buffers");
    if (int rc = mcmc_runner_validate(r)) return rc;
    mcmc_model* m = c->model;
    mcmc_ctx* ctx = m->ctx;
    if (int rc = set_device(ctx)) return rc;
    hipStream_t st = ctx->stream;
    const int d = m->args.d;
    const int64_t C = c->C;
    const Layout L = c->layout;
    const int64_t nkept = nkept_of(*r);
    const int64_t nw = (C + 63) / 64;
    if (c->steps_done + r->len > 0xffffffffLL) return fail(MCMC_E_INVALID_ARG, "step counter exceeds 2^32");
    const bool on_dev = out && out->on_device;
    const bool want_samples = out && out->samples;
    const bool grad_sampler = c->sa.kind != SK_RWM && c->sa.kind != SK_RAM;   // RWM, RAM: no gradients
    const bool want_grads = out && out->gradients && grad_sampler && c->store_grads;
    const bool want_bits = out && out->accept_bits;

    // output buffers in the C ABI layout ([nkept][d][C]) on the device
    double* d_samples = nullptr;
    double* d_grads = nullptr;
    uint64_t* d_bits = nullptr;
    const size_t nsamp = (size_t)nkept * (size_t)d * (size_t)C;
    if (want_samples) {
        if (on_dev) d_samples = out->samples;
        else {
            if (int rc = ensure(c->out_samples, nsamp * 8)) return rc;
            d_samples = (double*)c->out_samples.p;
        }
    }
    if (want_grads) {
        if (on_dev) d_grads = out->gradients;
        else {
            if (int rc = ensure(c->out_grads, nsamp * 8)) return rc;
            d_grads = (double*)c->out_grads.p;
        }
    }
    if (want_bits) {
        if (on_dev) d_bits = out->accept_bits;
        else {
            if (int rc = ensure(c->out_bits, (size_t)nkept * nw * 8)) return rc;
            d_bits = (uint64_t*)c->out_bits.p;
        }
    }
    // wave-per-chain kernels write kept rows chain-major ([nkept][C][ld]); transposed after the loop
    double* k_samples = d_samples;
    double* k_grads = d_grads;
    if (L == LAYOUT_WPC) {
        const size_t nstage = (size_t)nkept * (size_t)C * (size_t)c->ld;
        if (want_samples) {
            if (int rc = ensure(c->stage_samples, nstage * 8)) return rc;
            k_samples = (double*)c->stage_samples.p;
        }
        if (want_grads) {
            if (int rc = ensure(c->stage_grads, nstage * 8)) return rc;
            k_grads = (double*)c->stage_grads.p;
        }
    }

    KernelArgs a = base_args(m, C, c->ld);
    a.sa = c->sa;
    a.st = c->st;
    StepArgs& s = a.s;
    s.chain0 = (uint32_t)c->offset;
    s.key0 = (uint32_t)c->seed;
    s.key1 = (uint32_t)(c->seed >> 32);
    s.run_step0 = c->steps_done;
    s.burnin = r->burnin;
    s.thinning = r->thinning;
    s.len = r->len;
    s.tuner_burnin = c->tuner_burnin >= 0 ? c->tuner_burnin : r->burnin;   // MALA.jl:116, HMC.jl:167, HMCDA.jl:133
    s.scale = c->d_scale_eff;
    s.scale1 = c->scale1;
    s.scale_uniform = c->scale_uniform;

    s.samples = k_samples;
    s.grads = k_grads;
    s.acc_bits = d_bits;
    s.nw = nw;
    const bool host_evals = evals_on_host(c);
    s.n_evals = host_evals ? nullptr : c->d_evals;
    s.order = nullptr;
    c->last_order = false;
    // regression tiles run their leapfrog loop to their longest chain.  (The lane / pair layouts were measured
    // with the same order and it did not pay: DESIGN.md §5.3.)
    static const bool order_off = [] {                 // MCMCHIP_TRAJ_ORDER=0: identity order (A/B measurements)
        const char* e = std::getenv("MCMCHIP_TRAJ_ORDER");
        return e != nullptr && e[0] == '0';
    }();
    if (!order_off && L == LAYOUT_GLM && C > 16 && (c->sa.kind == SK_HMCDA || (c->sa.kind == SK_HMC && c->sa.tuner))) {
        if (int rc = glm_trajectory_order(c, st)) return rc;
        s.order = (const int32_t*)c->order_buf.p;
        c->last_order = true;
    }

    // storeLeaps: one step per launch; before each kept step, a record launch of its trajectory
    const bool rec = c->h_lpars != nullptr;
    const int64_t spl = rec ? 1 : launch_steps(c, r->len);
    const size_t lsz = rec ? (size_t)(c->leap_cap + 1) * (size_t)d * (size_t)C : 0;   // doubles per kept step
    const size_t lsc = rec ? (size_t)(c->leap_cap + 1) * (size_t)C : 0;
    const size_t nk = (size_t)nkept;
    double* dl = nullptr;
    if (rec) {
        if (int rc = ensure(c->leap_buf, nk * (3 * lsz + 2 * lsc) * 8 + nk * (size_t)C * 4)) return rc;
        dl = (double*)c->leap_buf.p;
        HIP_TRY(mcmc_fill_f64(dl, (int64_t)(nk * (3 * lsz + 2 * lsc)), __builtin_nan(""), st));
        HIP_TRY(hipMemsetAsync(dl + nk * (3 * lsz + 2 * lsc), 0, nk * (size_t)C * 4, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventRecord(ctx->ev0, st));
    if (want_bits && L != LAYOUT_LPC) HIP_TRY(hipMemsetAsync(d_bits, 0, (size_t)nkept * nw * 8, st));
    for (int64_t done = 0; done < r->len; done += spl) {
        const int64_t n = std::min(spl, r->len - done);
        s.step_begin = c->steps_done + done + 1;
        s.nsteps = (int32_t)n;
        int64_t kk;
        if (rec && kept_index(done + 1, r->burnin, r->thinning, r->len, &kk)) {
            LeapRec lr;
            lr.cap = c->leap_cap;
            lr.pars = dl + (size_t)kk * lsz;
            lr.grads = dl + nk * lsz + (size_t)kk * lsz;
            lr.mom = dl + 2 * nk * lsz + (size_t)kk * lsz;
            lr.lp = dl + 3 * nk * lsz + (size_t)kk * lsc;
            lr.H = dl + 3 * nk * lsz + nk * lsc + (size_t)kk * lsc;
            lr.nl = (int32_t*)(dl + 3 * nk * lsz + 2 * nk * lsc) + (size_t)kk * (size_t)C;
            HIP_TRY(launch_record(L, a, lr, st));
        }
        g_step_kernel[0] = 0;
        HIP_TRY(launch_chain_step(c, a, st));
        c->step_kernel = g_step_kernel;
        if (host_evals) c->h_evals += C * n;
    }
    HIP_TRY(hipEventRecord(ctx->ev1, st));
    if (L == LAYOUT_WPC) {
        if (want_samples) HIP_TRY(mcmc_transpose(d_samples, C, k_samples, c->ld, nkept, C, d, st));
        if (want_grads) HIP_TRY(mcmc_transpose(d_grads, C, k_grads, c->ld, nkept, C, d, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    auto t1 = std::chrono::steady_clock::now();
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    c->steps_done += r->len;
    if (rec) {
        HIP_TRY(d2h(ctx, c->h_lpars, dl, nk * lsz * 8));
        HIP_TRY(d2h(ctx, c->h_lgrads, dl + nk * lsz, nk * lsz * 8));
        HIP_TRY(d2h(ctx, c->h_lmom, dl + 2 * nk * lsz, nk * lsz * 8));
        HIP_TRY(d2h(ctx, c->h_llp, dl + 3 * nk * lsz, nk * lsc * 8));
        HIP_TRY(d2h(ctx, c->h_lH, dl + 3 * nk * lsz + nk * lsc, nk * lsc * 8));
        HIP_TRY(d2h(ctx, c->h_lnl, dl + 3 * nk * lsz + 2 * nk * lsc, nk * (size_t)C * 4));
        c->h_lpars = nullptr;                          // one run consumes the registration
    }

    if (out) {
        out->nkept = nkept;
        out->runtime_s = std::chrono::duration<double>(t1 - t0).count();
        out->kernel_ms = ms;
        const size_t rowb = (size_t)C * 8, drow = (size_t)ldc * 8;
        const size_t nwl = (size_t)(ldc + 63) / 64;
        auto c0 = std::chrono::steady_clock::now();
        if (!on_dev) {
            if (want_samples) HIP_TRY(d2h_rows(ctx, out->samples, drow, d_samples, rowb, (size_t)nkept * d));
            if (want_grads) HIP_TRY(d2h_rows(ctx, out->gradients, drow, d_grads, rowb, (size_t)nkept * d));
            if (want_bits) HIP_TRY(d2h_rows(ctx, out->accept_bits, nwl * 8, d_bits, (size_t)nw * 8, (size_t)nkept));
        }
        if (out->final_x) {
            if (on_dev) {
                HIP_TRY(state_to_cols(L, out->final_x, C, c->st.x, c->ld, d, C, st));
            } else {
                if (int rc = ensure(c->out_tmp, (size_t)d * C * 8)) return rc;
                HIP_TRY(state_to_cols(L, (double*)c->out_tmp.p, C, c->st.x, c->ld, d, C, st));
                HIP_TRY(d2h_rows(ctx, out->final_x, drow, c->out_tmp.p, rowb, (size_t)d));
            }
        }
        if (out->final_lp)
            HIP_TRY(hipMemcpyAsync(out->final_lp, c->st.lp, (size_t)C * 8,
                                   on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (copy_s) *copy_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    }
    return MCMC_OK;
}

// ------------------------------------------------------------------ debug probes
// ------------------------------------------------------------------ SeqMC (SeqMC.jl:21-122)
extern "C" int mcmc_seqmc_validate(const mcmc_seqmc_cfg* cfg) {
    if (!cfg) return fail(MCMC_E_INVALID_ARG, "seqmc cfg is NULL");
    char buf[160];
    if (!(cfg->burnin >= 0)) {
        snprintf(buf, sizeof buf, "Burnin rounds (%lld) should be >= 0", (long long)cfg->burnin);        // SeqMC.jl:30
        return fail(MCMC_E_INVALID_ARG, buf);
    }
    if (!(cfg->steps > cfg->burnin)) {
        snprintf(buf, sizeof buf, "Steps (%lld) should be > to burnin (%lld)", (long long)cfg->steps,
                 (long long)cfg->burnin);                                                                 // SeqMC.jl:31
        return fail(MCMC_E_INVALID_ARG, buf);
    }
    return MCMC_OK;
}

// One sampler step of every chain of `c` from its current state, nothing kept (the SamplerTask's
// `consume` inside run_seqmc, SeqMC.jl:69).
static int step_once(mcmc_chains* c, hipStream_t st) {
    mcmc_model* m = c->model;
    KernelArgs a = base_args(m, c->C, c->ld);
    a.sa = c->sa;
    a.st = c->st;
    StepArgs& s = a.s;
    s.chain0 = (uint32_t)c->offset;
    s.key0 = (uint32_t)c->seed;
    s.key1 = (uint32_t)(c->seed >> 32);
    s.run_step0 = c->steps_done;
    s.burnin = 0;
    s.thinning = 1;
    s.len = 1;
    s.tuner_burnin = 0;
    s.scale = c->d_scale_eff;
    s.scale1 = c->scale1;
    s.scale_uniform = c->scale_uniform;
    s.samples = nullptr;
    s.grads = nullptr;
    s.acc_bits = nullptr;
    s.nw = (c->C + 63) / 64;
    s.n_evals = evals_on_host(c) ? nullptr : c->d_evals;
    s.step_begin = c->steps_done + 1;
    s.nsteps = 1;
    HIP_TRY(launch_chain_step(c, a, st));
    if (evals_on_host(c)) c->h_evals += c->C;
    c->steps_done += 1;
    return MCMC_OK;
}

extern "C" int mcmc_run_seqmc(mcmc_chains* const* targets, int32_t ntargets, int64_t npart, const double* particles,
                              const mcmc_seqmc_cfg* cfg, uint64_t seed, int32_t on_device, double* samples,
                              double* weights, int32_t* resampled, double* runtime_s) {
    if (!targets || ntargets < 1 || !particles || !cfg) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    if (int r = mcmc_seqmc_validate(cfg)) return r;
    if (npart < 1) return fail(MCMC_E_INVALID_ARG, "need at least one particle");
    for (int t = 0; t < ntargets; ++t)
        if (!targets[t]) return fail(MCMC_E_INVALID_ARG, "NULL target");
    mcmc_ctx* ctx = targets[0]->model->ctx;
    const int d = targets[0]->model->args.d;
    for (int t = 0; t < ntargets; ++t) {
        if (targets[t]->model->args.d != d)
            return fail(MCMC_E_INVALID_ARG, "Models do not have the same parameter vector size");  // SeqMC.jl:49
        if (targets[t]->model->ctx != ctx) return fail(MCMC_E_INVALID_ARG, "targets live on different contexts");
        if (targets[t]->C != npart) return fail(MCMC_E_INVALID_ARG, "every target needs nchains == npart");
    }
    if (cfg->steps > 0xffffffffLL) return fail(MCMC_E_INVALID_ARG, "steps exceed 2^32");
    if (int r = set_device(ctx)) return r;
    hipStream_t st = ctx->stream;
    const size_t nd = (size_t)d * (size_t)npart, N = (size_t)npart;
    const int64_t nstore = cfg->steps - cfg->burnin;
    double *parsA = nullptr, *parsB = nullptr, *logW = nullptr, *lt = nullptr, *lt2 = nullptr, *ll0 = nullptr,
           *cp = nullptr, *dsamp = nullptr, *dw = nullptr;
    int32_t *flags = nullptr;
    int rc = MCMC_OK;
    auto t0 = std::chrono::steady_clock::now();
    do {
        if ((rc = dmalloc(&parsA, nd)) || (rc = dmalloc(&parsB, nd)) || (rc = dmalloc(&logW, N)) ||
            (rc = dmalloc(&lt, N)) || (rc = dmalloc(&lt2, N)) || (rc = dmalloc(&ll0, N)) || (rc = dmalloc(&cp, N)) ||
            (rc = dmalloc(&flags, (size_t)cfg->steps * ntargets)))
            break;
        if (on_device) {
            dsamp = samples;
            dw = weights;
        } else if ((samples && (rc = dmalloc(&dsamp, (size_t)nstore * nd))) ||
                   (weights && (rc = dmalloc(&dw, (size_t)nstore * N)))) {
            break;
        }
        hipError_t e = on_device ? hipMemcpyAsync(parsA, particles, nd * 8, hipMemcpyDeviceToDevice, st)
                                 : h2d(ctx, parsA, particles, nd * 8);
        if (e == hipSuccess) e = dzero(ctx, logW, N * 8);                       // logW = zeros(npart)
        if (e == hipSuccess) e = dzero(ctx, lt, N * 8);                         // logtarget = zeros(npart)
        for (int64_t i = 1; e == hipSuccess && i <= cfg->steps; ++i) {
            for (int t = 0; e == hipSuccess && t < ntargets; ++t) {
                mcmc_chains* c = targets[t];
                KernelArgs a = base_args(c->model, c->C, c->ld);
                // MCMC.reset(t, pars[n]): state <- particle, logtarget <- eval (RWM.jl:49, MALA.jl:75-78)
                e = cols_to_state(c->layout, c->st.x, c->ld, parsA, npart, d, npart, st);
                if (e == hipSuccess) e = launch_eval(c->layout, a, c->st.x, c->st.lp, c->st.g, 0, st);
                if (e == hipSuccess) e = hipMemcpyAsync(ll0, c->st.lp, N * 8, hipMemcpyDeviceToDevice, st);
                if (e != hipSuccess) break;
                if ((rc = step_once(c, st))) break;                             // sample = consume(t.task)
                e = state_to_cols(c->layout, parsA, npart, c->st.x, c->ld, d, npart, st);   // pars[n] = ppars
                if (e == hipSuccess) e = mcmc_seqmc_weights(npart, logW, ll0, lt, c->st.lp, st);
                int32_t* flag = flags + (size_t)(i - 1) * ntargets + t;
                if (e == hipSuccess) e = mcmc_seqmc_scan(npart, logW, cfg->trigger, cp, flag, st);
                if (e == hipSuccess)
                    e = mcmc_seqmc_resample(npart, d, cp, flag, seed, (uint32_t)i, (uint32_t)t, parsA, parsB, lt, lt2,
                                            logW, st);
                std::swap(parsA, parsB);
                std::swap(lt, lt2);
            }
            if (rc) break;
            if (e == hipSuccess) e = dzero(ctx, lt, N * 8);                     // logtarget = zeros(npart)
            if (e == hipSuccess && i > cfg->burnin && (dsamp || dw)) {
                const size_t row = (size_t)(i - cfg->burnin - 1);
                double* ps = dsamp ? dsamp + row * nd : parsB;                  // parsB: scratch when not wanted
                double* pw = dw ? dw + row * N : ll0;
                e = mcmc_seqmc_store(npart, d, parsA, logW, ps, pw, st);
            }
        }
        if (rc) break;
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess && !on_device) {
            if (samples) e = d2h(ctx, samples, dsamp, (size_t)nstore * nd * 8);
            if (e == hipSuccess && weights) e = d2h(ctx, weights, dw, (size_t)nstore * N * 8);
        }
        if (e == hipSuccess && resampled) {
            e = on_device ? hipMemcpyAsync(resampled, flags, (size_t)cfg->steps * ntargets * 4, hipMemcpyDeviceToDevice, st)
                          : d2h(ctx, resampled, flags, (size_t)cfg->steps * ntargets * 4);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("seqmc: ") + hipGetErrorString(e));
    } while (0);
    (void)hipStreamSynchronize(st);
    if (runtime_s) *runtime_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    dfree(parsA); dfree(parsB); dfree(logW); dfree(lt); dfree(lt2); dfree(ll0); dfree(cp); dfree(flags);
    if (!on_device) { dfree(dsamp); dfree(dw); }
    return rc;
}

extern "C" int mcmc_stats_ess(mcmc_ctx* ctx, const double* samples, int64_t nkept, int64_t d, int64_t nchains,
                              int32_t vtype, int64_t maxlag, int64_t batchlen, int32_t on_device, double* ess,
                              double* var) {
    if (!ctx || !samples || !ess) return fail(MCMC_E_INVALID_ARG, "NULL argument");
    if (vtype != MCMC_VAR_IMSE && vtype != MCMC_VAR_IPSE && vtype != MCMC_VAR_BM)       // ess.jl:7
        return fail(MCMC_E_INVALID_ARG, "Unknown ESS type " + std::to_string(vtype));
    if (nkept < 2 || d <= 0 || nchains <= 0) return fail(MCMC_E_INVALID_ARG, "need nkept >= 2, d > 0, nchains > 0");
    if (d > 65535) return fail(MCMC_E_UNSUPPORTED, "d > 65535");
    if (maxlag <= 0) maxlag = nkept - 1;
    if (maxlag > nkept - 1) return fail(MCMC_E_INVALID_ARG, "maxlag should be < nkept");
    if (vtype == MCMC_VAR_BM && !(batchlen > 0 && nkept / batchlen > 1))                   // var.jl:22
        return fail(MCMC_E_INVALID_ARG, "Choose batch size such that the number of batches is greather than one");
    if (int r = set_device(ctx)) return r;
    hipStream_t st = ctx->stream;
    const size_t ns = (size_t)nkept * (size_t)d * (size_t)nchains, no = (size_t)d * (size_t)nchains;
    const double* ds = samples;
    double *dsb = nullptr, *de = ess, *dv = var;
    int rc = MCMC_OK;
    do {
        if (!on_device) {
            if ((rc = dmalloc(&dsb, ns))) break;
            if ((rc = dmalloc(&de, no))) break;
            if (var && (rc = dmalloc(&dv, no))) break;
            if (h2d(ctx, dsb, samples, ns * 8) != hipSuccess) { rc = fail(MCMC_E_HIP, "samples upload failed"); break; }
            ds = dsb;
        }
        hipError_t e = mcmc_launch_ess(ds, nkept, d, nchains, vtype, maxlag, batchlen, de, dv, st);
        if (e == hipSuccess && !on_device) e = d2h(ctx, ess, de, no * 8);
        if (e == hipSuccess && !on_device && var) e = d2h(ctx, var, dv, no * 8);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("ess: ") + hipGetErrorString(e));
    } while (0);
    if (!on_device) {
        (void)hipStreamSynchronize(st);
        dfree(dsb);
        dfree(de);
        dfree(dv);
    }
    return rc;
}

extern "C" int mcmc_debug_detmath(mcmc_ctx* ctx, int op, int64_t n, const double* x, const double* y, double* out) {
    if (!ctx || !x || !out || n <= 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    if (int r = set_device(ctx)) return r;
    const size_t nout = (op == 6) ? 4 * (size_t)n : (size_t)n;
    double *dx = nullptr, *dy = nullptr, *dout = nullptr;
    int rc = MCMC_OK;
    do {
        if ((rc = dmalloc(&dx, (size_t)n))) break;
        if ((rc = dmalloc(&dy, (size_t)n))) break;
        if ((rc = dmalloc(&dout, nout))) break;
        hipError_t e = h2d(ctx, dx, x, (size_t)n * 8);
        if (e == hipSuccess && y) e = h2d(ctx, dy, y, (size_t)n * 8);
        if (e == hipSuccess) e = mcmc_detmath(op, n, dx, dy, dout, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = d2h(ctx, out, dout, nout * 8);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("detmath probe: ") + hipGetErrorString(e));
    } while (0);
    dfree(dx);
    dfree(dy);
    dfree(dout);
    return rc;
}

extern "C" int mcmc_debug_philox(mcmc_ctx* ctx, int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    if (!ctx || !ctr || !key || !out || n <= 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    if (int r = set_device(ctx)) return r;
    uint32_t *dc = nullptr, *dk = nullptr, *dout = nullptr;
    int rc = MCMC_OK;
    do {
        if ((rc = dmalloc(&dc, 4 * (size_t)n))) break;
        if ((rc = dmalloc(&dk, 2 * (size_t)n))) break;
        if ((rc = dmalloc(&dout, 4 * (size_t)n))) break;
        hipError_t e = h2d(ctx, dc, ctr, 16 * (size_t)n);
        if (e == hipSuccess) e = h2d(ctx, dk, key, 8 * (size_t)n);
        if (e == hipSuccess) e = mcmc_philox(n, dc, dk, dout, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = d2h(ctx, out, dout, 16 * (size_t)n);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("philox probe: ") + hipGetErrorString(e));
    } while (0);
    dfree(dc);
    dfree(dk);
    dfree(dout);
    return rc;
}

extern "C" int mcmc_debug_mfma_f64(mcmc_ctx* ctx, int nk, const double* A, const double* B, const double* C,
                                   double* D) {
    if (!ctx || !A || !B || !C || !D || nk <= 0) return fail(MCMC_E_INVALID_ARG, "bad argument");
    if (int r = set_device(ctx)) return r;
    double *dA = nullptr, *dB = nullptr, *dC = nullptr, *dD = nullptr;
    int rc = MCMC_OK;
    do {
        if ((rc = dmalloc(&dA, 64 * (size_t)nk))) break;
        if ((rc = dmalloc(&dB, 64 * (size_t)nk))) break;
        if ((rc = dmalloc(&dC, 256))) break;
        if ((rc = dmalloc(&dD, 256))) break;
        hipError_t e = h2d(ctx, dA, A, 512 * (size_t)nk);
        if (e == hipSuccess) e = h2d(ctx, dB, B, 512 * (size_t)nk);
        if (e == hipSuccess) e = h2d(ctx, dC, C, 2048);
        if (e == hipSuccess) e = mcmc_mfma_probe(dA, dB, dC, dD, nk, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = d2h(ctx, D, dD, 2048);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("mfma probe: ") + hipGetErrorString(e));
    } while (0);
    dfree(dA); dfree(dB); dfree(dC); dfree(dD);
    return rc;
}
