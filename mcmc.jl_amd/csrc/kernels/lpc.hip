// lpc.hip -- dispatch of the lane-per-chain kernels (d <= 32) on the model kind; the kernels live in
// lpc_impl.hpp, instantiated per model by lpc_<model>.hip.
#include "layout_api.hpp"

hipError_t mcmc_launch_lpc_step(const mcmc::KernelArgs& a, hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 32) return hipErrorInvalidValue;
    if (a.sa.kind == SK_RAM) {
        switch (a.m.kind) {
            case MK_ISO: return mcmc_lpc_ram_iso(a, st);
            case MK_NORMAL: return mcmc_lpc_ram_normal(a, st);
            case MK_ABS_NORMAL: return mcmc_lpc_ram_absnormal(a, st);
            case MK_DIST: return mcmc_lpc_ram_dist(a, st);
            case MK_OU: return mcmc_lpc_ram_ou(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    switch (a.m.kind) {
        case MK_ISO: return mcmc_lpc_step_iso(a, st);
        case MK_NORMAL: return mcmc_lpc_step_normal(a, st);
        case MK_ABS_NORMAL: return mcmc_lpc_step_absnormal(a, st);
        case MK_DIST: return mcmc_lpc_step_dist(a, st);
        case MK_DIST_OBS: return mcmc_lpc_step_distobs(a, st);
        case MK_OU: return mcmc_lpc_step_ou(a, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_lpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 32) return hipErrorInvalidValue;
    switch (a.m.kind) {
        case MK_ISO: return mcmc_lpc_eval_iso(a, xin, lp, g, check, st);
        case MK_NORMAL: return mcmc_lpc_eval_normal(a, xin, lp, g, check, st);
        case MK_ABS_NORMAL: return mcmc_lpc_eval_absnormal(a, xin, lp, g, check, st);
        case MK_DIST: return mcmc_lpc_eval_dist(a, xin, lp, g, check, st);
        case MK_DIST_OBS: return mcmc_lpc_eval_distobs(a, xin, lp, g, check, st);
        case MK_OU: return mcmc_lpc_eval_ou(a, xin, lp, g, check, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_lpc_record(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 32) return hipErrorInvalidValue;
    switch (a.m.kind) {
        case MK_ISO: return mcmc_lpc_record_iso(a, r, st);
        case MK_NORMAL: return mcmc_lpc_record_normal(a, r, st);
        case MK_ABS_NORMAL: return mcmc_lpc_record_absnormal(a, r, st);
        case MK_DIST: return mcmc_lpc_record_dist(a, r, st);
        case MK_DIST_OBS: return mcmc_lpc_record_distobs(a, r, st);
        case MK_OU: return mcmc_lpc_record_ou(a, r, st);
        default: return hipErrorInvalidValue;
    }
}

int mcmc_lpc_max_d() { return 32; }
