// wpc.hip -- dispatch of the wave- and block-per-chain kernels (32 < d <= 16384) on the model kind; the kernels
// live in wpc_impl.hpp, instantiated per model by wpc_<model>.hip.
#include "layout_api.hpp"

hipError_t mcmc_launch_wpc_step(const mcmc::KernelArgs& a, hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 16384) return hipErrorInvalidValue;
    if (a.sa.kind == SK_RAM) {
        if (a.s.d > mcmc_wpc_ram_max_d()) return hipErrorInvalidValue;
        switch (a.m.kind) {
            case MK_ISO: return mcmc_wpc_ram_iso(a, st);
            case MK_NORMAL: return mcmc_wpc_ram_normal(a, st);
            case MK_ABS_NORMAL: return mcmc_wpc_ram_absnormal(a, st);
            case MK_DIST: return mcmc_wpc_ram_dist(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    switch (a.m.kind) {
        case MK_ISO: return mcmc_wpc_step_iso(a, st);
        case MK_NORMAL: return mcmc_wpc_step_normal(a, st);
        case MK_ABS_NORMAL: return mcmc_wpc_step_absnormal(a, st);
        case MK_DIST: return mcmc_wpc_step_dist(a, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_wpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 16384) return hipErrorInvalidValue;
    switch (a.m.kind) {
        case MK_ISO: return mcmc_wpc_eval_iso(a, xin, lp, g, check, st);
        case MK_NORMAL: return mcmc_wpc_eval_normal(a, xin, lp, g, check, st);
        case MK_ABS_NORMAL: return mcmc_wpc_eval_absnormal(a, xin, lp, g, check, st);
        case MK_DIST: return mcmc_wpc_eval_dist(a, xin, lp, g, check, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_wpc_record(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st) {
    using namespace mcmc;
    if (a.s.d < 1 || a.s.d > 16384) return hipErrorInvalidValue;
    switch (a.m.kind) {
        case MK_ISO: return mcmc_wpc_record_iso(a, r, st);
        case MK_NORMAL: return mcmc_wpc_record_normal(a, r, st);
        case MK_ABS_NORMAL: return mcmc_wpc_record_absnormal(a, r, st);
        case MK_DIST: return mcmc_wpc_record_dist(a, r, st);
        default: return hipErrorInvalidValue;
    }
}

int mcmc_wpc_max_d() { return 16384; }
int mcmc_wpc_ram_max_d() { return 1024; }
