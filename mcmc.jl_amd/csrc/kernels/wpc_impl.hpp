// wpc_impl.hpp -- wave-per-chain kernels (32 < d <= 2048): one wave = one chain (4 chains per 256-thread
// block); see samplers.hpp for the step code and its reference lines.  Included by one translation
// unit per model (wpc_<model>.hip); wpc.hip dispatches on the model kind.
#pragma once
#include "../samplers.hpp"
#include "layout_api.hpp"

namespace mcmc {

constexpr int kChainsPerBlock = kBlock / 64;

// F: d == 256 NB (WaveChain FULL)
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock) void wpc_rwm(KernelArgs a) { rwm_body<WaveChain<NB, F>, M>(a); }
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock) void wpc_mala(KernelArgs a) { mala_body<WaveChain<NB, F>, M>(a); }
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__(kBlock) void wpc_hmc(KernelArgs a) { hmc_body<WaveChain<NB, F>, M, DA>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void wpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<WaveChain<NB>, M>(a, xin, lp, g, check);
}

template <int NB, bool F, class M>
static hipError_t wpc_launch_model(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    static const char* const fam[] = {"", "wpc_rwm<%d, %s, %s>", "wpc_mala<%d, %s, %s>", "wpc_hmc<%d, %s, %s, false>",
                                      "wpc_hmc<%d, %s, %s, true>"};
    if (a.sa.kind >= SK_RWM && a.sa.kind <= SK_HMCDA)
        mcmc_note_step_kernel(fam[a.sa.kind], NB, F ? "true" : "false", M::kName);
    switch (a.sa.kind) {
        case SK_RWM: wpc_rwm<NB, F, M><<<grid, kBlock, 0, st>>>(a); break;
        case SK_MALA: wpc_mala<NB, F, M><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMC: wpc_hmc<NB, F, M, false><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMCDA: wpc_hmc<NB, F, M, true><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// SPEC: instantiate the FULL (d == 256 NB) variants too -- for the models the benchmarks run
template <int NB, class M, bool SPEC>
static hipError_t wpc_launch_nb(const KernelArgs& a, hipStream_t st) {
    if (SPEC && a.s.d == 256 * NB) return wpc_launch_model<NB, SPEC, M>(a, st);
    return wpc_launch_model<NB, false, M>(a, st);
}

// G = Philox blocks per lane: d <= 256 G, 4 (l + 64k) + e < d
static inline int wpc_nb_for(int d) {
    if (d <= 256) return 1;
    if (d <= 512) return 2;
    if (d <= 1024) return 4;
    if (d <= 2048) return 8;
    return 0;
}

template <class M, bool SPEC>
static hipError_t wpc_step(const KernelArgs& a, hipStream_t st) {
    switch (wpc_nb_for(a.s.d)) {
        case 1: return wpc_launch_nb<1, M, SPEC>(a, st);
        case 2: return wpc_launch_nb<2, M, SPEC>(a, st);
        case 4: return wpc_launch_nb<4, M, SPEC>(a, st);
        case 8: return wpc_launch_nb<8, M, SPEC>(a, st);
        default: return hipErrorInvalidValue;
    }
}

template <class M>
static hipError_t wpc_eval_m(const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                             hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    switch (wpc_nb_for(a.s.d)) {
        case 1: wpc_eval<1, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 2: wpc_eval<2, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 4: wpc_eval<4, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 8: wpc_eval<8, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// storeLeaps records (samplers.hpp hmc_record_body), generic mapping only: a diagnostic
template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void wpc_hmc_rec(KernelArgs a, LeapRec r) { hmc_record_body<WaveChain<NB>, M, DA>(a, r); }

template <class M>
static hipError_t wpc_record_m(const KernelArgs& a, const LeapRec& r, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    const bool da = a.sa.kind == SK_HMCDA;
#define WPC_REC(NB)                                                       \
    case NB:                                                              \
        if (da) wpc_hmc_rec<NB, M, true><<<grid, kBlock, 0, st>>>(a, r);   \
        else wpc_hmc_rec<NB, M, false><<<grid, kBlock, 0, st>>>(a, r);     \
        break;
    switch (wpc_nb_for(a.s.d)) {
        WPC_REC(1) WPC_REC(2) WPC_REC(4) WPC_REC(8)
        default: return hipErrorInvalidValue;
    }
#undef WPC_REC
    return hipGetLastError();
}

}  // namespace mcmc

#define WPC_UNIT(name, Model, SPEC)                                                                      \
    hipError_t mcmc_wpc_step_##name(const mcmc::KernelArgs& a, hipStream_t st) {                         \
        return mcmc::wpc_step<mcmc::Model, SPEC>(a, st);                                                \
    }                                                                                                    \
    hipError_t mcmc_wpc_eval_##name(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, \
                                    int check, hipStream_t st) {                                         \
        return mcmc::wpc_eval_m<mcmc::Model>(a, xin, lp, g, check, st);                                 \
    }                                                                                                    \
    hipError_t mcmc_wpc_record_##name(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st) { \
        return mcmc::wpc_record_m<mcmc::Model>(a, r, st);                                               \
    }
