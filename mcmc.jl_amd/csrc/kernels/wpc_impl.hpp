// wpc_impl.hpp -- wave-per-chain kernels (32 < d <= 2048): one wave = one chain (4 chains per 256-thread
// block), and block-per-chain kernels (2048 < d <= 16384): W = 4 or 8 waves = one chain; see samplers.hpp for
// the step code and its reference lines.  Included by one translation
// unit per model (wpc_<model>.hip); wpc.hip dispatches on the model kind.
#pragma once
#include "../samplers.hpp"
#include "layout_api.hpp"

namespace mcmc {

constexpr int kChainsPerBlock = kBlock / 64;

// F: d == 256 NB (WaveChain FULL).  The Box-Muller tables: from LDS for NB >= 4 (two waves per SIMD anyway by their
// registers, so two 56 KB blocks per CU cost nothing; config 4 is NB = 4), from global memory for NB <= 2 (three or
// four waves per SIMD, which 56 KB blocks would cut to two)
template <int NB>
constexpr int wpc_tab() { return NB >= 4 ? kTabLds : kTabGlobal; }
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock) void wpc_rwm(KernelArgs a) { rwm_body<WaveChain<NB, F, 1, wpc_tab<NB>()>, M>(a); }
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock) void wpc_mala(KernelArgs a) { mala_body<WaveChain<NB, F, 1, wpc_tab<NB>()>, M>(a); }
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__(kBlock) void wpc_hmc(KernelArgs a) {
    hmc_body<WaveChain<NB, F, 1, wpc_tab<NB>()>, M, DA>(a);
}
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void wpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<WaveChain<NB>, M>(a, xin, lp, g, check);
}

// block per chain, d > 2048: W waves hold the chain's coordinates (WaveChain<8, false, W>), one chain per block
template <int W, class M>
__global__ __launch_bounds__(64 * W) void bpc_rwm(KernelArgs a) { rwm_body<WaveChain<8, false, W, kTabLds>, M>(a); }
template <int W, class M>
__global__ __launch_bounds__(64 * W) void bpc_mala(KernelArgs a) { mala_body<WaveChain<8, false, W, kTabLds>, M>(a); }
template <int W, class M, bool DA>
__global__ __launch_bounds__(64 * W) void bpc_hmc(KernelArgs a) { hmc_body<WaveChain<8, false, W, kTabLds>, M, DA>(a); }
template <int W, class M>
__global__ __launch_bounds__(64 * W) void bpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<WaveChain<8, false, W>, M>(a, xin, lp, g, check);
}
template <int W, class M, bool DA>
__global__ __launch_bounds__(64 * W) void bpc_hmc_rec(KernelArgs a, LeapRec r) {
    hmc_record_body<WaveChain<8, false, W>, M, DA>(a, r);
}

// waves per chain for d > 2048 (G = 8 coordinates' blocks per lane: d <= 2048 W); 0: not built
static inline int bpc_waves_for(int d) { return d <= 2048 ? 1 : d <= 8192 ? 4 : d <= 16384 ? 8 : 0; }

template <int W, class M>
static hipError_t bpc_launch(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)a.s.C);
    static const char* const fam[] = {"", "bpc_rwm<%d, %s>", "bpc_mala<%d, %s>", "bpc_hmc<%d, %s, false>",
                                      "bpc_hmc<%d, %s, true>"};
    if (a.sa.kind >= SK_RWM && a.sa.kind <= SK_HMCDA) mcmc_note_step_kernel(fam[a.sa.kind], W, M::kName);
    switch (a.sa.kind) {
        case SK_RWM: bpc_rwm<W, M><<<grid, 64 * W, 0, st>>>(a); break;
        case SK_MALA: bpc_mala<W, M><<<grid, 64 * W, 0, st>>>(a); break;
        case SK_HMC: bpc_hmc<W, M, false><<<grid, 64 * W, 0, st>>>(a); break;
        case SK_HMCDA: bpc_hmc<W, M, true><<<grid, 64 * W, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
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
    switch (bpc_waves_for(a.s.d)) {
        case 4: return bpc_launch<4, M>(a, st);
        case 8: return bpc_launch<8, M>(a, st);
        default: break;
    }
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
    switch (bpc_waves_for(a.s.d)) {
        case 4: bpc_eval<4, M><<<(unsigned)a.s.C, 256, 0, st>>>(a, xin, lp, g, check); return hipGetLastError();
        case 8: bpc_eval<8, M><<<(unsigned)a.s.C, 512, 0, st>>>(a, xin, lp, g, check); return hipGetLastError();
        default: break;
    }
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
    switch (bpc_waves_for(a.s.d)) {
        case 4:
            if (da) bpc_hmc_rec<4, M, true><<<(unsigned)a.s.C, 256, 0, st>>>(a, r);
            else bpc_hmc_rec<4, M, false><<<(unsigned)a.s.C, 256, 0, st>>>(a, r);
            return hipGetLastError();
        case 8:
            if (da) bpc_hmc_rec<8, M, true><<<(unsigned)a.s.C, 512, 0, st>>>(a, r);
            else bpc_hmc_rec<8, M, false><<<(unsigned)a.s.C, 512, 0, st>>>(a, r);
            return hipGetLastError();
        default: break;
    }
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
