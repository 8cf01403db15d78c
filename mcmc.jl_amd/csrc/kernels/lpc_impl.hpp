// lpc_impl.hpp -- lane-per-chain kernels (d <= 32): one thread = one chain; see samplers.hpp for the
// step code and its reference lines.  Included by one translation unit per model (lpc_<model>.hip)
// so that the instantiations compile in parallel; lpc.hip dispatches on the model kind.
#pragma once
#include "../samplers.hpp"
#include "layout_api.hpp"

namespace mcmc {

// F: d == 4 NB (LaneChain FULL); US: uniform RWM scale
template <int NB, bool F, class M, bool US>
__global__ __launch_bounds__(kBlock, 2) void lpc_rwm(KernelArgs a) { rwm_body<LaneChain<NB, F>, M, US>(a); }
template <int NB, bool F, class M>
__global__ __launch_bounds__(kBlock, 2) void lpc_mala(KernelArgs a) { mala_body<LaneChain<NB, F>, M>(a); }
template <int NB, bool F, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpc_hmc(KernelArgs a) { hmc_body<LaneChain<NB, F>, M, DA>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void lpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<LaneChain<NB>, M>(a, xin, lp, g, check);
}

template <int NB, bool F, class M>
static hipError_t lpc_launch_model(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    switch (a.sa.kind) {
        case SK_RWM:
            if (a.s.scale_uniform) lpc_rwm<NB, F, M, true><<<grid, kBlock, 0, st>>>(a);
            else lpc_rwm<NB, F, M, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case SK_MALA: lpc_mala<NB, F, M><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMC: lpc_hmc<NB, F, M, false><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMCDA: lpc_hmc<NB, F, M, true><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// SPEC: instantiate the FULL (d == 4 NB) variants too -- for the models the benchmarks run
template <int NB, class M, bool SPEC>
static hipError_t lpc_launch_nb(const KernelArgs& a, hipStream_t st) {
    if (SPEC && a.s.d == 4 * NB) return lpc_launch_model<NB, SPEC, M>(a, st);
    return lpc_launch_model<NB, false, M>(a, st);
}

template <class M, bool SPEC>
static hipError_t lpc_step(const KernelArgs& a, hipStream_t st) {
    switch ((a.s.d + 3) / 4) {
        case 1: return lpc_launch_nb<1, M, SPEC>(a, st);
        case 2: return lpc_launch_nb<2, M, SPEC>(a, st);
        case 3: return lpc_launch_nb<3, M, SPEC>(a, st);
        case 4: return lpc_launch_nb<4, M, SPEC>(a, st);
        case 5: return lpc_launch_nb<5, M, SPEC>(a, st);
        case 6: return lpc_launch_nb<6, M, SPEC>(a, st);
        case 7: return lpc_launch_nb<7, M, SPEC>(a, st);
        case 8: return lpc_launch_nb<8, M, SPEC>(a, st);
        default: return hipErrorInvalidValue;
    }
}

template <class M>
static hipError_t lpc_eval_m(const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                             hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    switch ((a.s.d + 3) / 4) {
        case 1: lpc_eval<1, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 2: lpc_eval<2, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 3: lpc_eval<3, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 4: lpc_eval<4, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 5: lpc_eval<5, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 6: lpc_eval<6, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 7: lpc_eval<7, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        case 8: lpc_eval<8, M><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// storeLeaps records (samplers.hpp hmc_record_body), generic mapping only: a diagnostic
template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void lpc_hmc_rec(KernelArgs a, LeapRec r) { hmc_record_body<LaneChain<NB>, M, DA>(a, r); }

template <class M>
static hipError_t lpc_record_m(const KernelArgs& a, const LeapRec& r, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    const bool da = a.sa.kind == SK_HMCDA;
#define LPC_REC(NB)                                                       \
    case NB:                                                              \
        if (da) lpc_hmc_rec<NB, M, true><<<grid, kBlock, 0, st>>>(a, r);   \
        else lpc_hmc_rec<NB, M, false><<<grid, kBlock, 0, st>>>(a, r);     \
        break;
    switch ((a.s.d + 3) / 4) {
        LPC_REC(1) LPC_REC(2) LPC_REC(3) LPC_REC(4) LPC_REC(5) LPC_REC(6) LPC_REC(7) LPC_REC(8)
        default: return hipErrorInvalidValue;
    }
#undef LPC_REC
    return hipGetLastError();
}

}  // namespace mcmc

// one translation unit per model: LPC_UNIT(iso, IsoDot, true) defines mcmc_lpc_step_iso / mcmc_lpc_eval_iso
#define LPC_UNIT(name, Model, SPEC)                                                                      \
    hipError_t mcmc_lpc_step_##name(const mcmc::KernelArgs& a, hipStream_t st) {                         \
        return mcmc::lpc_step<mcmc::Model, SPEC>(a, st);                                                \
    }                                                                                                    \
    hipError_t mcmc_lpc_eval_##name(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, \
                                    int check, hipStream_t st) {                                         \
        return mcmc::lpc_eval_m<mcmc::Model>(a, xin, lp, g, check, st);                                 \
    }                                                                                                    \
    hipError_t mcmc_lpc_record_##name(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st) { \
        return mcmc::lpc_record_m<mcmc::Model>(a, r, st);                                               \
    }

// RAM kernels live in their own translation units (lpc_ram_*.hip, built without machine LICM: hoisted
// fp64 constants would pin the scalar file the factor addressing needs); LPC_RAM_UNIT(iso, IsoDot)
// defines mcmc_lpc_ram_iso.
namespace mcmc {
template <int NB, class M>
__global__ __launch_bounds__(kBlock, NB <= 4 ? 2 : 1) void lpc_ram(KernelArgs a) { ram_body<LaneChain<NB, false>, M>(a); }

template <class M>
static hipError_t lpc_ram_step(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    switch ((a.s.d + 3) / 4) {
        case 1: lpc_ram<1, M><<<grid, kBlock, 0, st>>>(a); break;
        case 2: lpc_ram<2, M><<<grid, kBlock, 0, st>>>(a); break;
        case 3: lpc_ram<3, M><<<grid, kBlock, 0, st>>>(a); break;
        case 4: lpc_ram<4, M><<<grid, kBlock, 0, st>>>(a); break;
        case 5: lpc_ram<5, M><<<grid, kBlock, 0, st>>>(a); break;
        case 6: lpc_ram<6, M><<<grid, kBlock, 0, st>>>(a); break;
        case 7: lpc_ram<7, M><<<grid, kBlock, 0, st>>>(a); break;
        case 8: lpc_ram<8, M><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
}  // namespace mcmc

#define LPC_RAM_UNIT(name, Model)                                                \
    hipError_t mcmc_lpc_ram_##name(const mcmc::KernelArgs& a, hipStream_t st) { \
        return mcmc::lpc_ram_step<mcmc::Model>(a, st);                          \
    }
