// lpc.hip -- lane-per-chain instantiations of the fused sampler kernels (d <= 32).
// One thread = one chain; see samplers.hpp for the step code and its reference lines.
#include "../samplers.hpp"

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
static hipError_t launch_model(const KernelArgs& a, hipStream_t st) {
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

template <int NB, bool F>
static hipError_t launch_nbf(const KernelArgs& a, hipStream_t st) {
    if (a.m.kind == MK_ISO) return launch_model<NB, F, IsoDot>(a, st);
    if (a.m.kind == MK_NORMAL) return launch_model<NB, F, NormalDSL>(a, st);
    if (a.m.kind == MK_ABS_NORMAL) return launch_model<NB, F, AbsNormalDSL>(a, st);
    if (a.m.kind == MK_DIST) return launch_model<NB, F, DistDSL>(a, st);
    return hipErrorInvalidValue;
}

template <int NB>
static hipError_t launch_nb(const KernelArgs& a, hipStream_t st) {
    return a.s.d == 4 * NB ? launch_nbf<NB, true>(a, st) : launch_nbf<NB, false>(a, st);
}

template <int NB>
static hipError_t launch_eval_nb(const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                 hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kBlock - 1) / kBlock));
    if (a.m.kind == MK_ISO) lpc_eval<NB, IsoDot><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_NORMAL) lpc_eval<NB, NormalDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_ABS_NORMAL) lpc_eval<NB, AbsNormalDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_DIST) lpc_eval<NB, DistDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

static int nb_for(int d) { return d >= 1 && d <= 32 ? (d + 3) / 4 : 0; }

}  // namespace mcmc

hipError_t mcmc_launch_lpc_step(const mcmc::KernelArgs& a, hipStream_t st) {
    switch (mcmc::nb_for(a.s.d)) {
        case 1: return mcmc::launch_nb<1>(a, st);
        case 2: return mcmc::launch_nb<2>(a, st);
        case 3: return mcmc::launch_nb<3>(a, st);
        case 4: return mcmc::launch_nb<4>(a, st);
        case 5: return mcmc::launch_nb<5>(a, st);
        case 6: return mcmc::launch_nb<6>(a, st);
        case 7: return mcmc::launch_nb<7>(a, st);
        case 8: return mcmc::launch_nb<8>(a, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_lpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st) {
    switch (mcmc::nb_for(a.s.d)) {
        case 1: return mcmc::launch_eval_nb<1>(a, xin, lp, g, check, st);
        case 2: return mcmc::launch_eval_nb<2>(a, xin, lp, g, check, st);
        case 3: return mcmc::launch_eval_nb<3>(a, xin, lp, g, check, st);
        case 4: return mcmc::launch_eval_nb<4>(a, xin, lp, g, check, st);
        case 5: return mcmc::launch_eval_nb<5>(a, xin, lp, g, check, st);
        case 6: return mcmc::launch_eval_nb<6>(a, xin, lp, g, check, st);
        case 7: return mcmc::launch_eval_nb<7>(a, xin, lp, g, check, st);
        case 8: return mcmc::launch_eval_nb<8>(a, xin, lp, g, check, st);
        default: return hipErrorInvalidValue;
    }
}

int mcmc_lpc_max_d() { return 32; }
