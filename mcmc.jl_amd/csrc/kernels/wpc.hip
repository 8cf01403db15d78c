// wpc.hip -- wave-per-chain instantiations of the fused sampler kernels (32 < d <= 2048).
// One wave = one chain (4 chains per 256-thread block); see samplers.hpp for the step code and its reference lines.
#include "../samplers.hpp"

namespace mcmc {

constexpr int kChainsPerBlock = kBlock / 64;

template <int NB, class M>
__global__ __launch_bounds__(kBlock) void wpc_rwm(KernelArgs a) { rwm_body<WaveChain<NB>, M>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void wpc_mala(KernelArgs a) { mala_body<WaveChain<NB>, M>(a); }
template <int NB, class M, bool DA>
__global__ __launch_bounds__(kBlock) void wpc_hmc(KernelArgs a) { hmc_body<WaveChain<NB>, M, DA>(a); }
template <int NB, class M>
__global__ __launch_bounds__(kBlock) void wpc_eval(KernelArgs a, const double* xin, double* lp, double* g,
                                                   int32_t check) {
    eval_body<WaveChain<NB>, M>(a, xin, lp, g, check);
}

template <int NB, class M>
static hipError_t launch_model(const KernelArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    switch (a.sa.kind) {
        case SK_RWM: wpc_rwm<NB, M><<<grid, kBlock, 0, st>>>(a); break;
        case SK_MALA: wpc_mala<NB, M><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMC: wpc_hmc<NB, M, false><<<grid, kBlock, 0, st>>>(a); break;
        case SK_HMCDA: wpc_hmc<NB, M, true><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int NB>
static hipError_t launch_nb(const KernelArgs& a, hipStream_t st) {
    if (a.m.kind == MK_ISO) return launch_model<NB, IsoDot>(a, st);
    if (a.m.kind == MK_NORMAL) return launch_model<NB, NormalDSL>(a, st);
    if (a.m.kind == MK_ABS_NORMAL) return launch_model<NB, AbsNormalDSL>(a, st);
    if (a.m.kind == MK_DIST) return launch_model<NB, DistDSL>(a, st);
    return hipErrorInvalidValue;
}

template <int NB>
static hipError_t launch_eval_nb(const KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                 hipStream_t st) {
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    if (a.m.kind == MK_ISO) wpc_eval<NB, IsoDot><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_NORMAL) wpc_eval<NB, NormalDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_ABS_NORMAL) wpc_eval<NB, AbsNormalDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else if (a.m.kind == MK_DIST) wpc_eval<NB, DistDSL><<<grid, kBlock, 0, st>>>(a, xin, lp, g, check);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// G = 4-coordinate groups per lane: d <= 256 G
static int nb_for(int d) {
    if (d <= 256) return 1;
    if (d <= 512) return 2;
    if (d <= 1024) return 4;
    if (d <= 2048) return 8;
    return 0;
}

}  // namespace mcmc

hipError_t mcmc_launch_wpc_step(const mcmc::KernelArgs& a, hipStream_t st) {
    switch (mcmc::nb_for(a.s.d)) {
        case 1: return mcmc::launch_nb<1>(a, st);
        case 2: return mcmc::launch_nb<2>(a, st);
        case 4: return mcmc::launch_nb<4>(a, st);
        case 8: return mcmc::launch_nb<8>(a, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t mcmc_launch_wpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st) {
    switch (mcmc::nb_for(a.s.d)) {
        case 1: return mcmc::launch_eval_nb<1>(a, xin, lp, g, check, st);
        case 2: return mcmc::launch_eval_nb<2>(a, xin, lp, g, check, st);
        case 4: return mcmc::launch_eval_nb<4>(a, xin, lp, g, check, st);
        case 8: return mcmc::launch_eval_nb<8>(a, xin, lp, g, check, st);
        default: return hipErrorInvalidValue;
    }
}

int mcmc_wpc_max_d() { return 2048; }
