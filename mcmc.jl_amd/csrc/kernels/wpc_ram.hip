// wpc_ram.hip -- wave-per-chain RAM kernels (src/samplers/RAM.jl:41-79) for 32 < d <= 1024, every separable
// model kind: ram_wave.hpp ram_wave_body over the wave layout of the jump factor (two chains per wave up to d = 256,
// one beyond).
#include <cstdlib>
#include "wpc_impl.hpp"
#include "../ram_wave.hpp"

namespace mcmc {

template <int G, class M>
__global__ __launch_bounds__(kBlock) void wpc_ram(KernelArgs a) { ram_wave_body<WaveChain<G, false>, M>(a); }

// 32 < d <= 256: two chains per wave (HalfWaveChain), so a column's pivot (three readlanes, a square root and three
// divisions) serves two chains' rows; G slot groups of 128 coordinates
template <int G, class M>
__global__ __launch_bounds__(kBlock, 3) void wpc_ram2(KernelArgs a) { ram_wave_body<HalfWaveChain<G>, M>(a); }
// Three waves per SIMD (168 VGPRs): at d = 256 the G = 2 kernel spills ~35 VGPRs (outside the column loop's
// critical path) and still runs 7 % faster than at two waves, 206 VGPRs (r4l: 9.06 against 8.44e6 chain-steps/s;
// d = 128 fits 168 without spills either way).  MCMCHIP_RAM_WAVES=2 selects the two-wave build (a bench A/B switch).
template <int G, class M>
__global__ __launch_bounds__(kBlock) void wpc_ram2w2(KernelArgs a) { ram_wave_body<HalfWaveChain<G>, M>(a); }

static int ram_waves_override() {
    static const int v = [] {
        const char* e = getenv("MCMCHIP_RAM_WAVES");
        return e != nullptr ? atoi(e) : 0;
    }();
    return v;
}

constexpr int kRamHalfMaxD = 256;

template <class M>
static hipError_t wpc_ram_step(const KernelArgs& a, hipStream_t st) {
    if (a.s.d <= kRamHalfMaxD) {
        constexpr int cpb = 2 * kChainsPerBlock;
        const dim3 grid((unsigned)((a.s.C + cpb - 1) / cpb));
        const int g = a.s.d <= 128 ? 1 : 2;
        if (ram_waves_override() == 2) {
            mcmc_note_step_kernel("wpc_ram2w2<%d, %s>", g, M::kName);
            if (g == 1) wpc_ram2w2<1, M><<<grid, kBlock, 0, st>>>(a);
            else wpc_ram2w2<2, M><<<grid, kBlock, 0, st>>>(a);
            return hipGetLastError();
        }
        mcmc_note_step_kernel("wpc_ram2<%d, %s>", g, M::kName);
        if (g == 1) wpc_ram2<1, M><<<grid, kBlock, 0, st>>>(a);
        else wpc_ram2<2, M><<<grid, kBlock, 0, st>>>(a);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((a.s.C + kChainsPerBlock - 1) / kChainsPerBlock));
    const int g = wpc_nb_for(a.s.d);
    mcmc_note_step_kernel("wpc_ram<%d, %s>", g, M::kName);
    switch (g) {
        case 2: wpc_ram<2, M><<<grid, kBlock, 0, st>>>(a); break;
        case 4: wpc_ram<4, M><<<grid, kBlock, 0, st>>>(a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mcmc

hipError_t mcmc_wpc_ram_iso(const mcmc::KernelArgs& a, hipStream_t st) { return mcmc::wpc_ram_step<mcmc::IsoDot>(a, st); }
hipError_t mcmc_wpc_ram_normal(const mcmc::KernelArgs& a, hipStream_t st) {
    return mcmc::wpc_ram_step<mcmc::NormalDSL>(a, st);
}
hipError_t mcmc_wpc_ram_absnormal(const mcmc::KernelArgs& a, hipStream_t st) {
    return mcmc::wpc_ram_step<mcmc::AbsNormalDSL>(a, st);
}
hipError_t mcmc_wpc_ram_dist(const mcmc::KernelArgs& a, hipStream_t st) { return mcmc::wpc_ram_step<mcmc::DistDSL>(a, st); }
