// layout_api.hpp -- per-model entry points of the lane-per-chain and wave-per-chain kernel units
// (lpc_<model>.hip, wpc_<model>.hip); lpc.hip / wpc.hip dispatch on ModelArgs.kind.
#pragma once
#include "../host/kernels_api.hpp"

#define MCMC_LAYOUT_UNIT_DECL(prefix, name)                                                            \
    hipError_t mcmc_##prefix##_step_##name(const mcmc::KernelArgs& a, hipStream_t st);                \
    hipError_t mcmc_##prefix##_eval_##name(const mcmc::KernelArgs& a, const double* xin, double* lp,  \
                                           double* g, int check, hipStream_t st);          \
    hipError_t mcmc_##prefix##_record_##name(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st);
MCMC_LAYOUT_UNIT_DECL(lpc, iso)
MCMC_LAYOUT_UNIT_DECL(lpc, normal)
MCMC_LAYOUT_UNIT_DECL(lpc, absnormal)
MCMC_LAYOUT_UNIT_DECL(lpc, dist)
MCMC_LAYOUT_UNIT_DECL(lpc, distobs)
MCMC_LAYOUT_UNIT_DECL(lpc, ou)
MCMC_LAYOUT_UNIT_DECL(wpc, iso)
MCMC_LAYOUT_UNIT_DECL(wpc, normal)
MCMC_LAYOUT_UNIT_DECL(wpc, absnormal)
MCMC_LAYOUT_UNIT_DECL(wpc, dist)
// lane-per-chain RAM kernels (lpc_ram_a.hip, lpc_ram_b.hip)
hipError_t mcmc_lpc_ram_iso(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_lpc_ram_normal(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_lpc_ram_absnormal(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_lpc_ram_dist(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_lpc_ram_ou(const mcmc::KernelArgs& a, hipStream_t st);      // lpc_ram_ou.hip
// wave-per-chain RAM kernels, 32 < d <= 1024 (wpc_ram.hip)
hipError_t mcmc_wpc_ram_iso(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_wpc_ram_normal(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_wpc_ram_absnormal(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_wpc_ram_dist(const mcmc::KernelArgs& a, hipStream_t st);
