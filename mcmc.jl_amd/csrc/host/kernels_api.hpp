// kernels_api.hpp -- launch entry points exported by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common.hpp"

namespace mcmc {
struct LpcArgs {
    StepArgs s;
    SamplerArgs sa;
    ModelArgs m;
    ChainState st;
};
}  // namespace mcmc

hipError_t mcmc_launch_lpc_step(const mcmc::LpcArgs& a, hipStream_t st);
hipError_t mcmc_launch_lpc_eval(const mcmc::LpcArgs& a, const double* xin, int64_t ldin, double* lp, double* g,
                                int check, hipStream_t st);
int mcmc_lpc_max_d();

hipError_t mcmc_fill_f64(double* p, int64_t n, double v, hipStream_t st);
hipError_t mcmc_fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t st);
hipError_t mcmc_broadcast_cols(double* dst, int64_t ldd, const double* v, int d, int64_t C, hipStream_t st);
hipError_t mcmc_copy_cols(double* dst, int64_t ldd, const double* src, int64_t lds, int d, int64_t C, hipStream_t st);
hipError_t mcmc_transpose(double* dst, const double* src, int64_t batch, int64_t R, int64_t S, hipStream_t st);
hipError_t mcmc_detmath(int op, int64_t n, const double* x, const double* y, double* out, hipStream_t st);
hipError_t mcmc_philox(int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out, hipStream_t st);
