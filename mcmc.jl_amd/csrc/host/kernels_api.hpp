// kernels_api.hpp -- launch entry points exported by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common.hpp"

namespace mcmc {
struct KernelArgs {
    StepArgs s;
    SamplerArgs sa;
    ModelArgs m;
    ChainState st;
};
}  // namespace mcmc

// The step kernel a launch function dispatched, as "family<template arguments>" (the instance name rocprofv3
// shows, without the namespace): the launch functions record it, mcmc_chains_step_kernel reports it (tests and
// bench.py check which instance ran).  Host-side, thread-local; printf-style.
void mcmc_note_step_kernel(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* mcmc_last_step_kernel();

// lane-per-chain kernels (d <= 32), state [d][ld]
hipError_t mcmc_launch_lpc_step(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_launch_lpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st);
int mcmc_lpc_max_d();
// wave-per-chain kernels (32 < d <= 4096), state [C][ld] (ld = row stride, multiple of 4)
hipError_t mcmc_launch_wpc_step(const mcmc::KernelArgs& a, hipStream_t st);
hipError_t mcmc_launch_wpc_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st);
int mcmc_wpc_max_d();
int mcmc_wpc_ram_max_d();
// regression models on fp64 MFMA, state [d][ld] (+ gradient [d][ld])
hipError_t mcmc_launch_glm_step(const mcmc::KernelArgs& a, hipStream_t st);
// storeLeaps: record the trajectory of the next step (HMC / HMCDA) without moving the chains
hipError_t mcmc_launch_lpc_record(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st);
hipError_t mcmc_launch_wpc_record(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st);
hipError_t mcmc_launch_glm_record(const mcmc::KernelArgs& a, const mcmc::LeapRec& r, hipStream_t st);
hipError_t mcmc_launch_glm_eval(const mcmc::KernelArgs& a, const double* xin, double* lp, double* g, int check,
                                hipStream_t st);
int mcmc_glm_max_d();
// RAM on regression targets, 32 < d <= 1024 (glm_ram_wave.hip): per step the eval kernel and the accept / factor-update
// kernel; u [C][ustride], nz [C], xprop [d][ld], lpp [C] are the device buffers between them.  st2 (may be null):
// a second stream on which half of a large batch runs, forked from and joined back to st by the two events
hipError_t mcmc_launch_glm_ram_wave(const mcmc::KernelArgs& a, double* u, double* nz, double* xprop, double* lpp,
                                    hipStream_t st, hipStream_t st2, hipEvent_t ev_fork, hipEvent_t ev_join);
int64_t mcmc_glm_ram_wave_ustride(int d);
// SeqMC population bookkeeping (seqmc.hip)
hipError_t mcmc_seqmc_weights(int64_t N, double* logW, const double* ll0, double* logtarget, const double* plogtarget,
                              hipStream_t st);
hipError_t mcmc_seqmc_scan(int64_t N, const double* logW, double trigger, double* cp, int32_t* flag, hipStream_t st);
hipError_t mcmc_seqmc_resample(int64_t N, int d, const double* cp, const int32_t* flag, uint64_t seed, uint32_t step,
                               uint32_t target, const double* pars, double* pars_out, const double* logtarget,
                               double* logtarget_out, double* logW, hipStream_t st);
hipError_t mcmc_seqmc_store(int64_t N, int d, const double* pars, const double* logW, double* samples, double* weights,
                            hipStream_t st);
// effective sample size of every (parameter, chain) series of samples [n][d][C] (stats.hip)
hipError_t mcmc_launch_ess(const double* samples, int64_t n, int64_t d, int64_t C, int32_t vtype, int64_t maxlag,
                           int64_t batchlen, double* ess, double* var, hipStream_t st);
// padded coordinate count of the regression kernels; their 16-chain tiles per workgroup
int mcmc_glm_d_pad(int d);
int mcmc_glm_tiles_per_wg(int d);
// the regression kernels' staged-tile image of X and Y (glm_layout.hpp): its size in doubles, and the packing
size_t mcmc_glm_image_doubles(int d, int64_t n);
void mcmc_glm_pack_image(int d, int64_t n, const double* X, const double* Y, const double* B, double* img);
// steps one launch of the regression step kernel may fuse (0: any)
int mcmc_glm_steps_per_launch(int d, int64_t n, int sampler_kind);

hipError_t mcmc_fill_f64(double* p, int64_t n, double v, hipStream_t st);
hipError_t mcmc_fill_f64_strided(double* p, int64_t nb, int64_t w, int64_t stride, double v, hipStream_t st);
hipError_t mcmc_fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t st);
hipError_t mcmc_broadcast_cols(double* dst, int64_t ldd, const double* v, int d, int64_t C, hipStream_t st);
hipError_t mcmc_broadcast_rows(double* dst, int64_t ldr, const double* v, int d, int64_t C, hipStream_t st);
hipError_t mcmc_copy_cols(double* dst, int64_t ldd, const double* src, int64_t lds, int d, int64_t C, hipStream_t st);
// dst[b][s][r] (row stride ldd) <- src[b][r][s] (row stride lds), r < R, s < S; batch strides R*lds / S*ldd
hipError_t mcmc_transpose(double* dst, int64_t ldd, const double* src, int64_t lds, int64_t batch, int64_t R,
                          int64_t S, hipStream_t st);
hipError_t mcmc_detmath(int op, int64_t n, const double* x, const double* y, double* out, hipStream_t st);
hipError_t mcmc_philox(int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out, hipStream_t st);
hipError_t mcmc_mfma_probe(const double* A, const double* B, const double* C, double* D, int nk, hipStream_t st);
