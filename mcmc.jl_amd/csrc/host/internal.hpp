// internal.hpp -- host-runtime entry points shared between runtime.cpp and group.cpp (not part of the C ABI).
#pragma once
#include <stdint.h>

#include <string>

#include "../../../include/mcmc_hip.h"

// set the calling thread's mcmc_last_error() message; returns code
int mcmc_set_error(int code, const std::string& msg);
// mcmc_run_serialmc with host outputs of a larger batch: rows ldc chains apart (runtime.cpp)
int mcmc_run_serialmc_ld(mcmc_chains* c, const mcmc_runner_cfg* r, mcmc_outputs* out, int64_t ldc, double* copy_s);
