"""ctypes binding of the C ABI declared in include/mcmc_hip.h.

This is the only way the Python host reaches the device: every numeric step
runs in libmcmc_hip.so (HIP kernels for gfx950).  There is no CPU fallback:
if the library is missing or no GPU is present the calls raise.
"""
from __future__ import annotations

import ctypes as ct
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCMCHIP_LIB", os.path.join(_HERE, "libmcmc_hip.so"))

# status codes (mcmc_hip.h)
MCMC_OK = 0
MCMC_E_INVALID_ARG = 1
MCMC_E_INIT_OUT_OF_SUPPORT = 2
MCMC_E_NEEDS_GRADIENT = 3
MCMC_E_HIP = 4
MCMC_E_OOM = 5
MCMC_E_UNSUPPORTED = 6

MODEL_ISO_NORMAL_DOT = 1
MODEL_NORMAL_DSL = 2
MODEL_LOGISTIC = 3
MODEL_LINEAR = 4
MODEL_ABS_NORMAL_DSL = 5
MODEL_DIST_DSL = 6
MODEL_PROBIT = 7
MODEL_DIST_OBS = 8
MODEL_OU = 9

# MCMC_DIST_* (include/mcmc_hip.h)
DISTS = {"Normal": 1, "Uniform": 2, "Weibull": 3, "Beta": 4, "TDist": 5, "Exponential": 6, "Gamma": 7,
         "Cauchy": 8, "LogNormal": 9, "Laplace": 10}

SAMPLER_RWM = 1
SAMPLER_MALA = 2
SAMPLER_HMC = 3
SAMPLER_HMCDA = 4
SAMPLER_RAM = 5

VAR_IMSE = 1
VAR_IPSE = 2
VAR_BM = 3

EXPORTED_SYMBOLS = (
    "mcmc_last_error", "mcmc_abi_version", "mcmc_device_count",
    "mcmc_ctx_create", "mcmc_ctx_destroy", "mcmc_ctx_synchronize",
    "mcmc_model_create", "mcmc_model_destroy", "mcmc_model_eval",
    "mcmc_sampler_validate", "mcmc_runner_validate",
    "mcmc_chains_create", "mcmc_chains_destroy", "mcmc_chains_reset", "mcmc_chains_set_state", "mcmc_chains_fork",
    "mcmc_chains_steps_done", "mcmc_chains_evals",
    "mcmc_chains_ram_factor", "mcmc_chains_tuner_state",
    "mcmc_chains_set_steps_per_launch", "mcmc_chains_set_store_gradients", "mcmc_chains_set_tuner_burnin",
    "mcmc_chains_reserve_outputs",
    "mcmc_chains_launches", "mcmc_chains_step_kernel", "mcmc_chains_store_leaps", "mcmc_run_serialmc",
    "mcmc_group_create", "mcmc_group_destroy", "mcmc_group_size", "mcmc_group_plan", "mcmc_group_chains_create",
    "mcmc_group_chains_destroy", "mcmc_group_chains_reset", "mcmc_group_chains_steps_done",
    "mcmc_group_chains_set_steps_per_launch", "mcmc_group_chains_block", "mcmc_group_run_serialmc",
    "mcmc_group_last_pin_s",
    "mcmc_debug_group_inject_failure",
    "mcmc_seqmc_validate", "mcmc_run_seqmc", "mcmc_stats_ess", "mcmc_debug_detmath", "mcmc_debug_philox",
    "mcmc_debug_mfma_f64", "mcmc_debug_chains_order",
)


class ModelDesc(ct.Structure):
    _fields_ = [
        ("kind", ct.c_int32), ("has_gradient", ct.c_int32), ("d", ct.c_int64),
        ("init", ct.POINTER(ct.c_double)), ("scale", ct.POINTER(ct.c_double)),
        ("mu", ct.c_double), ("sigma", ct.c_double),
        ("prior_sigma", ct.c_double), ("noise_sigma", ct.c_double), ("link_sign", ct.c_double),
        ("n", ct.c_int64), ("X", ct.POINTER(ct.c_double)), ("Y", ct.POINTER(ct.c_double)),
        ("dist", ct.c_int32),
    ]


class SamplerCfg(ct.Structure):
    _fields_ = [
        ("kind", ct.c_int32), ("scale", ct.c_double), ("drift_step", ct.c_double),
        ("n_leaps", ct.c_int64), ("leap_step", ct.c_double),
        ("rate", ct.c_double), ("len", ct.c_double), ("shrinkage", ct.c_double),
        ("t0", ct.c_double), ("step", ct.c_double),
        ("tuner", ct.c_int32), ("adapt_step", ct.c_int64), ("max_step", ct.c_int64),
        ("target_path", ct.c_double), ("target_rate", ct.c_double), ("max_leaps", ct.c_int64),
    ]


class RunnerCfg(ct.Structure):
    _fields_ = [("burnin", ct.c_int64), ("thinning", ct.c_int64), ("len", ct.c_int64)]


class Outputs(ct.Structure):
    _fields_ = [
        ("samples", ct.c_void_p), ("gradients", ct.c_void_p), ("accept_bits", ct.c_void_p),
        ("final_x", ct.c_void_p), ("final_lp", ct.c_void_p), ("on_device", ct.c_int32),
        ("runtime_s", ct.c_double), ("kernel_ms", ct.c_double), ("nkept", ct.c_int64),
    ]


class MCMCError(RuntimeError):
    """Raised for a non-zero status; `.code` is the mcmc_hip.h status."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class OutOfSupportError(MCMCError, AssertionError):
    pass


_lib = None


def load() -> ct.CDLL:
    """Load libmcmc_hip.so; raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmcmc_hip.so not found at {LIB_PATH}: run __graft_entry__.build() "
                          "(make -C mcmc.jl_amd) first")
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's): import it first when present so
    # one HIP runtime serves both torch tensors and this library.  Loading /opt/rocm's runtime first
    # leaves a later torch without devices ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ct.CDLL(LIB_PATH)
    P = ct.c_void_p
    pp = ct.POINTER(ct.c_void_p)
    i64, i32, u64 = ct.c_int64, ct.c_int32, ct.c_uint64
    dp = ct.POINTER(ct.c_double)
    sig = {
        "mcmc_last_error": (ct.c_char_p, []),
        "mcmc_abi_version": (ct.c_int, []),
        "mcmc_device_count": (ct.c_int, [ct.POINTER(ct.c_int)]),
        "mcmc_ctx_create": (ct.c_int, [ct.c_int, pp]),
        "mcmc_ctx_destroy": (ct.c_int, [P]),
        "mcmc_ctx_synchronize": (ct.c_int, [P]),
        "mcmc_model_create": (ct.c_int, [P, ct.POINTER(ModelDesc), pp]),
        "mcmc_model_destroy": (ct.c_int, [P]),
        "mcmc_model_eval": (ct.c_int, [P, i64, dp, dp, dp]),
        "mcmc_sampler_validate": (ct.c_int, [ct.POINTER(SamplerCfg)]),
        "mcmc_runner_validate": (ct.c_int, [ct.POINTER(RunnerCfg)]),
        "mcmc_chains_create": (ct.c_int, [P, ct.POINTER(SamplerCfg), i64, i64, u64, dp, pp]),
        "mcmc_chains_destroy": (ct.c_int, [P]),
        "mcmc_chains_reset": (ct.c_int, [P]),
        "mcmc_chains_set_state": (ct.c_int, [P, dp, dp]),
        "mcmc_chains_fork": (ct.c_int, [P, i64, i64, pp]),
        "mcmc_chains_steps_done": (ct.c_int, [P, ct.POINTER(i64)]),
        "mcmc_chains_evals": (ct.c_int, [P, ct.POINTER(i64)]),
        "mcmc_chains_ram_factor": (ct.c_int, [P, ct.c_void_p]),
        "mcmc_chains_tuner_state": (ct.c_int, [P, ct.c_void_p, ct.c_void_p, ct.c_void_p]),
        "mcmc_chains_set_steps_per_launch": (ct.c_int, [P, i64]),
        "mcmc_chains_set_store_gradients": (ct.c_int, [P, i32]),
        "mcmc_chains_set_tuner_burnin": (ct.c_int, [P, i64]),
        "mcmc_chains_reserve_outputs": (ct.c_int, [P, i64, i32]),
        "mcmc_chains_launches": (ct.c_int, [P, i64, ct.POINTER(i64)]),
        "mcmc_chains_step_kernel": (ct.c_int, [P, ct.c_char_p, i64]),
        "mcmc_chains_store_leaps": (ct.c_int, [P, i64, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p,
                                               ct.c_void_p, ct.c_void_p]),
        "mcmc_run_serialmc": (ct.c_int, [P, ct.POINTER(RunnerCfg), ct.POINTER(Outputs)]),
        "mcmc_group_create": (ct.c_int, [ct.POINTER(ct.c_int32), i32, pp]),
        "mcmc_group_destroy": (ct.c_int, [P]),
        "mcmc_group_size": (ct.c_int, [P, ct.POINTER(i32)]),
        "mcmc_group_plan": (ct.c_int, [i64, i32, ct.POINTER(i64), ct.POINTER(i64)]),
        "mcmc_group_chains_create": (ct.c_int, [P, ct.POINTER(ModelDesc), ct.POINTER(SamplerCfg), i64, i64, u64, dp,
                                                pp]),
        "mcmc_group_chains_destroy": (ct.c_int, [P]),
        "mcmc_group_chains_reset": (ct.c_int, [P]),
        "mcmc_group_chains_steps_done": (ct.c_int, [P, ct.POINTER(i64)]),
        "mcmc_group_chains_set_steps_per_launch": (ct.c_int, [P, i64]),
        "mcmc_group_chains_block": (ct.c_int, [P, i32, pp, ct.POINTER(i64), ct.POINTER(i64)]),
        "mcmc_group_run_serialmc": (ct.c_int, [P, ct.POINTER(RunnerCfg), ct.POINTER(Outputs),
                                               ct.POINTER(ct.c_double)]),
        "mcmc_group_last_pin_s": (ct.c_int, [P, ct.POINTER(ct.c_double)]),
        "mcmc_debug_group_inject_failure": (ct.c_int, [P, i32]),
        "mcmc_seqmc_validate": (ct.c_int, [ct.c_void_p]),
        "mcmc_run_seqmc": (ct.c_int, [ct.POINTER(ct.c_void_p), i32, i64, ct.c_void_p, ct.c_void_p, u64, i32,
                                      ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.POINTER(ct.c_double)]),
        "mcmc_stats_ess": (ct.c_int, [P, ct.c_void_p, i64, i64, i64, i32, i64, i64, i32, ct.c_void_p,
                                      ct.c_void_p]),
        "mcmc_debug_detmath": (ct.c_int, [P, ct.c_int, i64, dp, dp, dp]),
        "mcmc_debug_philox": (ct.c_int, [P, i64, ct.POINTER(ct.c_uint32), ct.POINTER(ct.c_uint32),
                                         ct.POINTER(ct.c_uint32)]),
        "mcmc_debug_mfma_f64": (ct.c_int, [P, ct.c_int, dp, dp, dp, dp]),
        "mcmc_debug_chains_order": (ct.c_int, [P, ct.POINTER(i32), ct.POINTER(i32)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(status: int) -> None:
    if status != MCMC_OK:
        msg = load().mcmc_last_error().decode(errors="replace")
        if status == MCMC_E_INIT_OUT_OF_SUPPORT:
            raise OutOfSupportError(status, msg)
        raise MCMCError(status, msg)


def dptr(a):
    """double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(ct.POINTER(ct.c_double))
