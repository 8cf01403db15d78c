"""mcmchip -- MI355X (gfx950) many-chain MCMC inner loop behind MCMC.jl's API.

Host mirror of the reference's model x sampler x runner interface; every step
runs in the HIP kernels of libmcmc_hip.so through the C ABI (include/mcmc_hip.h).
"""
from ._lib import MCMCError, OutOfSupportError, load as load_library, LIB_PATH  # noqa: F401
from .api import (  # noqa: F401
    IsoNormalDot, NormalDSL, AbsNormalDSL, DistDSL, DistObsDSL, LogisticRegression, LinearRegression, ProbitRegression, vaso_data,
    OrnsteinUhlenbeck, ou_series,
    MCMCLikelihoodModel, model,
    RWM, MALA, HMC, HMCDA, RAM, EmpMCTuner, EmpiricalMCMCTuner, SerialMC, MCMCTask, MCMCChain,
    run, prun, resume, reset, srand, drawn_key, device_count,
)
from .seqmc import SeqMC, SeqMCChain, run_seqmc, resume_seqmc  # noqa: F401
from . import stats  # noqa: F401
from .stats import acceptance, mean, var, ess, actime, mcvar_iid, mcvar_bm, mcvar_imse, mcvar_ipse  # noqa: F401

MCMCLikModel = MCMCLikelihoodModel
__version__ = "0.1.0"
