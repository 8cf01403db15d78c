// lpc_ram_b.hip -- lane-per-chain RAM kernels (src/samplers/RAM.jl) of the abs-Normal and v ~ Dist targets
#include "lpc_impl.hpp"
LPC_RAM_UNIT(absnormal, AbsNormalDSL)
LPC_RAM_UNIT(dist, DistDSL)
