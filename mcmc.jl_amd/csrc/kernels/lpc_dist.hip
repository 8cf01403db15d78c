// lpc_dist.hip -- lane-per-chain kernels of v ~ Dist(p1, p2) (MCMCDerivRules.jl:56-104)
#include "lpc_impl.hpp"
LPC_UNIT(dist, DistDSL, false)
