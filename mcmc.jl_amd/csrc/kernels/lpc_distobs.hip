// lpc_distobs.hip -- lane-per-chain kernels of y = x * v; y ~ Dist(p1, p2) (benchmarks/benchunits/bare_distribs.jl)
#include "lpc_impl.hpp"
LPC_UNIT(distobs, DistObsDSL, false)
