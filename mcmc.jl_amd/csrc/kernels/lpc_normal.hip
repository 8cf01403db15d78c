// lpc_normal.hip -- lane-per-chain kernels of v ~ Normal(mu, sigma) (README.md:67-72)
#include "lpc_impl.hpp"
LPC_UNIT(normal, NormalDSL, true)
