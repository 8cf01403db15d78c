// lpc_absnormal.hip -- lane-per-chain kernels of y = abs(x); y ~ Normal(mu, sigma) (README.md:246-251)
#include "lpc_impl.hpp"
LPC_UNIT(absnormal, AbsNormalDSL, false)
