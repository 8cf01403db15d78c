// wpc_absnormal.hip -- wave-per-chain kernels of y = abs(x); y ~ Normal(mu, sigma)
#include "wpc_impl.hpp"
WPC_UNIT(absnormal, AbsNormalDSL, false)
