// wpc_normal.hip -- wave-per-chain kernels of v ~ Normal(mu, sigma)
#include "wpc_impl.hpp"
WPC_UNIT(normal, NormalDSL, false)
