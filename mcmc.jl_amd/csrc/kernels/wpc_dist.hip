// wpc_dist.hip -- wave-per-chain kernels of v ~ Dist(p1, p2)
#include "wpc_impl.hpp"
WPC_UNIT(dist, DistDSL, false)
