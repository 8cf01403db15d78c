// lpc_ou.hip -- lane-per-chain kernels of the Ornstein-Uhlenbeck model (examples/ornstein.jl:19-30; models.hpp OUDSL)
#include "lpc_impl.hpp"
LPC_UNIT(ou, OUDSL, false)
