// lpc_ram_ou.hip -- lane-per-chain RAM kernels (src/samplers/RAM.jl) of the Ornstein-Uhlenbeck model
// (examples/ornstein.jl:34 runs it under RAM())
#include "lpc_impl.hpp"
LPC_RAM_UNIT(ou, OUDSL)
