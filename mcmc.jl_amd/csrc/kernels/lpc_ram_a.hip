// lpc_ram_a.hip -- lane-per-chain RAM kernels (src/samplers/RAM.jl) of the iso-Normal and Normal targets
#include "lpc_impl.hpp"
LPC_RAM_UNIT(iso, IsoDot)
LPC_RAM_UNIT(normal, NormalDSL)
