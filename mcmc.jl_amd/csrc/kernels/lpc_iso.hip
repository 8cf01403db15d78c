// lpc_iso.hip -- lane-per-chain kernels of model(v -> -dot(v,v)) (README.md:60,63)
#include "lpc_impl.hpp"
LPC_UNIT(iso, IsoDot, true)
