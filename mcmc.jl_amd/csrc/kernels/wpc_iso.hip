// wpc_iso.hip -- wave-per-chain kernels of model(v -> -dot(v,v))
#include "wpc_impl.hpp"
WPC_UNIT(iso, IsoDot, true)
