// glm_mala1.hip -- the single-slice regression MALA kernels (glm_mala1<NM>, glm.hip) in a translation unit of
// their own, built WITH machine LICM: the tile loop's fp64 polynomial constants and LDS addresses are hoisted
// out of it (these one-step kernels have the registers for them).  glm.o is built without machine LICM, which
// there keeps hoisted constants from pinning registers across the step loops of the other kernels (Makefile).
#define GLM_MALA1_UNIT 1
#include "glm.hip"
