// sweep_gauss_mean.hip -- nmc_k_sweep instantiated for the gauss_mean family (sweep_ops.h).
#include "sweep_ops.h"

NMC_DEFINE_SWEEP_CALL(nmc_sweep_gauss_mean, make_gauss)
