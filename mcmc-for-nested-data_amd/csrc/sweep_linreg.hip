// sweep_linreg.hip -- nmc_k_sweep instantiated for the linreg family (sweep_ops.h).
#include "sweep_ops.h"

NMC_DEFINE_SWEEP_CALL(nmc_sweep_linreg, make_linreg)
