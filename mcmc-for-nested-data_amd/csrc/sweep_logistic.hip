// sweep_logistic.hip -- nmc_k_sweep instantiated for the logistic family (sweep_ops.h).
#include "sweep_ops.h"

NMC_DEFINE_SWEEP_CALL(nmc_sweep_logistic, make_logistic)
