// fam_logistic.hip -- step/LL kernels instantiated for the Bernoulli-logit family
// (cfg 5's 8-parameter logistic model).
#include "fam_ops.h"
#include "fam_make.h"

NMC_DEFINE_FAMILY_CALL(nmc_call_logistic, make_logistic)
