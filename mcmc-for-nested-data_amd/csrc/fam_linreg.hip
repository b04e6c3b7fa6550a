// fam_linreg.hip -- step/LL kernels instantiated for the Gaussian linear-regression
// family (example/regression.py:53-67; cfg 1/3/4).
#include "fam_ops.h"
#include "fam_make.h"

NMC_DEFINE_FAMILY_CALL(nmc_call_linreg, make_linreg)
