// fam_gauss_mean.hip -- step/LL kernels instantiated for the Gaussian-means family
// (example/distribution.py:18-24; cfg 2).
#include "fam_ops.h"
#include "fam_make.h"

NMC_DEFINE_FAMILY_CALL(nmc_call_gauss_mean, make_gauss)
