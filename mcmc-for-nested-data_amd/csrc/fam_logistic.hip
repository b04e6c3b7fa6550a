// fam_logistic.hip -- step/LL kernels instantiated for the Bernoulli-logit family
// (cfg 5's 8-parameter logistic model).
#include "fam_ops.h"

template <int NF>
static FamLogistic<NF> make_logistic(const std::vector<double>& c) {
  FamLogistic<NF> f{};
  f.intercept = (int)c[1];
  return f;
}

NMC_DEFINE_FAMILY_CALL(nmc_call_logistic, make_logistic)
