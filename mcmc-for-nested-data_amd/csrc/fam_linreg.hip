// fam_linreg.hip -- step/LL kernels instantiated for the Gaussian linear-regression
// family (example/regression.py:53-67; cfg 1/3/4).
#include "fam_ops.h"

template <int NF>
static FamLinreg<NF> make_linreg(const std::vector<double>& c) {
  FamLinreg<NF> f{};
  f.intercept = (int)c[1];
  f.sigma_known = c[2];
  f.log_sigma_known = c.size() > 3 ? c[3] : 0.0;
  f.inv_s2_known = c[2] > 0 ? 1.0 / (c[2] * c[2]) : 0.0;
  return f;
}

NMC_DEFINE_FAMILY_CALL(nmc_call_linreg, make_linreg)
