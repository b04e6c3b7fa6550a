// fam_gauss_mean.hip -- step/LL kernels instantiated for the Gaussian-means family
// (example/distribution.py:18-24; cfg 2).
#include "fam_ops.h"

template <int NF>
static FamGaussMean<NF> make_gauss(const std::vector<double>& c) {
  FamGaussMean<NF> f{};
  f.bad = 0;
  for (int j = 0; j < NF; ++j) {
    f.sd[j] = c[j];
    f.lsd[j] = c[NF + j];
    f.isd2[j] = 1.0 / (c[j] * c[j]);
    if (!(c[j] > 0.0)) f.bad = 1;
  }
  return f;
}

NMC_DEFINE_FAMILY_CALL(nmc_call_gauss_mean, make_gauss)
