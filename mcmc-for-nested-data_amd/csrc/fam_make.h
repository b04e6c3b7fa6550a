// fam_make.h -- the family functors from a context's model constants (nmc_create's
// ll_consts), shared by the family translation units (fam_*.hip) and the sweep-kernel ones
// (sweep_*.hip).
#pragma once
#include <vector>

#include "families.h"

template <int NF>
static inline FamLinreg<NF> make_linreg(const std::vector<double>& c) {
  FamLinreg<NF> f{};
  f.intercept = (int)c[1];
  f.sigma_known = c[2];
  f.log_sigma_known = c.size() > 3 ? c[3] : 0.0;
  f.inv_s2_known = c[2] > 0 ? 1.0 / (c[2] * c[2]) : 0.0;
  return f;
}

template <int NF>
static inline FamGaussMean<NF> make_gauss(const std::vector<double>& c) {
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

template <int NF>
static inline FamLogistic<NF> make_logistic(const std::vector<double>& c) {
  FamLogistic<NF> f{};
  f.intercept = (int)c[1];
  return f;
}
