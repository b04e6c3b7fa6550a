// softplus.h -- numpy.logaddexp(0, eta) in plain IEEE fp64 operations (host and device).
//
// The logistic likelihood (cfg 5, posteriorSampling.py:61-102 with y eta - logaddexp(0, eta))
// spends almost all of its per-row work here: the library's exp() and log1p() cost 181
// VALU instructions on gfx950 (log1p alone 135: a double-double evaluation), against ~12
// for the rest of the row.  This restates the function with one range-reduced exp and one
// range-reduced log1p:
//
//   logaddexp(0, eta) = max(eta, 0) + log1p(exp(-|eta|))
//   e = exp(x), x = -|eta| in [-746, 0]: x = k ln2 + r (Cody-Waite, |r| <= ln2 / 2),
//       exp(r) by its Taylor series to r^13 (truncation < 5e-18 relative), scaled by 2^k
//   log1p(e), e in [0, 1]: e > 1/2 uses 1 + e = 2 (1 + (e - 1) / 2) (e - 1 exact), so the
//       argument f of log1p(f) lies in (-0.25, 0.5]; log1p(f) = 2 atanh(s),
//       s = f / (2 + f), |s| <= 0.2: 2 s + s^3 (2/3 + s^2 (2/5 + ... + s^20 2/23))
//       (the first omitted term is < 1e-18 of the result)
//
// Every operation is an IEEE-rounded add / multiply / fma / divide, rint or ldexp, so the
// host and the device compute the same bits (tests/test_softplus.py checks the host form
// against a 50-digit reference: within 2.5 ulp of the exact value everywhere, mean 0.35, and numpy's
// special values: +-inf, NaN, logaddexp(0, 0) = ln 2 exactly).  Built-in and user
// families share it (nmc_logaddexp0), so they stay bit-identical.
#pragma once
#ifndef __HIPCC_RTC__
#include <math.h>
#endif

#ifndef NMC_HD
#define NMC_HD __host__ __device__ __forceinline__
#endif

NMC_HD double nmc_exp_neg(double x) {   // exp(x) for x <= 0 (NaN propagates)
  if (x < -746.0) x = -746.0;          // (exp underflows to 0 below -745.13; NaN compares false)
  const double kd = rint(x * 1.4426950408889634);                 // x / ln 2
  double r = fma(kd, -6.93147180369123816490e-01, x);             // ln 2 high part
  r = fma(kd, -1.90821492927058770002e-10, r);                    // ln 2 low part
  double p = 1.6059043836821613e-10;                              // 1/13!
  p = fma(p, r, 2.08767569878681e-09);
  p = fma(p, r, 2.505210838544172e-08);
  p = fma(p, r, 2.755731922398589e-07);
  p = fma(p, r, 2.7557319223985893e-06);
  p = fma(p, r, 2.48015873015873e-05);
  p = fma(p, r, 0.0001984126984126984);
  p = fma(p, r, 0.001388888888888889);
  p = fma(p, r, 0.008333333333333333);
  p = fma(p, r, 0.041666666666666664);
  p = fma(p, r, 0.16666666666666666);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  // (a NaN x leaves kd NaN: it is never converted to int -- p is NaN, and so is the result)
  return ldexp(p, kd == kd ? (int)kd : 0);
}

NMC_HD double nmc_log1p_unit(double e) {   // log1p(e) for e in [0, 1] (NaN propagates)
  const bool big = e > 0.5;                        // (e - 1 is then exact: Sterbenz)
  const double f = big ? (e - 1.0) * 0.5 : e;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double q = 0.08695652173913043;                                 // 2/23
  q = fma(q, z, 0.09523809523809523);                             // 2/21
  q = fma(q, z, 0.10526315789473684);                             // 2/19
  q = fma(q, z, 0.11764705882352941);                             // 2/17
  q = fma(q, z, 0.13333333333333333);                             // 2/15
  q = fma(q, z, 0.15384615384615385);                             // 2/13
  q = fma(q, z, 0.18181818181818182);                             // 2/11
  q = fma(q, z, 0.2222222222222222);                              // 2/9
  q = fma(q, z, 0.2857142857142857);                              // 2/7
  q = fma(q, z, 0.4);                                             // 2/5
  q = fma(q, z, 0.6666666666666666);                              // 2/3
  const double l = fma(s * z, q, 2.0 * s);                        // 2 atanh(s)
  return big ? 0.6931471805599453 + (l + 2.3190468138462996e-17) : l;   // ln 2 in two parts
}

// numpy.logaddexp(0, eta) (npy_logaddexp: x == y -> x + ln 2, NaN propagating)
NMC_HD double nmc_softplus(double eta) {
  const double m = eta > 0.0 ? eta : 0.0;
  const double r = m + nmc_log1p_unit(nmc_exp_neg(-fabs(eta)));
  return eta == 0.0 ? 0.6931471805599453 : r;
}
