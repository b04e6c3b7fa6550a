// special.h -- device log-densities and special functions of the hot path.
//
// * nmc_norm_logpdf  : scipy.stats.norm(loc, scale).logpdf as the reference calls it
//   for proposals and hyper-priors (posteriorSampling.py:291-294, :500-502):
//   y = (x-loc)/scale; (-(y*y)/2 - log(sqrt(2 pi))) - log(scale); NaN if !(scale>0).
// * nmc_prior_logpdf : the scipy frozen priors usable with none/complete pooling.
// * nmc_igamci       : scipy.special.gammainccinv(a, q), the inverse-CDF the
//   reference's invgamma.rvs uses (posteriorSampling.py:498 -> scipy
//   _distn_infrastructure rvs: 1/gammainccinv(a, U) * scale); replay mode only.
// * nmc_pairwise_sum : numpy's float64 add.reduce order (numpy.mean / numpy.sum of
//   posteriorSampling.py:485, :494), so hyper means match the reference bit for bit.
#pragma once
#ifndef __HIPCC_RTC__   // (hiprtc, user families: the runtime provides these)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#endif

#include "../../include/nestmc.h"

#define NMC_LOG_C 0.9189385332046727            // log(sqrt(2*pi)) as scipy computes it
#define NMC_LOG_PI 1.1447298858494002
#define NMC_LN2 0.6931471805599453

__device__ __forceinline__ double nmc_nan() { return __builtin_nan(""); }

// norm.logpdf with log(scale) precomputed by the caller (lsd = log(scale)).
__device__ __forceinline__ double nmc_norm_logpdf(double x, double loc, double scale,
                                                  double lsd) {
  const double y = (x - loc) / scale;
  if (!(scale > 0.0) || isnan(y)) return nmc_nan();
  return (-(y * y) / 2.0 - NMC_LOG_C) - lsd;
}

// The same with the reciprocal of the scale precomputed (isd = 1/scale; <= 1 ulp
// from the division form): the partial-pooling priors on the decision's path.
__device__ __forceinline__ double nmc_norm_logpdf_r(double x, double loc, double scale,
                                                    double isd, double lsd) {
  const double y = (x - loc) * isd;
  if (!(scale > 0.0) || isnan(y)) return nmc_nan();
  return (-(y * y) / 2.0 - NMC_LOG_C) - lsd;
}

__device__ __forceinline__ double nmc_xlogy(double c, double y) {
  if (c == 0.0 && !isnan(y)) return 0.0;
  return c * log(y);
}

// prm[8] = {loc, scale, shape, gammaln(shape), log(scale), 0,0,0} (host computes
// gammaln and log(scale) with scipy/numpy, so those terms are bit-identical): scipy rv_continuous.logpdf:
// x' = (x-loc)/scale; NaN if bad args / NaN x'; -inf outside the support;
// else _logpdf(x') - log(scale)   (scipy/stats/_distn_infrastructure.py logpdf).
__device__ inline double nmc_prior_logpdf(int fam, const double* prm, double x) {
  const double loc = prm[0], scale = prm[1], a = prm[2], lga = prm[3], ls = prm[4];
  const double y = (x - loc) / scale;
  if (!(scale > 0.0) || isnan(y)) return nmc_nan();
  const double ninf = -__builtin_inf();
  switch (fam) {
    case NMC_PRIOR_NORM:
      return (-(y * y) / 2.0 - NMC_LOG_C) - ls;
    case NMC_PRIOR_GAMMA:
      if (!(y >= 0.0)) return ninf;
      return ((nmc_xlogy(a - 1.0, y) - y) - lga) - ls;
    case NMC_PRIOR_UNIFORM:
      if (!(y >= 0.0 && y <= 1.0)) return ninf;
      return 0.0 - ls;
    case NMC_PRIOR_EXPON:
      if (!(y >= 0.0)) return ninf;
      return -y - ls;
    case NMC_PRIOR_HALFNORM:
      if (!(y >= 0.0)) return ninf;
      return (0.5 * log(2.0 / 3.141592653589793) - y * y / 2.0) - ls;
    case NMC_PRIOR_CAUCHY:
      return (-NMC_LOG_PI - log1p(y * y)) - ls;
    case NMC_PRIOR_LAPLACE:
      return log(0.5 * exp(-fabs(y))) - ls;
    case NMC_PRIOR_LOGNORM: {          // scipy _lognorm_logpdf, open support
      if (!(y > 0.0)) return ninf;
      const double lx = log(y);
      return (-(lx * lx) / (2.0 * (a * a)) - log(a * y * 2.5066282746310002)) - ls;
    }
    case NMC_PRIOR_INVGAMMA:
      if (!(y > 0.0)) return ninf;
      return ((-(a + 1.0) * log(y) - lga) - 1.0 / y) - ls;
    default:
      return nmc_nan();
  }
}

// ---------------------------------------------------------------------------
// numpy pairwise summation of n values get(i) (numpy/_core/src/umath/loops_utils.h)
// ---------------------------------------------------------------------------
template <class Get>
__device__ __forceinline__ double nmc_pairwise_leaf(const Get& get, int s, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += get(s + i);
    return res;
  }
  double r0 = get(s + 0), r1 = get(s + 1), r2 = get(s + 2), r3 = get(s + 3);
  double r4 = get(s + 4), r5 = get(s + 5), r6 = get(s + 6), r7 = get(s + 7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += get(s + i + 0); r1 += get(s + i + 1); r2 += get(s + i + 2); r3 += get(s + i + 3);
    r4 += get(s + i + 4); r5 += get(s + i + 5); r6 += get(s + i + 6); r7 += get(s + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += get(s + i);
  return res;
}

// numpy's recursion n -> (n2, n - n2), n2 = n/2 rounded down to a multiple of 8,
// unrolled at compile time to depth D (exact numpy order for n <= 128 * 2^D; deeper
// blocks fall back to the 8-accumulator leaf).  No stack, no scratch memory.
template <int D, class Get>
__device__ __forceinline__ double nmc_pairwise_rec(const Get& get, int s, int n) {
  if constexpr (D == 0) {
    return nmc_pairwise_leaf(get, s, n);
  } else {
    if (n <= 128) return nmc_pairwise_leaf(get, s, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    const double l = nmc_pairwise_rec<D - 1>(get, s, n2);
    return l + nmc_pairwise_rec<D - 1>(get, s + n2, n - n2);
  }
}

template <class Get>
__device__ __forceinline__ double nmc_pairwise_sum(const Get& get, int n) {
  return nmc_pairwise_rec<3>(get, 0, n);   // exact numpy order up to 1024 groups
}

// ---------------------------------------------------------------------------
// regularised incomplete gamma and its inverse (replay mode: the reference's U)
// ---------------------------------------------------------------------------
// P(a,x), Q(a,x): series for x < a+1, Lentz continued fraction otherwise.
__device__ inline void nmc_gamma_pq(double a, double x, double lga, double* P, double* Q) {
  if (!(x > 0.0)) { *P = 0.0; *Q = 1.0; return; }
  if (isinf(x)) { *P = 1.0; *Q = 0.0; return; }
  const double lpre = a * log(x) - x - lga;
  if (x < a + 1.0) {
    double ap = a, term = 1.0 / a, sum = term;
    for (int n = 0; n < 2000; ++n) {
      ap += 1.0;
      term *= x / ap;
      sum += term;
      if (fabs(term) < fabs(sum) * 1e-17) break;
    }
    const double p = sum * exp(lpre);
    *P = p;
    *Q = 1.0 - p;
  } else {
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 2000; ++i) {
      const double an = -i * (i - a);
      b += 2.0;
      d = an * d + b;
      if (fabs(d) < tiny) d = tiny;
      c = b + an / c;
      if (fabs(c) < tiny) c = tiny;
      d = 1.0 / d;
      const double del = d * c;
      h *= del;
      if (fabs(del - 1.0) < 1e-17) break;
    }
    const double q = exp(lpre) * h;
    *Q = q;
    *P = 1.0 - q;
  }
}

// Acklam's inverse normal CDF (|rel err| < 1.2e-9): initial guess only.
__device__ inline double nmc_ndtri_approx(double p) {
  const double a1 = -3.969683028665376e+01, a2 = 2.209460984245205e+02,
               a3 = -2.759285104469687e+02, a4 = 1.383577518672690e+02,
               a5 = -3.066479806614716e+01, a6 = 2.506628277459239e+00;
  const double b1 = -5.447609879822406e+01, b2 = 1.615858368580409e+02,
               b3 = -1.556989798598866e+02, b4 = 6.680131188771972e+01,
               b5 = -1.328068155288572e+01;
  const double c1 = -7.784894002430293e-03, c2 = -3.223964580411365e-01,
               c3 = -2.400758277161838e+00, c4 = -2.549732539343734e+00,
               c5 = 4.374664141464968e+00, c6 = 2.938163982698783e+00;
  const double d1 = 7.784695709041462e-03, d2 = 3.224671290700398e-01,
               d3 = 2.445134137142996e+00, d4 = 3.754408661907416e+00;
  if (p < 0.02425) {
    const double q = sqrt(-2.0 * log(p));
    return (((((c1 * q + c2) * q + c3) * q + c4) * q + c5) * q + c6) /
           ((((d1 * q + d2) * q + d3) * q + d4) * q + 1.0);
  }
  if (p > 1.0 - 0.02425) {
    const double q = sqrt(-2.0 * log(1.0 - p));
    return -(((((c1 * q + c2) * q + c3) * q + c4) * q + c5) * q + c6) /
           ((((d1 * q + d2) * q + d3) * q + d4) * q + 1.0);
  }
  const double q = p - 0.5, r = q * q;
  return (((((a1 * r + a2) * r + a3) * r + a4) * r + a5) * r + a6) * q /
         (((((b1 * r + b2) * r + b3) * r + b4) * r + b5) * r + 1.0);
}

// x such that Q(a, x) = q (scipy.special.gammainccinv).  Safeguarded Halley on
// whichever of P = 1-q / Q = q is the smaller tail, bracketed, to full precision.
__device__ inline double nmc_igamci(double a, double q, double lga) {
  if (isnan(q) || isnan(a) || !(a > 0.0) || q < 0.0 || q > 1.0) return nmc_nan();
  if (q == 0.0) return __builtin_inf();
  if (q == 1.0) return 0.0;
  const bool useq = q < 0.5;
  const double target = useq ? q : 1.0 - q;
  // Wilson-Hilferty start, small-x series start for small shape / lower tail
  const double z = nmc_ndtri_approx(1.0 - q);   // lower-tail quantile of the result
  double x = a * pow(1.0 - 1.0 / (9.0 * a) + z / (3.0 * sqrt(a)), 3.0);
  if (!(x > 0.0) || a < 1.0) {
    const double p = 1.0 - q;
    const double xs = exp((log(p) + lgamma(a + 1.0)) / a);
    if (!(x > 0.0) || (xs < a && p < 0.5)) x = xs;
    if (!(x > 0.0)) x = 1e-300;
  }
  double lo = 0.0, hi = __builtin_inf();
  for (int it = 0; it < 200; ++it) {
    double P, Q;
    nmc_gamma_pq(a, x, lga, &P, &Q);
    const double f = useq ? (Q - target) : (P - target);  // Q decreasing, P increasing
    // update bracket
    const bool too_big = useq ? (f < 0.0) : (f > 0.0);
    if (too_big) hi = x; else lo = x;
    if (f == 0.0) break;
    const double dens = exp((a - 1.0) * log(x) - x - lga);     // dP/dx
    const double fp = useq ? -dens : dens;
    double xn;
    if (fp != 0.0 && isfinite(fp)) {
      const double t = f / fp;
      const double corr = 1.0 - 0.5 * t * ((a - 1.0) / x - 1.0);
      xn = x - ((corr > 0.1 && corr < 10.0) ? t / corr : t);
    } else {
      xn = nmc_nan();
    }
    if (!(xn > lo && xn < hi)) xn = isinf(hi) ? (lo > 0.0 ? 2.0 * lo : 2.0 * x) : 0.5 * (lo + hi);
    if (fabs(xn - x) <= 4e-16 * fabs(x)) { x = xn; break; }
    x = xn;
  }
  return x;
}
