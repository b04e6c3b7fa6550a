// families.h -- device log-likelihood families (the user logLikelihoodFunction of
// posteriorSampling.py:61-102, restated per model the reference ships/benchmarks).
//
// A family is evaluated chain-on-lane: every lane of a wavefront holds ONE chain's
// parameter values in registers while the whole wave walks the same observation
// rows, so row loads are wave-uniform (scalar loads) and each 16-72 byte row feeds
// 64 chains.  Per family:
//   Reg      per-lane resolved parameters (built once per group step by prepare())
//   accum()  per-observation contribution to NACC fp64 accumulators
//   finish() group log-likelihood from the accumulators and the row count
//   obs_ll() one observation's log-likelihood in the reference's own formula
//            (StepMethod.logLikelihood rows, posteriorSampling.py:656-659)
//   gconst()/finish_fast() the same group LL with the per-group constant hoisted
//            out of the decision's critical path (<= 1 ulp from finish())
// Algebra is restructured (e.g. sum r^2 then scale once) but no fast-math: NaN and
// inf propagate exactly as the reference's MH branches (:347-367) need.
#pragma once
#ifndef __HIPCC_RTC__   // (hiprtc, user families: the runtime provides these)
#include <hip/hip_runtime.h>
#include <math.h>
#endif

#include "special.h"
#include "softplus.h"

#define NMC_MAXP 16

// numpy.logaddexp(0, eta) (npy_logaddexp: x == y -> x + ln 2; else max + log1p(exp(-|x - y|)),
// NaN propagating), branch-free: one range-reduced exp and one range-reduced log1p per lane
// whatever the sign of eta (softplus.h: ~50 VALU instructions against 181 for the library's
// exp + log1p, within 2.5 ulp).  +-inf give inf / 0, NaN gives NaN, eta == 0 gives ln 2.
__device__ __forceinline__ double nmc_logaddexp0(double eta) { return nmc_softplus(eta); }

// ---------------------------------------------------------------------------
// Gaussian linear regression (example/regression.py:53-67; cfg 3/4 with sigma=1):
//   rows [x_1..x_K, y] (K = NF-1); params [b0 if intercept, b_1..b_K, sigma if
//   sigma is sampled].  ll_i = norm(loc=y, scale=sigma).logpdf(yhat),
//   group LL = -0.5 sum (yhat-y)^2 / sigma^2 - n (log sqrt(2 pi) + log sigma).
// ---------------------------------------------------------------------------
template <int NF>
struct FamLinreg {
  static constexpr int NFIELDS = NF;
  static constexpr int MAXP = NF + 1;   // parameters a row of NF fields can involve
  static constexpr int NACC = 1;
  static constexpr int K = NF - 1;
  static constexpr bool ASM_ROWS = NF == 2;   // {x, y} rows: hand-written LDS row loop
  int intercept;
  double sigma_known;   // > 0: fixed noise sd; else sigma is the last parameter
  double log_sigma_known;
  double inv_s2_known;  // 1 / sigma_known^2

  struct Reg { double b0, b[K > 0 ? K : 1], sig; };

  __device__ __forceinline__ Reg prepare(const double* th) const {
    Reg r;
    r.b0 = intercept ? th[0] : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) r.b[j] = intercept ? th[j + 1] : th[j];
    r.sig = sigma_known > 0.0 ? sigma_known : (intercept ? th[K + 1] : th[K]);
    return r;
  }
  // residual e = (b0 - y) + sum_j x_j b_j, accumulated with fmas from the intercept side
  // (every likelihood path -- LDS asm loop, pair loop, scalar loop -- forms the same e)
  __device__ __forceinline__ void accum(const Reg& r, const double* __restrict__ row,
                                        double* acc) const {
    double e = r.b0 - row[K];
#pragma unroll
    for (int j = 0; j < K; ++j) e = fma(row[j], r.b[j], e);
    acc[0] = fma(e, e, acc[0]);
  }
  // N rows, written stage by stage so the N dependence chains interleave
  template <int N>
  __device__ __forceinline__ void accumN(const Reg& r, const double* __restrict__ rows,
                                         double (&a)[4][NACC]) const {
    double e[N];
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = r.b0 - rows[i * NF + K];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i) e[i] = fma(rows[i * NF + j], r.b[j], e[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) a[i & 3][0] = fma(e[i], e[i], a[i & 3][0]);
  }
  __device__ __forceinline__ double finish(const Reg& r, const double* acc, long n) const {
    if (n == 0) return 0.0;
    const double s = r.sig;
    if (!(s > 0.0)) return nmc_nan();
    const double ls = sigma_known > 0.0 ? log_sigma_known : log(s);
    return -0.5 * (acc[0] / (s * s)) - (double)n * (NMC_LOG_C + ls);
  }
  // Per-group constant of finish_fast (once per launch): n (log sqrt(2 pi) + log sigma).
  __device__ __forceinline__ double gconst(long n) const {
    return sigma_known > 0.0 ? (double)n * (NMC_LOG_C + log_sigma_known) : 0.0;
  }
  // the family's constants held in registers for a persistent launch (a local copy of the
  // family): the step kernel's loop is built without machine loop-invariant code motion, so
  // 1 / sigma^2 (finish_fast) and the layout words prepare() branches on would otherwise be
  // scalar loads of the kernel argument on the decision's and the restart's critical paths
  __device__ __forceinline__ void hold() {
    asm volatile("" : "+v"(inv_s2_known), "+v"(sigma_known), "+v"(intercept));
  }
  // finish() on the decision's critical path: known sigma -> one multiply-add.
  __device__ __forceinline__ double finish_fast(const Reg& r, const double* acc, long n,
                                                double gc) const {
    if (n == 0) return 0.0;
    if (sigma_known > 0.0) return -0.5 * (acc[0] * inv_s2_known) - gc;
    return finish(r, acc, n);
  }
  __device__ __forceinline__ double obs_ll(const Reg& r, const double* __restrict__ row) const {
    double yh = 0.0;
    if (intercept) yh = r.b0;                        // numpy.sum(X * beta, axis=1)
#pragma unroll
    for (int j = 0; j < K; ++j) yh = yh + row[j] * r.b[j];
    const double s = r.sig;
    if (!(s > 0.0)) return nmc_nan();
    const double t = (yh - row[K]) / s;
    const double ls = sigma_known > 0.0 ? log_sigma_known : log(s);
    return (-(t * t) / 2.0 - NMC_LOG_C) - ls;
  }
};

// ---------------------------------------------------------------------------
// Gaussian means (example/distribution.py:18-24): rows [m_0..m_{P-1}], one field
// per parameter; ll_i = sum_j norm(m_j, sd_j).logpdf(theta_j).
// ---------------------------------------------------------------------------
template <int NF>
struct FamGaussMean {
  static constexpr int NFIELDS = NF;
  static constexpr bool ASM_ROWS = false;
  static constexpr int MAXP = NF + 1;   // parameters a row of NF fields can involve
  static constexpr int NACC = NF;
  double sd[NF];
  double lsd[NF];   // log(sd_j), host (numpy) computed
  double isd2[NF];  // 1 / sd_j^2
  int bad;          // some sd_j <= 0: every group LL is NaN

  struct Reg { double t[NF]; };

  __device__ __forceinline__ Reg prepare(const double* th) const {
    Reg r;
#pragma unroll
    for (int j = 0; j < NF; ++j) r.t[j] = th[j];
    return r;
  }
  __device__ __forceinline__ void accum(const Reg& r, const double* __restrict__ row,
                                        double* acc) const {
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const double e = r.t[j] - row[j];
      acc[j] = fma(e, e, acc[j]);
    }
  }
  template <int N>
  __device__ __forceinline__ void accumN(const Reg& r, const double* __restrict__ rows,
                                         double (&a)[4][NACC]) const {
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const double e = r.t[j] - rows[i * NF + j];
        a[i & 3][j] = fma(e, e, a[i & 3][j]);
      }
  }
  __device__ __forceinline__ double finish(const Reg&, const double* acc, long n) const {
    if (n == 0) return 0.0;
    double out = 0.0;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      if (!(sd[j] > 0.0)) return nmc_nan();
      out += -0.5 * (acc[j] / (sd[j] * sd[j])) - (double)n * (NMC_LOG_C + lsd[j]);
    }
    return out;
  }
  __device__ __forceinline__ double gconst(long n) const {
    double c = 0.0;
#pragma unroll
    for (int j = 0; j < NF; ++j) c += (double)n * (NMC_LOG_C + lsd[j]);
    return c;
  }
  __device__ __forceinline__ void hold() {   // (FamLinreg::hold)
#pragma unroll
    for (int j = 0; j < NF; ++j) asm volatile("" : "+v"(isd2[j]));
  }
  __device__ __forceinline__ double finish_fast(const Reg&, const double* acc, long n,
                                                double gc) const {
    if (n == 0) return 0.0;
    if (bad) return nmc_nan();
    double q = 0.0;
#pragma unroll
    for (int j = 0; j < NF; ++j) q += -0.5 * (acc[j] * isd2[j]);
    return q - gc;
  }
  __device__ __forceinline__ double obs_ll(const Reg& r, const double* __restrict__ row) const {
    double out = 0.0;
#pragma unroll
    for (int j = 0; j < NF; ++j) out = out + nmc_norm_logpdf(r.t[j], row[j], sd[j], lsd[j]);
    return out;
  }
};

// ---------------------------------------------------------------------------
// Logistic regression (cfg 5): rows [x_1..x_K, y]; params [b0 if intercept, b_1..b_K];
//   eta = b0 + x.b, ll_i = y eta - logaddexp(0, eta).
// ---------------------------------------------------------------------------
template <int NF>
struct FamLogistic {
  static constexpr int NFIELDS = NF;
  static constexpr bool ASM_ROWS = false;
  static constexpr int MAXP = NF + 1;   // parameters a row of NF fields can involve
  static constexpr int NACC = 1;
  static constexpr int K = NF - 1;
  int intercept;

  struct Reg { double b0, b[K > 0 ? K : 1]; };

  __device__ __forceinline__ Reg prepare(const double* th) const {
    Reg r;
    r.b0 = intercept ? th[0] : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) r.b[j] = intercept ? th[j + 1] : th[j];
    return r;
  }
  __device__ __forceinline__ static double logaddexp0(double eta) { return nmc_logaddexp0(eta); }
  __device__ __forceinline__ void accum(const Reg& r, const double* __restrict__ row,
                                        double* acc) const {
    double eta = r.b0;
#pragma unroll
    for (int j = 0; j < K; ++j) eta = fma(row[j], r.b[j], eta);
    acc[0] += row[K] * eta - logaddexp0(eta);
  }
  template <int N>
  __device__ __forceinline__ void accumN(const Reg& r, const double* __restrict__ rows,
                                         double (&a)[4][NACC]) const {
    double eta[N];
#pragma unroll
    for (int i = 0; i < N; ++i) eta[i] = r.b0;
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i) eta[i] = fma(rows[i * NF + j], r.b[j], eta[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) a[i & 3][0] += rows[i * NF + K] * eta[i] - logaddexp0(eta[i]);
  }
  __device__ __forceinline__ double finish(const Reg&, const double* acc, long n) const {
    return n == 0 ? 0.0 : acc[0];
  }
  __device__ __forceinline__ double gconst(long) const { return 0.0; }
  __device__ __forceinline__ void hold() {}   // (FamLinreg::hold; no constants)
  __device__ __forceinline__ double finish_fast(const Reg& r, const double* acc, long n,
                                                double) const {
    return finish(r, acc, n);
  }
  __device__ __forceinline__ double obs_ll(const Reg& r, const double* __restrict__ row) const {
    double eta = 0.0;
    if (intercept) eta = r.b0;
#pragma unroll
    for (int j = 0; j < K; ++j) eta = eta + row[j] * r.b[j];
    return row[K] * eta - logaddexp0(eta);
  }
};
