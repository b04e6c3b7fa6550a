// rng.h -- the sampler's random streams (host + device).
//
// Replaces the numpy legacy MT19937 draws of the reference hot loop:
//   proposal normal   posteriorSampling.py:306   (Parameter.propose)
//   accept uniform    posteriorSampling.py:362   (Parameter.step, branch 4)
//   hyper normal      posteriorSampling.py:487   (HyperParameter._updateMean)
//   hyper invgamma    posteriorSampling.py:498   (HyperParameter._sampleInvChisq)
// by a counter-based Philox4x32-10 stream, so every (chain, iteration, group,
// parameter) draw is independent of launch geometry, GPU count and of which
// branch other groups took.  Spec (shared with oracle/philox.py):
//   key = (global chain id, seed), counter = (iteration, group, param, purpose)
//   block -> two 53-bit uniforms in [0,1): ((x1<<32|x0)>>11)*2^-53, ((x3<<32|x2)>>11)*2^-53
//   normal = sqrt(-2 log(1-ua)) * cos(2 pi ub)          (Box-Muller, cos branch)
// Compiled with -ffp-contract=off: every expression rounds exactly as written.
#pragma once
#ifndef __HIPCC_RTC__   // (hiprtc, user families: the runtime provides these)
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#define NMC_HD __host__ __device__ __forceinline__

enum {
  NMC_PURPOSE_PROPOSAL = 0,
  NMC_PURPOSE_ACCEPT = 1,
  NMC_PURPOSE_HYPER_NORMAL = 2,
  NMC_PURPOSE_GAMMA_BOOST = 3,
  NMC_PURPOSE_GAMMA_BASE = 16,
  NMC_GAMMA_MAX_ATTEMPTS = 64
};

struct nmc_u4 { uint32_t x0, x1, x2, x3; };

NMC_HD nmc_u4 nmc_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                         uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return nmc_u4{c0, c1, c2, c3};
}

struct nmc_d2 { double a, b; };

NMC_HD nmc_d2 nmc_uniform2(uint32_t it, uint32_t group, uint32_t param, uint32_t purpose,
                           uint32_t chain, uint32_t seed) {
  const nmc_u4 x = nmc_philox(it, group, param, purpose, chain, seed);
  const uint64_t a = (((uint64_t)x.x1 << 32) | x.x0) >> 11;
  const uint64_t b = (((uint64_t)x.x3 << 32) | x.x2) >> 11;
  const double inv53 = 1.0 / 9007199254740992.0;
  return nmc_d2{(double)a * inv53, (double)b * inv53};
}

// The Box-Muller transform's two transcendentals, restated for their argument ranges:
// the library's fp64 log and cos cost 76 and 109 fp64 instructions on gfx950 (double-
// double evaluation; cos also carries a Payne-Hanek reduction for large arguments), which
// made every step variate 291 fp64 instructions and the fill 0.58 us per cfg-3 iteration
// (profiles/r05/r05c_fillbench.json).  Both below are within ~1 ulp of the exact value
// (tools/varmath_check.hip), like the library's; the oracle keeps numpy's log and cos
// (tests compare at rtol 1e-14).
//
// log(x) for x in [0, 1]: x = m 2^e with m in [sqrt(1/2), sqrt(2)) (frexp, exact), log(m) =
// 2 atanh(s), s = (m - 1) / (m + 1), |s| <= 0.1716 (m - 1 exact: Sterbenz), the series to
// s^23 (the first omitted term < 1e-18 relative); e ln 2 in two parts (ln2_hi has 32
// significant bits, so e * ln2_hi is exact).  0 -> -inf, NaN propagates.
NMC_HD double nmc_log_unit(double x) {
  int e = 0;
  double m = frexp(x, &e);                       // m in [0.5, 1)
  if (m < 0.70710678118654752) {
    m = m + m;
    e -= 1;
  }
  const double f = m - 1.0;
  const double s = f / (m + 1.0);
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
  const double ed = (double)e;
  const double l = fma(s * z, q, fma(ed, 1.9082149292705877e-10, 2.0 * s));   // + e ln2_lo
  const double r = fma(ed, 0.6931471803691238, l);                            // + e ln2_hi
  return x == 0.0 ? -__builtin_huge_val() : (x == x ? r : x);
}

// cos(2 pi u) for u in [0, 1) (the 53-bit uniform): reduced exactly in u -- cos(2 pi u) =
// cos(2 pi (1 - u)) = -cos(2 pi (1/2 - v)) = sin(2 pi (1/4 - w)), every difference exact
// (Sterbenz) -- to t in [0, 1/8] (angle <= pi/4), then the cos or sin Taylor polynomial in
// t^2 through the t^18 / t^19 terms (the first omitted term < 1e-18 relative).
NMC_HD double nmc_cos2pi(double u) {
  const double v = u > 0.5 ? 1.0 - u : u;        // [0, 1/2]
  const bool neg = v > 0.25;
  const double w = neg ? 0.5 - v : v;            // [0, 1/4]
  const bool sn = w > 0.125;
  const double t = sn ? 0.25 - w : w;            // [0, 1/8]
  const double x = t * t;
  double c = -0.03638284114254567;
  c = fma(c, x, 0.28200596845579123);
  c = fma(c, x, -1.714390711088672);
  c = fma(c, x, 7.903536371318469);
  c = fma(c, x, -26.4262567833744);
  c = fma(c, x, 60.24464137187666);
  c = fma(c, x, -85.45681720669373);
  c = fma(c, x, 64.9393940226683);
  c = fma(c, x, -19.739208802178716);
  c = fma(c, x, 1.0);
  double p = -0.012031585942120627;
  p = fma(p, x, 0.10422916220813984);
  p = fma(p, x, -0.7181223017785006);
  p = fma(p, x, 3.819952584848282);
  p = fma(p, x, -15.09464257682299);
  p = fma(p, x, 42.058693944897655);
  p = fma(p, x, -76.70585975306139);
  p = fma(p, x, 81.60524927607506);
  p = fma(p, x, -41.34170224039976);
  p = fma(p * x, t, 6.283185307179586 * t);      // sin(2 pi t)
  const double r = sn ? p : c;
  return neg ? -r : r;
}

NMC_HD double nmc_box_muller(double ua, double ub) {
  return sqrt(-2.0 * nmc_log_unit(1.0 - ua)) * nmc_cos2pi(ub);
}

NMC_HD double nmc_normal(uint32_t it, uint32_t group, uint32_t param, uint32_t purpose,
                         uint32_t chain, uint32_t seed) {
  const nmc_d2 u = nmc_uniform2(it, group, param, purpose, chain, seed);
  return nmc_box_muller(u.a, u.b);
}

// Gamma(a, 1) by Marsaglia & Tsang (2000) with the squeeze test; attempt k uses
// purposes 16+2k (normal) and 17+2k (uniform); shape < 1 boosts with U^(1/a).
// The hyper update draws sigma2 = scale / Gamma(a) ~ Inv-chi2 exactly as the
// reference's invgamma(a, scale) (posteriorSampling.py:497-498) in distribution.
NMC_HD double nmc_gamma_mt(double a, uint32_t it, uint32_t param, uint32_t chain,
                           uint32_t seed) {
  const bool boost = a < 1.0;
  const double aa = boost ? a + 1.0 : a;
  const double d = aa - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double x = d;
  for (int k = 0; k < NMC_GAMMA_MAX_ATTEMPTS; ++k) {
    const double z = nmc_normal(it, 0, param, NMC_PURPOSE_GAMMA_BASE + 2 * k, chain, seed);
    const double u =
        nmc_uniform2(it, 0, param, NMC_PURPOSE_GAMMA_BASE + 2 * k + 1, chain, seed).a;
    const double v = 1.0 + c * z;
    if (!(v > 0.0)) continue;
    const double v3 = v * v * v;
    const double z2 = z * z;
    if (u < 1.0 - 0.0331 * (z2 * z2) || log(u) < 0.5 * z2 + d * (1.0 - v3 + log(v3))) {
      x = d * v3;
      break;
    }
  }
  if (boost) {
    const double ub = nmc_uniform2(it, 0, param, NMC_PURPOSE_GAMMA_BOOST, chain, seed).a;
    x = x * exp(log(1.0 - ub) / a);
  }
  return x;
}
