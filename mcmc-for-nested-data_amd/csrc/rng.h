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

NMC_HD double nmc_box_muller(double ua, double ub) {
  return sqrt(-2.0 * log(1.0 - ua)) * cos(6.283185307179586 * ub);
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
