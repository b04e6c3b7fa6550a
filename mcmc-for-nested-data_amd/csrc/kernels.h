// kernels.h -- the MCMC step kernels for gfx950 (CDNA4, wave64, fp64).
//
// Layout: chain-on-lane.  A workgroup owns one (chain block of 64 chains, group g)
// pair; its W wavefronts split group g's observation rows (CSR range
// off[g]..off[g+1]) into W contiguous chunks.  Every lane holds its chain's P
// parameter values (the proposal for parameter p, the current values for the
// others -- posteriorSampling.py:615-623) in registers and accumulates the family's
// log-likelihood over its wave's chunk; the rows are wave-uniform, so they stream
// through the scalar cache and each row serves 64 chains.  The W partial sums meet
// in LDS (fixed order), and wave 0 runs the Metropolis epilogue SIMT-wide, one
// chain per lane:
//   prior log-density  (partial: the Gaussian hyper-prior, lazily refreshed after
//                       each Gibbs update; none/complete: the scipy prior family)
//   branch order       posteriorSampling.py:347-367 (IEEE isfinite, no fast-math)
//   accept / reject    :369-383, group LL propagation :608-610
//   tuning             :385-437 on tune iterations (:875-878)
//   recording          :887-889 into the device sample store [row][col][C]
//   next proposal      :304-306 for the same parameter's next iteration
// Partial pooling couples the groups of a chain once per parameter step
// (HyperParameter.update, :463-498): extra workgroups of the SAME launch run the
// Gibbs update of the previous parameter, which no concurrent step reads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "families.h"
#include "rng.h"
#include "special.h"

struct Dev {
  int C, G, P, pooling, nf, chain_base, rng_mode, W, CB;
  uint32_t seed;
  const int64_t* off;
  const double* obs;
  const int* pfam;       // [P]
  const double* ppar;    // [P][8]
  double* value;         // [P][G][C]
  double* lp;            // [P][G][C]
  double* ll;            // [G][C]
  double* scale;         // [P][G][C]
  double* prop;          // [P][G][C]  proposal for the parameter's next step
  int* nacc;             // [P][G][C]  since last tune
  int* nrej;
  long long* tacc;       // [P][G][C]  total accepted
  double* mu;            // [P][C]
  double* s2;
  double* hsd;           // sqrt(s2)
  double* hlsd;          // log(sqrt(s2))
  double ha, hlga;       // invgamma shape a = (G-1)/2 and gammaln(a)
  const double* rz;      // replay [iter][P][G][C]
  const double* ru;
  const double* rhz;     // replay [iter][P][C]
  const double* rhu;
  int replay_n;
  int burn, thin, tune_interval, n_rows, cols;
  double* samples;       // [row][col][C]
  uint8_t* tflag;        // trace [iter][P][G][C]
  double* tllp;
  int trace_n;
};

__device__ __forceinline__ int nmc_record_row(const Dev& d, int iter) {
  if (iter < d.burn || (iter % d.thin) != 0) return -1;
  const int first = ((d.burn + d.thin - 1) / d.thin) * d.thin;
  const int row = (iter - first) / d.thin;
  return row < d.n_rows ? row : -1;
}

__device__ __forceinline__ double nmc_prop_z(const Dev& d, int iter, int p, int g, int c) {
  if (d.rng_mode == NMC_RNG_REPLAY) {
    if (iter >= d.replay_n) return nmc_nan();
    return d.rz[(((size_t)iter * d.P + p) * d.G + g) * d.C + c];
  }
  return nmc_normal(iter, g, p, NMC_PURPOSE_PROPOSAL, d.chain_base + c, d.seed);
}

__device__ __forceinline__ double nmc_accept_u(const Dev& d, int iter, int p, int g, int c) {
  if (d.rng_mode == NMC_RNG_REPLAY) {
    if (iter >= d.replay_n) return nmc_nan();
    return d.ru[(((size_t)iter * d.P + p) * d.G + g) * d.C + c];
  }
  return nmc_uniform2(iter, g, p, NMC_PURPOSE_ACCEPT, d.chain_base + c, d.seed).a;
}

// Parameter.tune (posteriorSampling.py:385-437)
__device__ __forceinline__ void nmc_tune(double& s, int& na, int& nr) {
  const double tot = (double)na + (double)nr;
  if (!(tot > 0.0)) return;
  const double rate = (double)na / tot;
  double f = 1.0;
  if (rate < 0.001) f = 0.1;
  else if (rate < 0.05) f = 0.5;
  else if (rate < 0.2) f = 0.9;
  else if (rate > 0.95) f = 10.0;
  else if (rate > 0.75) f = 2.0;
  else if (rate > 0.5) f = 1.1;
  const double ns = s * f;
  na = 0;
  nr = 0;
  if (ns != 0.0) s = ns;
}

// ---------------------------------------------------------------------------
// Gibbs update of one parameter's hyper-parameters for one chain per lane
// (HyperParameter._updateMean :481-487, _updateVar :489-498).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void nmc_hyper_body(const Dev& d, int cb, int hp, int hiter, int lane) {
  const int c = cb * 64 + lane;
  if (c >= d.C) return;
  const int G = d.G, C = d.C;
  const double* x = d.value + (size_t)hp * G * C + c;
  const double muhat = nmc_pairwise_sum([&](int i) { return x[(size_t)i * C]; }, G) / G;
  const double sd = sqrt(d.s2[hp * C + c] / G);
  const uint32_t chain = (uint32_t)(d.chain_base + c);
  double z;
  if (d.rng_mode == NMC_RNG_REPLAY)
    z = hiter < d.replay_n ? d.rhz[((size_t)hiter * d.P + hp) * C + c] : nmc_nan();
  else
    z = nmc_normal(hiter, 0, hp, NMC_PURPOSE_HYPER_NORMAL, chain, d.seed);
  const double m = muhat + sd * z;
  const double ss = nmc_pairwise_sum(
      [&](int i) { const double t = x[(size_t)i * C] - m; return t * t; }, G);
  const double hat = ss / (double)(G - 1);
  const double scale = d.ha * hat;
  double s2n;
  if (scale == 0.0) {
    s2n = 0.0;       // scipy rvs returns loc when scale == 0 (no draw)
  } else {
    double X;
    if (d.rng_mode == NMC_RNG_REPLAY)
      X = hiter < d.replay_n ? nmc_igamci(d.ha, d.rhu[((size_t)hiter * d.P + hp) * C + c], d.hlga)
                             : nmc_nan();
    else
      X = nmc_gamma_mt(d.ha, hiter, hp, chain, d.seed);
    s2n = (1.0 / X) * scale;
  }
  const double sdn = sqrt(s2n);
  d.mu[hp * C + c] = m;
  d.s2[hp * C + c] = s2n;
  d.hsd[hp * C + c] = sdn;
  d.hlsd[hp * C + c] = log(sdn);
  const int row = nmc_record_row(d, hiter);
  if (row >= 0) {
    double* out = d.samples + ((size_t)row * d.cols + (size_t)hp * (G + 2)) * C + c;
    out[0] = m;
    out[C] = s2n;
  }
}

// ---------------------------------------------------------------------------
// log-likelihood of one group over one wave's row chunk, chain-on-lane
// ---------------------------------------------------------------------------
// n rows starting at p (wave-uniform -> scalar loads).  R rows (~16 doubles) are
// requested together per iteration so each scalar-cache round trip feeds 2R-4R fp64
// VALU ops; the other waves on the SIMD cover the latency.  Four accumulator sets
// break the dependence chain.
template <class Fam>
__device__ __forceinline__ void nmc_ll_chunk(const Fam& fam, const typename Fam::Reg& reg,
                                             const double* __restrict__ p, int n,
                                             double (&acc)[Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  constexpr int R = (16 / NF) > 0 ? (16 / NF) : 1;
  double a[4][Fam::NACC];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) a[s][k] = 0.0;
  const int nb = n / R;
  for (int b = 0; b < nb; ++b) {
    const double* q = p + (size_t)b * (R * NF);
    double blk[R * NF];
#pragma unroll
    for (int j = 0; j < R * NF; ++j) blk[j] = q[j];
#pragma unroll
    for (int r = 0; r < R; ++r) fam.accum(reg, blk + r * NF, a[r & 3]);
  }
  for (int r = nb * R; r < n; ++r) fam.accum(reg, p + (size_t)r * NF, a[0]);
#pragma unroll
  for (int k = 0; k < Fam::NACC; ++k) acc[k] = (a[0][k] + a[1][k]) + (a[2][k] + a[3][k]);
}

// Whole-workgroup LL of group g for theta (registers); result valid in wave 0.
// Every thread of the block must call this (it contains a barrier when W > 1).
template <class Fam>
__device__ __forceinline__ double nmc_group_ll(const Dev& d, const Fam& fam, int g,
                                               const double (&th)[NMC_MAXP], double* red,
                                               const double* __restrict__ obs) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  const int64_t r0 = d.off[g], r1 = d.off[g + 1];
  const int64_t n = r1 - r0;
  const int64_t chunk = (n + d.W - 1) / d.W;
  const int64_t a = r0 + (int64_t)w * chunk;
  const int64_t e = a + chunk < r1 ? a + chunk : r1;
  const typename Fam::Reg reg = fam.prepare(th);
  double acc[Fam::NACC];
  const int64_t a0 = a < r1 ? a : r1;
  nmc_ll_chunk(fam, reg, obs + a0 * Fam::NFIELDS, (int)(e - a0), acc);
  if (d.W > 1) {
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) red[(k * d.W + w) * 64 + lane] = acc[k];
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int k = 0; k < Fam::NACC; ++k) {
        double s = red[(k * d.W) * 64 + lane];
        for (int v = 1; v < d.W; ++v) s += red[(k * d.W + v) * 64 + lane];
        acc[k] = s;
      }
    }
  }
  return fam.finish(reg, acc, (long)n);
}

template <class Fam>
__device__ __forceinline__ void nmc_load_theta(const Dev& d, int g, int c, int p,
                                               const double* prop_src,
                                               double (&th)[NMC_MAXP]) {
#pragma unroll
  for (int q = 0; q < NMC_MAXP; ++q) {
    th[q] = 0.0;
    if (q < d.P) {
      const size_t i = ((size_t)q * d.G + g) * d.C + c;
      th[q] = (q == p || p < 0) ? prop_src[i] : d.value[i];
    }
  }
}

// ---------------------------------------------------------------------------
// K_step: MH step of parameter p at iteration iter for every (chain, group), plus
// (partial pooling) the Gibbs update of parameter hp at iteration hiter.
// grid = CB*G step workgroups (+ CB hyper workgroups), block = 64*W threads.
// ---------------------------------------------------------------------------
template <class Fam>
__global__ void __launch_bounds__(1024)
nmc_k_step(Dev d, Fam fam, const double* __restrict__ obs, int iter, int p, int hp, int hiter) {
  extern __shared__ __attribute__((aligned(16))) double red[];
  const int nstep = d.CB * d.G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if ((int)blockIdx.x >= nstep) {
    if (w == 0) nmc_hyper_body(d, blockIdx.x - nstep, hp, hiter, lane);
    return;
  }
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const bool live = c < d.C;
  const int cc = live ? c : d.C - 1;
  double th[NMC_MAXP];
  nmc_load_theta<Fam>(d, g, cc, p, d.prop, th);
  const double llp = nmc_group_ll(d, fam, g, th, red, obs);
  if (w != 0 || !live) return;

  // ---- Metropolis epilogue: one chain per lane -------------------------
  double prop = 0.0;
#pragma unroll
  for (int q = 0; q < NMC_MAXP; ++q)
    if (q == p) prop = th[q];
  const size_t ip = ((size_t)p * d.G + g) * d.C + c;
  const size_t ig = (size_t)g * d.C + c;
  double v = d.value[ip];
  double s = d.scale[ip];
  const double LL = d.ll[ig];
  double lpc, lpp;
  if (d.pooling == NMC_POOL_PARTIAL) {
    const double m = d.mu[p * d.C + c], sd = d.hsd[p * d.C + c], lsd = d.hlsd[p * d.C + c];
    lpc = iter > 0 ? nmc_norm_logpdf(v, m, sd, lsd) : d.lp[ip];   // refreshed by setPrior :281
    lpp = nmc_norm_logpdf(prop, m, sd, lsd);
  } else {
    lpc = d.lp[ip];
    lpp = nmc_prior_logpdf(d.pfam[p], d.ppar + 8 * p, prop);
  }
  const double postp = lpp + llp;
  const double post = lpc + LL;
  const double diff = postp - post;
  bool acc;
  if (!isfinite(post) && isfinite(postp)) acc = true;          // :347-352
  else if (!isfinite(llp)) acc = false;                        // :354-356
  else if (!isfinite(diff)) acc = false;                       // :358-360
  else acc = log(nmc_accept_u(d, iter, p, g, c)) < diff;       // :362-364
  int na = d.nacc[ip], nr = d.nrej[ip];
  if (acc) {
    v = prop;
    d.value[ip] = prop;
    d.lp[ip] = lpp;
    d.ll[ig] = llp;
    ++na;
    d.tacc[ip] += 1;
  } else {
    d.lp[ip] = lpc;
    ++nr;
  }
  if (iter > 0 && iter < d.burn && iter % d.tune_interval == 0) nmc_tune(s, na, nr);
  d.nacc[ip] = na;
  d.nrej[ip] = nr;
  d.scale[ip] = s;
  d.prop[ip] = v + (1.0 * s) * nmc_prop_z(d, iter + 1, p, g, c);
  const int row = nmc_record_row(d, iter);
  if (row >= 0) {
    const int col = p * (d.G + (d.pooling == NMC_POOL_PARTIAL ? 2 : 0)) +
                    (d.pooling == NMC_POOL_PARTIAL ? 2 : 0) + g;
    d.samples[((size_t)row * d.cols + col) * d.C + c] = v;
  }
  if (iter < d.trace_n) {
    const size_t it = (((size_t)iter * d.P + p) * d.G + g) * d.C + c;
    d.tflag[it] = acc ? 1 : 0;
    d.tllp[it] = llp;
  }
}

// Gibbs update alone (P == 1, and the last parameter of a run).
__global__ void __launch_bounds__(64) nmc_k_hyper(Dev d, int hp, int hiter) {
  nmc_hyper_body(d, blockIdx.x, hp, hiter, threadIdx.x & 63);
}

// Proposals of every parameter for iteration iter (start of a run).
__global__ void __launch_bounds__(256) nmc_k_prop(Dev d, int iter) {
  const size_t n = (size_t)d.P * d.G * d.C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % d.C);
    const int g = (int)((i / d.C) % d.G);
    const int p = (int)(i / ((size_t)d.C * d.G));
    d.prop[i] = d.value[i] + (1.0 * d.scale[i]) * nmc_prop_z(d, iter, p, g, c);
  }
}

// Group sums for arbitrary theta [P][G][C] -> out [G][C].
template <class Fam>
__global__ void __launch_bounds__(1024)
nmc_k_group_ll(Dev d, Fam fam, const double* __restrict__ obs, const double* theta,
               double* out) {
  extern __shared__ __attribute__((aligned(16))) double red[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[NMC_MAXP];
  nmc_load_theta<Fam>(d, g, cc, -1, theta, th);
  const double s = nmc_group_ll(d, fam, g, th, red, obs);
  if (w == 0 && c < d.C) out[(size_t)g * d.C + c] = s;
}

// Per-observation LL at the current state -> out [C][n_obs].
template <class Fam>
__global__ void __launch_bounds__(64) nmc_k_obs_ll(Dev d, Fam fam, double* out, int64_t n_obs) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[NMC_MAXP];
  nmc_load_theta<Fam>(d, g, cc, -1, d.value, th);   // p < 0: every theta from d.value
  const typename Fam::Reg reg = fam.prepare(th);
  const int nf = Fam::NFIELDS;
  for (int64_t r = d.off[g]; r < d.off[g + 1]; ++r) {
    const double v = fam.obs_ll(reg, d.obs + r * nf);
    if (c < d.C) out[(size_t)c * n_obs + r] = v;
  }
}

// ---------------------------------------------------------------------------
// debug/verification kernels (device numerics against scipy / the oracle)
// ---------------------------------------------------------------------------
__global__ void nmc_k_debug_prior(int fam, const double* prm, const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = nmc_prior_logpdf(fam, prm, x[i]);
}

__global__ void nmc_k_debug_igamci(const double* a, const double* q, const double* lga, int n,
                                   double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = nmc_igamci(a[i], q[i], lga[i]);
}

// out[i] = {normal(purpose), uniform a, uniform b, gamma_mt(a)} for counters in ctr[i][5]
// = (iter, group, param, purpose, chain); gamma uses (iter, param, chain).
__global__ void nmc_k_debug_rng(const uint32_t* ctr, int n, uint32_t seed, double ga, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* k = ctr + 5 * i;
  const nmc_d2 u = nmc_uniform2(k[0], k[1], k[2], k[3], k[4], seed);
  out[4 * i + 0] = nmc_box_muller(u.a, u.b);
  out[4 * i + 1] = u.a;
  out[4 * i + 2] = u.b;
  out[4 * i + 3] = nmc_gamma_mt(ga, k[0], k[2], k[4], seed);
}
