// kernels_misc.h -- the non-template kernels (variate fill, the LAUNCH-mode closing
// Gibbs update, verification hooks); included by nestmc.hip only, so each is defined
// in exactly one translation unit.
#pragma once
#include "kernels.h"

// ---------------------------------------------------------------------------
// Variates for iterations [iter0, iter0 + T): one thread per (t, p, g, c) element
// of the step variates and per (t, p, c) of the hyper variates.  The hyper variates come
// first in the index space: their Gamma draws (rejection loops) are the longest threads,
// and started first they run under the bulk of the step variates instead of after it.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) nmc_k_fill(Dev d, int iter0, int T) {
  const size_t PGC = (size_t)d.P * d.G * d.C, PC = (size_t)d.P * d.C;
  const size_t n1 = d.zin ? 0 : (size_t)T * PGC;   // (zin: the step kernel draws these)
  const size_t n2 = d.pooling == NMC_POOL_PARTIAL ? (size_t)T * PC : 0;
  for (size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i0 < n1 + n2;
       i0 += (size_t)gridDim.x * blockDim.x) {
    // i0 < n2: hyper element i0; else step element i0 - n2
    const size_t i = i0 < n2 ? n1 + i0 : i0 - n2;
    if (i < n1) {
      const int t = (int)(i / PGC);
      const size_t r = i % PGC;
      const int c = (int)(r % d.C);
      const int g = (int)((r / d.C) % d.G);
      const int p = (int)(r / ((size_t)d.C * d.G));
      const int it = iter0 + t;
      double z, lu;
      nmc_step_variate(d, it, p, g, c, z, lu);
      d.vzl[2 * i] = z;
      d.vzl[2 * i + 1] = lu;
    } else {
      const size_t j = i - n1;
      const int t = (int)(j / PC);
      const size_t r = j % PC;
      const int c = (int)(r % d.C);
      const int p = (int)(r / d.C);
      const int it = iter0 + t;
      double hz, hx;
      if (d.rng_mode == NMC_RNG_REPLAY) {
        const size_t k = (size_t)it * PC + r;
        hz = it < d.replay_n ? d.rhz[k] : nmc_nan();
        hx = it < d.replay_n ? nmc_igamci(d.ha, d.rhu[k], d.hlga) : nmc_nan();
      } else {
        const uint32_t ch = (uint32_t)(d.chain_base + c);
        hz = nmc_normal(it, 0, p, NMC_PURPOSE_HYPER_NORMAL, ch, d.seed);
        hx = nmc_gamma_mt(d.ha, it, p, ch, d.seed);
      }
      d.vh[2 * j] = hz;
      d.vh[2 * j + 1] = hx;
    }
  }
}

// Gibbs update after iteration t alone (closes a chunk in launch-per-iteration mode);
// grid = RB workgroups (the step kernel's chain blocks).
__global__ void __launch_bounds__(1024) nmc_k_hyper(Dev d, const double* src, int t) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, C = d.C;
  const int c = nmc_lane_chain(d, blockIdx.x, lane);
  const int cc = c < C ? c : C - 1;
  const nmc_lds_layout L = nmc_lds(0, P, 1, d.nleaf, d.ntail, 0, d.G, 0);
  for (int p = w; p < P; p += W) {
    const double s2 = d.s2[nmc_hslot(d, t - 1) + (size_t)p * C + cc];   // after t-1
    lds[(L.hyp + NMC_HY_S2 * P + p) * 64 + lane] = s2;
    lds[(L.hyp + NMC_HY_SDM * P + p) * 64 + lane] = sqrt(s2 / d.G);
  }
  nmc_hyper_variates(d, blockIdx.x, t, lds, L, 0, W);
  nmc_drain_vm();
  __syncthreads();
  nmc_hyper<NMC_SRC_GLOBAL>(d, src, blockIdx.x, t, lds, L, true);
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
