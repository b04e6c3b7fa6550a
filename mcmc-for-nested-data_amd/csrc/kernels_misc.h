// kernels_misc.h -- the non-template kernels (variate fill, the LAUNCH-mode closing
// Gibbs update, verification hooks); included by nestmc.hip only, so each is defined
// in exactly one translation unit.
#pragma once
#include "kernels.h"

// ---------------------------------------------------------------------------
// Variates for iterations [iter0, iter0 + T), one launch: per (t, p, c) the hyper variates
// {hyper z, Gamma((G-1)/2)} (Marsaglia-Tsang on the Philox stream, or gammainccinv of the
// replayed uniform) and per (t, p, g, c) the step variates {z, log u} (nmc_step_variate).
// The hyper elements come first: their rejection loops are the longest, and started first
// they run under the bulk of the step elements.  The ring holds at most 1 GiB, so every
// element index fits 32 bits.
// ---------------------------------------------------------------------------
// {hyper z, Gamma draw} of hyper element i = (t, p, c) of iteration it (k: its replay index)
template <bool REPLAY>
__device__ __forceinline__ nmc_d2 nmc_fill_hyper(const Dev& d, int it, unsigned p, unsigned c,
                                                 size_t k) {
  nmc_d2 h;
  if constexpr (REPLAY) {
    h.a = it < d.replay_n ? d.rhz[k] : nmc_nan();
    h.b = it < d.replay_n ? nmc_igamci(d.ha, d.rhu[k], d.hlga) : nmc_nan();
  } else {
    const uint32_t ch = (uint32_t)(d.chain_base + (int)c);
    h.a = nmc_normal(it, 0, p, NMC_PURPOSE_HYPER_NORMAL, ch, d.seed);
    h.b = nmc_gamma_mt(d.ha, it, p, ch, d.seed);
  }
  return h;
}

// A resident grid (nmc_fill_blocks: a few 256-thread blocks per CU) walks the elements in
// grid-stride loops, the hyper elements first: 12.9 against 18.2 us for cfg 3's 20 iterations
// and 0.33 against 0.58 us per iteration (one thread per element: the blocks' dispatch and
// drain dominated, profiles/r05/r05f_fillbench.json).  REPLAY: the replayed reference
// variates (a separate instance: gammainccinv's registers would cost the Philox fill
// occupancy).
// MINB: blocks per CU (waves per SIMD) the register budget must allow -- 1 for the fill of
// the step stream (140 VGPRs); 4, 5, 6 or 8 (128, 96, 80, 64 VGPRs, with spills) for the prefill
// beside a resident step launch, whatever fits the VGPRs its waves leave on each SIMD
// (nestmc.hip nmc_set_resident): a fill that does not fit would wait for the launch to end
template <bool REPLAY, int MINB = 1>
__global__ void __launch_bounds__(256, MINB) nmc_k_fill(Dev d, int iter0, int T) {
  const unsigned C = (unsigned)d.C, GC = (unsigned)d.G * C, PGC = (unsigned)d.P * GC;
  const unsigned PC = (unsigned)d.P * C;
  const unsigned n1 = d.zin ? 0u : (unsigned)T * PGC;   // (zin: the step kernel draws these)
  const unsigned n2 = d.pooling == NMC_POOL_PARTIAL ? (unsigned)T * PC : 0u;
  const unsigned stride = gridDim.x * blockDim.x;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  for (unsigned i = tid; i < n2; i += stride) {   // hyper element i
    const unsigned t = i / PC, r = i - t * PC;
    const unsigned p = r / C, c = r - p * C;
    const int it = iter0 + (int)t;
    const nmc_d2 h = nmc_fill_hyper<REPLAY>(d, it, p, c, (size_t)it * PC + r);
    d.vh[2 * (size_t)i] = h.a;
    d.vh[2 * (size_t)i + 1] = h.b;
  }
  for (unsigned e = tid; e < n1; e += stride) {   // step element e
    const unsigned t = e / PGC, r = e - t * PGC;
    const unsigned p = r / GC, q = r - p * GC;
    const unsigned g = q / C, c = q - g * C;
    double z, lu;
    nmc_step_variate(d, iter0 + (int)t, (int)p, (int)g, (int)c, z, lu);
    d.vzl[2 * (size_t)e] = z;
    d.vzl[2 * (size_t)e + 1] = lu;
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

__global__ void nmc_k_debug_softplus(const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = nmc_softplus(x[i]);
}
