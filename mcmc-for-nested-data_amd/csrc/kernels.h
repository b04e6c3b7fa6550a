// kernels.h -- the MCMC sampling kernels for gfx950 (CDNA4, wave64, fp64).
//
// Layout: chain-on-lane.  A workgroup owns one (chain block of 64 chains, group g)
// pair; its W waves split the group's CSR rows obs[off[g]..off[g+1]).  Every lane of
// a wave holds ONE chain's parameters in registers while the whole wave walks the
// same rows, so a row is read with a wave-uniform scalar load (s_load, SGPR operands)
// and feeds 64 chains -- the cross-chain reuse that makes the dataset cache-resident.
//
// nmc_k_run runs the reference's Sampler._loop body (posteriorSampling.py:872-891)
// for iterations [i0, i1) of every (chain, group).  Per parameter step p
// (StepMethod.step :594-613):
//   1. every wave proposes theta_p' = theta_p + scale*z (Parameter.propose :304-306)
//      and accumulates the family log-likelihood over its row slice (:615-635);
//   2. partial sums go to LDS (double-buffered by step parity), ONE barrier;
//   3. every wave sums the W partials in the same fixed order and runs the identical
//      Metropolis decision (:334-383, branch order exact, IEEE isfinite), tuning
//      (:385-437) and group-LL propagation (:608-610) -- redundantly, so no second
//      barrier is needed to broadcast the result.  Wave 0 alone writes outputs.
// Per-(p, chain) state that changes (scale, log prior, counters) lives in LDS,
// double-buffered by iteration parity; the current values live in one LDS column per
// parameter (every wave writes the same value, so each wave sees its own write), the
// group LL in a register.
//
// Partial pooling couples the G groups of a chain through the Gibbs update of the
// hyper-parameters (HyperParameter.update :463-498).  Its update after iteration t-1
// is only needed by the Metropolis decisions of iteration t (the prior of each
// parameter), not by the likelihood.  So the update is computed right after the
// step-0 likelihood of iteration t, redundantly by every workgroup of the chain
// block, in numpy's pairwise-sum order (exact mean/variance parity):
//   * persistent mode (every workgroup resident): values are published write-through
//     (sc1 stores, vmcnt drain, one agent-scope counter add per workgroup and
//     iteration); a workgroup waits for its chain block's counter only AFTER its
//     step-0 likelihood, so the hand-off latency hides behind compute, and reads the
//     published values with sc1 loads (MI355X_MICROARCH.md, inter-workgroup
//     visibility: sc1 stores + counter + sc1 loads, no fences);
//   * launch-per-iteration mode (grid too large to be resident): the kernel
//     boundary publishes, plain loads read.
// Every spin is bounded: a timeout sets d.tmo and every workgroup drains.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "families.h"
#include "rng.h"
#include "special.h"

struct Dev {
  int C, G, P, pooling, nf, chain_base, rng_mode, W, CB;
  uint32_t seed;
  const int64_t* off;    // [G+1] CSR offsets
  const double* obs;     // [n_obs][nf]
  const int* pfam;       // [P]
  const double* ppar;    // [P][8]
  double* vb0;           // values after iteration t live in vb[t & 1]: [P][G][C]
  double* vb1;
  double* lp;            // [P][G][C]
  double* ll;            // [G][C]
  double* scale;         // [P][G][C]
  int* nacc;             // [P][G][C]  since last tune
  int* nrej;
  long long* tacc;       // [P][G][C]  total accepted
  double* mu;            // [2][P][C]: after iteration t in slot t & 1 (nmc_hslot)
  double* s2;
  double* hsd;           // sqrt(s2)
  double* hlsd;          // log(sqrt(s2))
  double ha, hlga;       // invgamma shape a = (G-1)/2 and gammaln(a)
  // numpy pairwise-sum plan over the G groups (numpy/_core/src/umath/loops_utils.h)
  const int* leaf;       // [nleaf+1] start of each <=128-element leaf block
  const int* merge;      // [nmerge][2] post-order merges: slot a += slot b
  int nleaf, nmerge, ntail;
  int nmax;              // rows of the largest group
  int hlds, naux;        // persistent partial: Gibbs payload via LDS, auxiliary waves
  int noprio;            // diagnostics: no issue priority for the latency-bound waves
  int rows_lds;          // 1: each workgroup stages its group's rows in LDS once per launch
  unsigned* cnt;         // [CB][P][32] publish counters (persistent partial), zeroed per launch
  unsigned* tmo;         // timeout word (persists; host checks it)
  // variates of iterations [vbase, vbase + vcap): filled by nmc_k_fill
  double* vzl;           // [t][P][G][C][2] {proposal normal, log accept uniform}
  double* vh;            // [t][P][C][2]    {hyper mean normal, hyper Gamma(a) draw}
  int vbase, vcap;
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
  unsigned long long* stamps;   // diagnostic build only (-DNMC_STAMPS)
};

// Diagnostic build only (make stamps -> libnestmc_stamps.so, never shipped): shader-
// clock stamps of workgroups 0 and last, waves 0 and W-1, first 8 iterations of a
// launch: stamps[((blk * 2 + wv) * 8 + iter) * 8 + slot].
#ifdef NMC_STAMPS
#define NMC_STAMP(t, slot)                                                              \
  do {                                                                                  \
    const int sb_ = blockIdx.x == 0 ? 0 : (blockIdx.x == gridDim.x - 1 ? 1 : -1);         \
    const int sw_ = w == 0 ? 0 : (w == W - 1 ? 1 : -1);                                 \
    if (d.stamps && sb_ >= 0 && sw_ >= 0 && (t) - i0 < 8 && lane == 0)                  \
      d.stamps[((sb_ * 2 + sw_) * 8 + ((t) - i0)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define NMC_STAMP_AT(k, slot)                                                           \
  do {                                                                                  \
    const int w_ = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                    \
    const int sb_ = blockIdx.x == 0 ? 0 : (blockIdx.x == gridDim.x - 1 ? 1 : -1);         \
    const int sw_ = w_ == 0 ? 0 : (w_ == (int)(blockDim.x >> 6) - 1 ? 1 : -1);          \
    if (d.stamps && (k) >= 0 && (k) < 8 && sb_ >= 0 && sw_ >= 0 && (threadIdx.x & 63) == 0) \
      d.stamps[((sb_ * 2 + sw_) * 8 + (k)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// auxiliary wave 1 of workgroup 0, into the wave-W-1 row of block 0 (slots 13-15)
#define NMC_STAMP_AUX(t, slot)                                                          \
  do {                                                                                  \
    if (d.stamps && blockIdx.x == 0 && w == 1 && (t) - i0 < 8 && lane == 0)              \
      d.stamps[((0 * 2 + 1) * 8 + ((t) - i0)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// compute wave half 0 (wave 1) of workgroup 0, into the control-wave row (slots 13-15)
#define NMC_STAMP_CMP(t, slot)                                                          \
  do {                                                                                  \
    if (d.stamps && blockIdx.x == 0 && w == 1 && (t) - i0 < 8 && lane == 0)              \
      d.stamps[((0 * 2 + 0) * 8 + ((t) - i0)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define NMC_STAMP_CMP(t, slot) do {} while (0)
#define NMC_STAMP_AUX(t, slot) do {} while (0)
#define NMC_STAMP(t, slot) do {} while (0)
#define NMC_STAMP_AT(k, slot) do {} while (0)
#endif

enum { NMC_RUN_HYPER_LOAD = 1 };
enum { NMC_SPIN_LIMIT = 1 << 22 };

// Offset of the hyper-parameter slot holding the state after iteration t ([2][P][C]:
// slot t & 1, like the values vb[t & 1]); a launch reads one slot and writes the other.
__device__ __forceinline__ size_t nmc_hslot(const Dev& d, int t) {
  return (size_t)(t & 1) * d.P * d.C;
}

__device__ __forceinline__ int nmc_record_row(const Dev& d, int iter) {
  if (iter < d.burn || (iter % d.thin) != 0) return -1;
  const int first = ((d.burn + d.thin - 1) / d.thin) * d.thin;
  const int row = (iter - first) / d.thin;
  return row < d.n_rows ? row : -1;
}

// Parameter.tune (posteriorSampling.py:385-437)
__device__ __forceinline__ void nmc_tune(double& s, double& na, double& nr) {
  const double tot = na + nr;
  if (!(tot > 0.0)) return;
  const double rate = na / tot;
  double f = 1.0;
  if (rate < 0.001) f = 0.1;
  else if (rate < 0.05) f = 0.5;
  else if (rate < 0.2) f = 0.9;
  else if (rate > 0.95) f = 10.0;
  else if (rate > 0.75) f = 2.0;
  else if (rate > 0.5) f = 1.1;
  const double ns = s * f;
  na = 0.0;
  nr = 0.0;
  if (ns != 0.0) s = ns;
}

// ---------------------------------------------------------------------------
// LDS carve, in columns of 64 doubles (one per lane); the host computes the same.
// ---------------------------------------------------------------------------
struct nmc_lds_layout {
  int th;      // [P]            current values (control wave writes, all read)
  int part;    // [NACC][16]     per-wave likelihood partial sums (unused slots: -0.0)
  int st;      // [5][P]         scale, log prior, n acc, n rej, total acc (control wave)
  int hyp;     // [6][P]         mu, sd, log sd, sigma2, sqrt(sigma2/G), 1/sd of the hyper-prior
  int hval;    // [2][G + 1]     Gibbs payload of one task, two buffers (payload-in-LDS mode)
  int hst;     // [P][nleaf][8 + ntail]  stream sums / tail elements (pairwise sum)
  int hleaf;   // [P][nleaf]     leaf sums
  int zl;      // [2][2]         {z, log u} of this and the next step (LDS-DMA, step parity)
  int hv;      // [2P]           {hyper z, gamma} of the Gibbs update (LDS-DMA)
  int cw;      // [15]           control-wave temporaries across the step barrier
  int flag;    // [1]            broadcast / epoch words
  int xchg;    // [2][8]         stream sums exchanged by the two compute waves
  int rows;    // [nrows_lds][NF] the group's observation rows (staged once per launch)
  int total;   // columns
};
__host__ __device__ inline nmc_lds_layout nmc_lds(int nacc, int P, int partial, int nleaf,
                                                  int ntail, int W, int G, int hlds,
                                                  int row_doubles = 0) {
  nmc_lds_layout L;
  L.th = 0;
  L.part = L.th + P;
  L.st = L.part + nacc * 16;   // 16 partial slots per accumulator (unused: -0.0)
  L.hyp = L.st + 5 * P;
  L.hval = L.hyp + (partial ? 6 * P : 0);
  L.hst = L.hval + (partial && hlds ? 2 * (G + 1) : 0);   // two task buffers, each + 1 DMA pad
  L.hleaf = L.hst + (partial ? P * nleaf * (8 + ntail) : 0);
  L.zl = L.hleaf + (partial ? P * nleaf : 0);
  L.hv = L.zl + 4;
  L.cw = L.hv + (partial ? 2 * P : 0);
  L.flag = L.cw + 15;
  L.xchg = L.flag + 1;
  L.rows = L.xchg + (partial && hlds ? 16 : 0);
  L.total = L.rows + (row_doubles + 63) / 64;
  return L;
}
enum { NMC_ST_S = 0, NMC_ST_LP, NMC_ST_NA, NMC_ST_NR, NMC_ST_TA };
enum { NMC_HY_MU = 0, NMC_HY_SD, NMC_HY_LSD, NMC_HY_S2, NMC_HY_SDM, NMC_HY_ISD };
// (PAC, PLP, PLL: the decided step's accept flag, log prior and log-likelihood, applied
// to the state by the control wave at the next step, off the critical path)
enum { NMC_CW_LU = 0, NMC_CW_LPC, NMC_CW_LPP, NMC_CW_PROP, NMC_CW_SA, NMC_CW_SR, NMC_CW_NAA,
       NMC_CW_NRA, NMC_CW_NAR, NMC_CW_NRR, NMC_CW_TA, NMC_CW_V, NMC_CW_PAC, NMC_CW_PLP,
       NMC_CW_PLL };

// Where the Gibbs update reads the published values: global (plain loads after a
// kernel boundary / sc1 loads in a persistent launch) or the LDS copy the
// auxiliary waves made during the step-0 likelihood.
enum { NMC_SRC_GLOBAL = 0, NMC_SRC_SC1 = 1, NMC_SRC_LDS = 2 };

template <int SRC>
__device__ __forceinline__ double nmc_ldv(const double* p) {
  if constexpr (SRC == NMC_SRC_SC1)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_load sc1
  else
    return *p;
}

// One wave copies 64 lanes x 16 bytes from global memory straight into LDS
// (global_load_lds_dwordx4: no VGPR destination, so the copy stays in flight across
// the scalar-load likelihood loop).  The issuing wave retires it with its own
// s_waitcnt vmcnt(0) before the barrier that precedes the first read.
typedef __attribute__((address_space(3))) void* nmc_lds_ptr;
typedef __attribute__((address_space(1))) const void* nmc_glb_ptr;
__device__ __forceinline__ void nmc_dma16(const double* src_lane, double* lds_dst) {
  __builtin_amdgcn_global_load_lds((nmc_glb_ptr)src_lane, (nmc_lds_ptr)lds_dst, 16, 0, 0);
}
__device__ __forceinline__ void nmc_drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// Gibbs update of the hyper-parameters after iteration t for chain block cb
// (HyperParameter._updateMean :481-487, _updateVar :489-498, setPrior :273-282),
// cooperatively by ALL threads of the workgroup (contains barriers).
// numpy's pairwise order: leaves of <= 128 groups, each summed as 8 interleaved
// accumulator streams r_j = x_j + x_{j+8} + ... combined ((r0+r1)+(r2+r3))+((r4+r5)+
// (r6+r7)) plus the tail added in sequence; leaves merged in numpy's recursion
// order (d.merge).  One stream per wave-iteration, loads issued together.
// In: values of iteration t ([P][G][C] at src, or the LDS hval copy); LDS hyp
//     sigma2/sdm columns of the previous update; LDS hv = {hyper normal, Gamma(a)
//     draw} of iteration t, [p][lane][2].
// Out: LDS hyp mu/sd/lsd/s2; write: global mu/s2/sd/lsd + the sample row of t.
// ---------------------------------------------------------------------------
template <int SRC, bool SQ>
__device__ __forceinline__ void nmc_hyper_streams(const Dev& d, const double* src, int cc,
                                                  double* lds, const nmc_lds_layout& L) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C, nl = d.nleaf, ncol = 8 + d.ntail;
  const int per = 8 + (d.ntail ? 1 : 0);
  const int nst = P * nl * per;
  for (int s = w; s < nst; s += W) {
    const int j = s % per, pl = s / per;    // pl = p * nleaf + leaf
    const int lf = pl % nl, p = pl / nl;
    const int a = nl == 1 ? 0 : d.leaf[lf], m = nl == 1 ? G : d.leaf[lf + 1] - a;
    const int m8 = m >= 8 ? m - m % 8 : 0;
    // element k of the leaf for this lane's chain
    const double* xp = SRC == NMC_SRC_LDS ? lds + (size_t)(L.hval + p * G + a) * 64 + lane
                                          : src + ((size_t)p * G + a) * C + cc;
    const size_t xs = SRC == NMC_SRC_LDS ? 64 : (size_t)C;
    double* out = lds + (size_t)(L.hst + pl * ncol) * 64 + lane;
    const double mu = SQ ? lds[(L.hyp + NMC_HY_MU * P + p) * 64 + lane] : 0.0;
    if (j < 8) {
      const int cnt = m8 >> 3;   // <= 16
      double t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = u < cnt ? nmc_ldv<SRC>(xp + (size_t)(j + 8 * u) * xs) : 0.0;
      double r = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (u < cnt) {
          double v = t[u];
          if (SQ) {
            v = v - mu;
            v = v * v;
          }
          r = u == 0 ? v : r + v;
        }
      }
      out[j * 64] = r;
    } else {
      for (int u = m8; u < m; ++u) {
        double v = nmc_ldv<SRC>(xp + (size_t)u * xs);
        if (SQ) {
          v = v - mu;
          v = v * v;
        }
        out[(8 + u - m8) * 64] = v;
      }
    }
  }
}

__device__ __forceinline__ double nmc_hyper_combine(const Dev& d, double* lds,
                                                    const nmc_lds_layout& L, int p, int lane) {
  const int nl = d.nleaf, ncol = 8 + d.ntail;
  for (int lf = 0; lf < nl; ++lf) {
    const int pl = p * nl + lf;
    const int m = nl == 1 ? d.G : d.leaf[lf + 1] - d.leaf[lf];
    const int m8 = m >= 8 ? m - m % 8 : 0;
    const double* r = lds + (size_t)(L.hst + pl * ncol) * 64 + lane;
    double res = m8 ? ((r[0] + r[64]) + (r[128] + r[192])) + ((r[256] + r[320]) + (r[384] + r[448]))
                    : 0.0;
    for (int u = m8; u < m; ++u) res += r[(8 + u - m8) * 64];
    lds[(L.hleaf + pl) * 64 + lane] = res;
  }
  for (int k = 0; k < d.nmerge; ++k) {
    double* A = lds + (L.hleaf + p * nl + d.merge[2 * k]) * 64 + lane;
    *A = *A + lds[(L.hleaf + p * nl + d.merge[2 * k + 1]) * 64 + lane];
  }
  return lds[(L.hleaf + p * nl) * 64 + lane];
}

// sqrt(sigma2 / G): the sd of the hyper mean's normal draw (eq. 11.12, :485),
// precomputed off the critical path for the next update.
__device__ __forceinline__ void nmc_hyper_sdm(const Dev& d, double* lds, const nmc_lds_layout& L,
                                              int lane) {
  for (int p = 0; p < d.P; ++p)
    lds[(L.hyp + NMC_HY_SDM * d.P + p) * 64 + lane] =
        sqrt(lds[(L.hyp + NMC_HY_S2 * d.P + p) * 64 + lane] / d.G);
}

// Issue the LDS-DMA of the hyper variates of iteration t (waves w = p % nw from
// w0; one 1 KiB block per parameter); the issuing waves drain before the next barrier.
__device__ __forceinline__ void nmc_hyper_variates(const Dev& d, int cb, int t, double* lds,
                                                   const nmc_lds_layout& L, int w0, int nw) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  for (int p = w - w0; p >= 0 && p < d.P; p += nw)
    nmc_dma16(d.vh + (((size_t)(t - d.vbase) * d.P + p) * d.C + cc) * 2,
              lds + L.hv * 64 + p * 128);
}

template <int SRC>
__device__ __forceinline__ void nmc_hyper(const Dev& d, const double* src, int cb, int t,
                                          double* lds, const nmc_lds_layout& L, bool write) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C;
  const int c = cb * 64 + lane;
  const int cc = c < C ? c : C - 1;
  nmc_hyper_streams<SRC, false>(d, src, cc, lds, L);
  __syncthreads();
  for (int p = w; p < P; p += W) {
    const double tot = nmc_hyper_combine(d, lds, L, p, lane);
    const double sdm = lds[(L.hyp + NMC_HY_SDM * P + p) * 64 + lane];
    const double hz = lds[L.hv * 64 + (p * 64 + lane) * 2];
    lds[(L.hyp + NMC_HY_MU * P + p) * 64 + lane] = tot / G + sdm * hz;   // mu ~ N(mean(x), sqrt(s2/G))
  }
  __syncthreads();
  nmc_hyper_streams<SRC, true>(d, src, cc, lds, L);
  __syncthreads();
  const int row = write ? nmc_record_row(d, t) : -1;
  for (int p = w; p < P; p += W) {
    const double ss = nmc_hyper_combine(d, lds, L, p, lane);
    const double hat = ss / (double)(G - 1);
    const double scale = d.ha * hat;
    const double hx = lds[L.hv * 64 + (p * 64 + lane) * 2 + 1];
    // scipy invgamma.rvs: (1/gammainccinv(a, U)) * scale + loc; loc when scale == 0
    const double s2n = scale == 0.0 ? 0.0 : (1.0 / hx) * scale;
    const double sdn = sqrt(s2n);
    const double lsd = log(sdn);
    const double m = lds[(L.hyp + NMC_HY_MU * P + p) * 64 + lane];
    lds[(L.hyp + NMC_HY_SD * P + p) * 64 + lane] = sdn;
    lds[(L.hyp + NMC_HY_LSD * P + p) * 64 + lane] = lsd;
    lds[(L.hyp + NMC_HY_S2 * P + p) * 64 + lane] = s2n;
    lds[(L.hyp + NMC_HY_ISD * P + p) * 64 + lane] = 1.0 / sdn;
    if (write && c < C) {
      const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
      d.mu[ho] = m;
      d.s2[ho] = s2n;
      d.hsd[ho] = sdn;
      d.hlsd[ho] = lsd;
      if (row >= 0) {
        double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
        out[0] = m;
        out[C] = s2n;
      }
    }
  }
  __syncthreads();
}

// ONE wave computes the Gibbs update of parameter p after iteration t for its 64
// chains (persistent payload-in-LDS mode, run by an auxiliary wave during the step-0
// likelihood): the chain block's published values of p (sc1 loads) are staged in
// LDS hval[p], then numpy's pairwise sums give mean and variance (G <= 128: one
// numpy leaf; the host enables this mode only then).
// hz/hx: this lane's hyper variates of (t, p).  Writes the LDS hyp columns of p.
// numpy's pairwise sum of one leaf (n <= 128 values v[i * 64], optionally squared
// deviations from mu): r_j = x_j + x_{j+8} + ..., ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
// then the n % 8 tail in order; n < 8: a plain sequential sum from 0.
template <bool SQ>
__device__ __forceinline__ double nmc_leaf_sum(const double* v, int n, double mu) {
  auto f = [&](int i) -> double {
    double x = v[i * 64];
    if (SQ) {
      x = x - mu;
      x = x * x;
    }
    return x;
  };
  const int m8 = n >= 8 ? n - n % 8 : 0;
  double res = 0.0;
  if (m8) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f(j);
    for (int i = 8; i < m8; i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + f(i + j);
    }
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
  for (int i = m8; i < n; ++i) res += f(i);
  return res;
}

// Groups [kb, ke) of the chain block's published values of parameter p (64 chains
// each) -> LDS hval, sc1 loads, 8 in flight (used when C is odd).
__device__ __forceinline__ void nmc_hyper_load(const Dev& d, const double* src, int p, int cc,
                                               int kb, int ke, double* lds,
                                               const nmc_lds_layout& L, int hoff) {
  const int lane = threadIdx.x & 63;
  const int C = d.C;
  src += (size_t)p * d.G * C;
  constexpr int NB = 8;   // the odd-C fallback of the LDS-DMA copy: few registers
  for (int k0 = kb; k0 < ke; k0 += NB) {
    double tv[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      tv[u] = k0 + u < ke ? nmc_ldv<NMC_SRC_SC1>(src + (size_t)(k0 + u) * C + cc) : 0.0;
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (k0 + u < ke) lds[(size_t)(L.hval + hoff + k0 + u) * 64 + lane] = tv[u];
  }
}

// The same by LDS-DMA (global_load_lds_dwordx4, sc1): one instruction moves two groups'
// 64-chain rows (lanes 0-31 / 32-63, two chains per lane) into two consecutive hval
// columns, so one wave has the whole payload in flight without registers.  Needs C
// even (16-byte rows); an odd group count writes one pad column past ke.  The issuing
// wave retires the copies with s_waitcnt vmcnt(0).
__device__ __forceinline__ void nmc_hyper_dma(const Dev& d, const double* src, int p, int cb,
                                              int kb, int ke, double* lds,
                                              const nmc_lds_layout& L, int hoff) {
  const int lane = threadIdx.x & 63;
  const double* s = src + (size_t)p * d.G * d.C + (size_t)cb * 64 + 2 * (lane & 31);
  for (int k0 = kb; k0 < ke; k0 += 2) {
    const int gk = k0 + (lane >> 5) < ke ? k0 + (lane >> 5) : ke - 1;
    __builtin_amdgcn_global_load_lds((nmc_glb_ptr)(s + (size_t)gk * d.C),
                                     (nmc_lds_ptr)(lds + (size_t)(L.hval + hoff + k0) * 64), 16,
                                     0, 16 /* sc1 */);
  }
}

// The Gibbs update of parameter p after iteration t for this wave's 64 chains from
// the LDS copy hval of p's values (G <= 128: one numpy leaf).  hz/hx: this lane's hyper
// variates of (t, p).  Writes the LDS hyp columns of p (and, if write, global + row).
__device__ __forceinline__ void nmc_hyper_compute(const Dev& d, int cb, int t, int p, double* lds,
                                                  const nmc_lds_layout& L, bool write, double hz,
                                                  double hx, int hoff) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G, C = d.C;
  const int c = cb * 64 + lane;
  const double* hv = lds + (size_t)(L.hval + hoff) * 64 + lane;   // hv[i * 64]: group i of p
  double* hy = lds + L.hyp * 64 + lane;
  const double sdm = sqrt(hy[(NMC_HY_S2 * P + p) * 64] / G);
  const double tot = nmc_leaf_sum<false>(hv, G, 0.0);
  const double mu = tot / G + sdm * hz;                        // mu ~ N(mean(x), sqrt(s2/G))
  const double ss = nmc_leaf_sum<true>(hv, G, mu);
  const double hat = ss / (double)(G - 1);
  const double scale = d.ha * hat;
  // scipy invgamma.rvs: (1/gammainccinv(a, U)) * scale + loc; loc when scale == 0
  const double s2n = scale == 0.0 ? 0.0 : (1.0 / hx) * scale;
  const double sdn = sqrt(s2n);
  const double lsd = log(sdn);
  hy[(NMC_HY_MU * P + p) * 64] = mu;
  hy[(NMC_HY_SD * P + p) * 64] = sdn;
  hy[(NMC_HY_LSD * P + p) * 64] = lsd;
  hy[(NMC_HY_S2 * P + p) * 64] = s2n;
  hy[(NMC_HY_ISD * P + p) * 64] = 1.0 / sdn;
  if (write && c < C) {
    const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
    d.mu[ho] = mu;
    d.s2[ho] = s2n;
    d.hsd[ho] = sdn;
    d.hlsd[ho] = lsd;
    const int row = nmc_record_row(d, t);
    if (row >= 0) {
      double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
      out[0] = mu;
      out[C] = s2n;
    }
  }
}

// The same update split over two waves (half 0 / 1 sum numpy streams 0-3 / 4-7 of both
// leaf sums and swap the stream sums through LDS, so both combine all eight in numpy's
// order); half 0 finishes and writes.  epoch: unique per task, > every earlier one.
// Both waves must call it (bounded spins).  Needs G >= 8.
__device__ __forceinline__ void nmc_hyper_compute2(const Dev& d, int cb, int t, int p, double* lds,
                                                   const nmc_lds_layout& L, bool write, double hz,
                                                   double hx, int hoff, int half, double epoch) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G, C = d.C;
  const int c = cb * 64 + lane;
  const double* hv = lds + (size_t)(L.hval + hoff) * 64 + lane;
  double* hy = lds + L.hyp * 64 + lane;
  double* xc = lds + (size_t)L.xchg * 64 + lane;
  double* fl = lds + L.flag * 64 + 16;
  const double sdm = sqrt(hy[(NMC_HY_S2 * P + p) * 64] / G);
  const int m8 = G - G % 8;
  auto leaf = [&](int st, bool sq, double mu) -> double {
    auto f = [&](int i) -> double {
      double x = hv[i * 64];
      if (sq) {
        x = x - mu;
        x = x * x;
      }
      return x;
    };
    double r[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) r[jj] = f(4 * half + jj);
    for (int i = 8; i < m8; i += 8) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) r[jj] = r[jj] + f(i + 4 * half + jj);
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) xc[(st * 8 + 4 * half + jj) * 64] = r[jj];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(fl + st * 2 + half, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (unsigned spins = 0;
         __hip_atomic_load(fl + st * 2 + (1 - half), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) !=
             epoch &&
         spins < NMC_SPIN_LIMIT;
         ++spins)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double rr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) rr[j] = xc[(st * 8 + j) * 64];
    double res = ((rr[0] + rr[1]) + (rr[2] + rr[3])) + ((rr[4] + rr[5]) + (rr[6] + rr[7]));
    for (int i = m8; i < G; ++i) res += f(i);
    return res;
  };
  const double tot = leaf(0, false, 0.0);
  const double mu = tot / G + sdm * hz;
  const double ss = leaf(1, true, mu);
  if (half != 0) return;
  const double hat = ss / (double)(G - 1);
  const double scale = d.ha * hat;
  const double s2n = scale == 0.0 ? 0.0 : (1.0 / hx) * scale;
  const double sdn = sqrt(s2n);
  const double lsd = log(sdn);
  hy[(NMC_HY_MU * P + p) * 64] = mu;
  hy[(NMC_HY_SD * P + p) * 64] = sdn;
  hy[(NMC_HY_LSD * P + p) * 64] = lsd;
  hy[(NMC_HY_S2 * P + p) * 64] = s2n;
  hy[(NMC_HY_ISD * P + p) * 64] = 1.0 / sdn;
  if (write && c < C) {
    const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
    d.mu[ho] = mu;
    d.s2[ho] = s2n;
    d.hsd[ho] = sdn;
    d.hlsd[ho] = lsd;
    const int row = nmc_record_row(d, t);
    if (row >= 0) {
      double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
      out[0] = mu;
      out[C] = s2n;
    }
  }
}

// The calling wave polls the chain block's publish counter until it reaches target
// (bounded; a timeout is recorded in d.tmo and reported by the host).  The counter is
// sharded 8 ways (workgroup g adds to shard g % 8, each shard on its own 128-B line)
// so the G arrivals do not serialise on one line; lanes 0-7 read the shards with one
// sc1 load and the wave sums them.  Wave-uniform result; call with the whole wave.
__device__ __forceinline__ unsigned* nmc_counter(const Dev& d, int cb, int p, int shard) {
  return d.cnt + (((size_t)cb * d.P + p) * 8 + shard) * 32;
}
__device__ __forceinline__ bool nmc_poll_published(const Dev& d, int cb, int p, unsigned target) {
  const int lane = threadIdx.x & 63;
  unsigned* ctr = nmc_counter(d, cb, p, lane & 7);
  for (unsigned spins = 0;; ++spins) {
    const unsigned v =
        lane < 8 ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += __builtin_amdgcn_readlane(v, k);
    if (tot >= target) return true;
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
      return false;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Whole-workgroup wait (thread 0 polls, result broadcast through LDS).
__device__ __forceinline__ bool nmc_wait_published(const Dev& d, int cb, int p, unsigned target,
                                                   double* lds, const nmc_lds_layout& L) {
  if (threadIdx.x < 64) {
    const bool r = nmc_poll_published(d, cb, p, target);
    if (threadIdx.x == 0) lds[L.flag * 64] = r ? 1.0 : 0.0;
  }
  __syncthreads();
  // keep the payload loads below the poll (no instruction: wavefront scope)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return lds[L.flag * 64] != 0.0;
}

// ---------------------------------------------------------------------------
// log-likelihood of one group over one row range, chain-on-lane: n rows from p
// (wave-uniform address: scalar loads from global memory, broadcast ds_reads from
// LDS), R rows (~BLK doubles) per block, four accumulator sets to break the
// dependence chain.
// ---------------------------------------------------------------------------
template <class Fam, int BLK = 16>
__device__ __forceinline__ void nmc_ll_rows(const Fam& fam, const typename Fam::Reg& reg,
                                            const double* __restrict__ p, int n,
                                            double (&acc)[Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  constexpr int R = (BLK / NF) > 0 ? (BLK / NF) : 1;
  double a[4][Fam::NACC];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) a[s][k] = 0.0;
  const int nb = n / R;
  for (int b = 0; b < nb; ++b) {
    double cur[R * NF];
#pragma unroll
    for (int j = 0; j < R * NF; ++j) cur[j] = p[(size_t)b * (R * NF) + j];
    fam.template accumN<R>(reg, cur, a);
  }
  for (int r = nb * R; r < n; ++r) fam.accum(reg, p + (size_t)r * NF, a[0]);
#pragma unroll
  for (int k = 0; k < Fam::NACC; ++k) acc[k] = (a[0][k] + a[1][k]) + (a[2][k] + a[3][k]);
}

// The same over rows staged in LDS: blocks of R rows read with wave-uniform
// (broadcast) ds_reads; block b+1 is requested before block b is consumed (LDS
// returns in order, so the wait covers only block b).
#ifndef NMC_LDS_ROW_DOUBLES
#define NMC_LDS_ROW_DOUBLES 16   // doubles per software-pipelined LDS block (8 regression rows)
#endif
template <class Fam>
__device__ __forceinline__ void nmc_ll_rows_lds(const Fam& fam, const typename Fam::Reg& reg,
                                                const double* __restrict__ p, int n,
                                                double (&acc)[Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  // 8-row blocks for 2-field rows (measured: -17 % per iteration for regression),
  // 8 doubles otherwise (register pressure of the wider families)
  constexpr int BD = NF <= 2 ? NMC_LDS_ROW_DOUBLES : 8;
  constexpr int R = (BD / NF) > 0 ? (BD / NF) : 1;
  double a[4][Fam::NACC];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) a[s][k] = 0.0;
  const int nb = n / R;
  if (nb > 0) {
    double cur[R * NF];
#pragma unroll
    for (int j = 0; j < R * NF; ++j) cur[j] = p[j];
    for (int b = 0; b < nb; ++b) {
      const int bn = b + 1 < nb ? b + 1 : b;
      double nxt[R * NF];
#pragma unroll
      for (int j = 0; j < R * NF; ++j) nxt[j] = p[(size_t)bn * (R * NF) + j];
      fam.template accumN<R>(reg, cur, a);
#pragma unroll
      for (int j = 0; j < R * NF; ++j) cur[j] = nxt[j];
    }
  }
  for (int r = nb * R; r < n; ++r) fam.accum(reg, p + (size_t)r * NF, a[0]);
#pragma unroll
  for (int k = 0; k < Fam::NACC; ++k) acc[k] = (a[0][k] + a[1][k]) + (a[2][k] + a[3][k]);
}

// Chunk k of nchunks of [r0, r1) (contiguous, balanced).
__device__ __forceinline__ void nmc_chunk(int64_t r0, int64_t r1, int k, int nchunks,
                                          int64_t* a, int* n) {
  const int64_t len = r1 - r0;
  const int64_t per = (len + nchunks - 1) / nchunks;
  int64_t s = r0 + (int64_t)k * per;
  int64_t e = s + per;
  if (s > r1) s = r1;
  if (e > r1) e = r1;
  *a = s;
  *n = (int)(e - s);
}

// theta[q] = src[q][g][c] for q < P.
template <int MP>
__device__ __forceinline__ void nmc_load_theta(const Dev& d, const double* src, int g, int c,
                                               double (&th)[MP]) {
#pragma unroll
  for (int q = 0; q < MP; ++q) {
    th[q] = 0.0;
    if (q < d.P) th[q] = src[((size_t)q * d.G + g) * d.C + c];
  }
}

// ---------------------------------------------------------------------------
// K_run: iterations [i0, i1) for every (chain, group); grid = CB*G workgroups of
// 64*W threads; dynamic LDS = nmc_lds(...).total columns.
// Wave roles (W > 1):
//   wave 0            control: proposal priors, Metropolis decision, tuning, state,
//                     sample/trace stores, variate DMA, publishing (no likelihood);
//   waves 1..NAUX     auxiliary (partial, payload-in-LDS mode): during the step-0
//                     likelihood they wait for the chain block's values and copy them
//                     into LDS; on every other step they evaluate likelihood tiles;
//   remaining waves   likelihood tiles.
// W == 1: the single wave does everything.
// Likelihood: each likelihood wave sums a contiguous row range; the control wave adds
// the partials in a fixed order.  W and the row ranges depend only on (N, P, G), and
// step 0 of partial pooling always uses the W-1-NAUX non-auxiliary waves, so the
// sums -- and the chains -- do not depend on the chain-block count, the launch mode
// or the number of GPUs.
//   flags & NMC_RUN_HYPER_LOAD: the hyper-parameters after iteration i0-1 are in
//     global memory (chunk start / initial state); otherwise (launch per iteration)
//     they are recomputed from vb[(i0-1)&1] at step 0 of i0.
//   MODE SYNC / SYNC_LDS (partial, persistent): publish every iteration, wait on
//     the chain block's counter before each Gibbs update, close with the update
//     after i1-1 (workgroups of group 0, which also record it).
// ---------------------------------------------------------------------------
// MODE: how the partial-pooling Gibbs update gets the chain block's values.
enum { NMC_MODE_NOPOOL = 0,      // none/complete pooling: no coupling
       NMC_MODE_LAUNCH = 1,      // one launch per iteration, plain loads after the boundary
       NMC_MODE_SYNC = 2,        // persistent, sc1 loads after the barrier
       NMC_MODE_SYNC_LDS = 3 };  // persistent, auxiliary waves copy the payload into LDS
template <class Fam, int MODE>
__global__ void __launch_bounds__(1024)
nmc_k_run(Dev d, Fam fam, const double* __restrict__ obs, int i0, int i1, int flags) {
  constexpr bool PARTIAL = MODE != NMC_MODE_NOPOOL;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C;
  const int b = blockIdx.x;
  const int g = b % G, cb = b / G;
  const int c = cb * 64 + lane;
  const bool live = c < C;
  const int cc = live ? c : C - 1;
  constexpr bool sync = MODE == NMC_MODE_SYNC || MODE == NMC_MODE_SYNC_LDS;
  constexpr bool hl = MODE == NMC_MODE_SYNC_LDS;  // payload-in-LDS Gibbs update
  const int naux = d.naux;       // reserved at step 0 of partial pooling in every mode
  const int row_doubles = d.rows_lds ? d.nmax * Fam::NFIELDS : 0;
  const nmc_lds_layout L =
      nmc_lds(Fam::NACC, P, PARTIAL, d.nleaf, d.ntail, W, G, hl ? 1 : 0, row_doubles);
  double* th = lds + L.th * 64 + lane;            // th[p * 64]: this lane's chain, parameter p
  double* st = lds + L.st * 64 + lane;            // st[(k * P + p) * 64]
  double* hy = lds + L.hyp * 64 + lane;           // hy[(k * P + p) * 64]
  const int64_t r0 = d.off[g];
  const int nrow = (int)(d.off[g + 1] - r0);
  const double* grows = obs + r0 * Fam::NFIELDS;
  const size_t PGC = (size_t)P * G * C;
  const size_t gc = (size_t)g * C + cc;
  const bool ctl = w == 0;
  // latency-bound roles (control, loaders, compute) issue ahead of the likelihood waves
  // sharing their SIMD, which fill the gaps
  if (W > 1 && w <= naux && !(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);

  // ---- prologue: values and state -> LDS (parameter p by wave p % W) ----
  const double* vin = ((i0 - 1) & 1) ? d.vb1 : d.vb0;
  for (int p = w; p < P; p += W) {
    const size_t ip = (size_t)p * G * C + gc;
    th[p * 64] = vin[ip];
    st[(NMC_ST_S * P + p) * 64] = d.scale[ip];
    st[(NMC_ST_LP * P + p) * 64] = d.lp[ip];
    st[(NMC_ST_NA * P + p) * 64] = (double)d.nacc[ip];
    st[(NMC_ST_NR * P + p) * 64] = (double)d.nrej[ip];
    st[(NMC_ST_TA * P + p) * 64] = (double)d.tacc[ip];
    if (PARTIAL) {
      // hyper-parameters after iteration i0-1 (chunk start), or after i0-2 when this
      // launch recomputes the update after i0-1 at step 0 (launch per iteration): that
      // update is written to the other slot, so no workgroup of this launch can read it
      const size_t ho =
          nmc_hslot(d, (flags & NMC_RUN_HYPER_LOAD) ? i0 - 1 : i0 - 2) + (size_t)p * C + cc;
      const double s2 = d.s2[ho];
      hy[(NMC_HY_MU * P + p) * 64] = d.mu[ho];
      hy[(NMC_HY_SD * P + p) * 64] = d.hsd[ho];
      hy[(NMC_HY_LSD * P + p) * 64] = d.hlsd[ho];
      hy[(NMC_HY_S2 * P + p) * 64] = s2;
      hy[(NMC_HY_SDM * P + p) * 64] = sqrt(s2 / G);
      hy[(NMC_HY_ISD * P + p) * 64] = 1.0 / d.hsd[ho];
    }
  }
  const double gcst = fam.gconst((long)nrow);   // per-group constant of finish_fast
  double LL = d.ll[gc];
  double* lrows = lds + L.rows * 64;
  if (d.rows_lds) {   // this group's rows -> LDS, once for the whole launch
    const int nd = nrow * Fam::NFIELDS;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
  }
  auto zl_src = [&](int tn, int pn) -> const double* {
    return d.vzl + ((size_t)(tn - d.vbase) * PGC + (size_t)pn * G * C + gc) * 2;
  };
  const int l0 = W == 1 ? 0 : 1 + naux;   // likelihood waves l0..W-1
  const int nll = W - l0;
  if (ctl) {     // {z, log u} of the first step -> LDS slot of step i0*P
    nmc_dma16(zl_src(i0, 0), lds + (L.zl + 2 * ((i0 * P) & 1)) * 64);
    for (int j = 0; j < Fam::NACC; ++j)   // x + (-0.0) == x: the fixed 16-slot sum
      for (int k = nll; k < 16; ++k) lds[(L.part + j * 16 + k) * 64 + lane] = -0.0;
    nmc_drain_vm();
    lds[L.flag * 64 + lane] = 0.0;
  }
  __syncthreads();

  bool ok = true;
  int pub_p = -1;     // control wave: parameter whose sc1 value store awaits its counter add
  int pend_p = -1, pend_t = 0;   // control wave: decided step whose state update is pending
  double* cwv = lds + L.cw * 64 + lane;    // cwv[k * 64]
  // the rest of a decided step's state update (:369-383, :608-610): counters, log prior,
  // log-likelihood, sample and trace rows
  auto apply_pending = [&]() {
    const int q = pend_p, tq = pend_t;
    const bool accept = cwv[NMC_CW_PAC * 64] != 0.0;
    const double llp = cwv[NMC_CW_PLL * 64];
    st[(NMC_ST_LP * P + q) * 64] = cwv[NMC_CW_PLP * 64];
    st[(NMC_ST_NA * P + q) * 64] = cwv[(accept ? NMC_CW_NAA : NMC_CW_NAR) * 64];
    st[(NMC_ST_NR * P + q) * 64] = cwv[(accept ? NMC_CW_NRA : NMC_CW_NRR) * 64];
    st[(NMC_ST_TA * P + q) * 64] = cwv[NMC_CW_TA * 64] + (accept ? 1.0 : 0.0);
    if (accept) LL = llp;
    if (live) {
      const int row = nmc_record_row(d, tq);
      if (row >= 0) {
        const int col = q * (G + (PARTIAL ? 2 : 0)) + (PARTIAL ? 2 : 0) + g;
        d.samples[((size_t)row * d.cols + col) * C + c] = th[q * 64];
      }
      if (tq < d.trace_n) {
        const size_t it = (((size_t)tq * P + q) * G + g) * C + c;
        d.tflag[it] = accept ? 1 : 0;
        d.tllp[it] = llp;
      }
    }
    pend_p = -1;
  };
  for (int t = i0; t < i1 && ok; ++t) {
    NMC_STAMP(t, 0);
    const bool tune = t > 0 && t < d.burn && t % d.tune_interval == 0;
    for (int p = 0; p < P; ++p) {
      const int sp = (t * P + p) & 1;
      // Gibbs update of every parameter at step 0 (launch-per-iteration / fallback)
      const bool hyper_now =
          !hl && PARTIAL && p == 0 && t > 0 && !(t == i0 && (flags & NMC_RUN_HYPER_LOAD));
      // payload-in-LDS: the Gibbs update of parameter q after iteration tq is task
      // k = tq*P + q; every workgroup publishes it right after its decision at global step
      // k, so it is counted at the start of step k+1.  P == 1: the auxiliary waves load and
      // compute task gs-1 at step gs (needed at once).  P >= 2 (two-stage pipeline): the
      // loader waves copy task gs-1 into LDS buffer (gs-1)&1 at step gs, the compute wave
      // updates task gs-2 from buffer gs&1 -- needed first at step gs-2+P.
      const int gs = t * P + p, gs0 = i0 * P;
      const bool pipe = hl && P >= 2;
      const int aq = p > 0 ? p - 1 : P - 1;        // loaders' task: (atq, aq) = gs-1
      const int atq = p > 0 ? t : t - 1;
      const bool aux_now = hl && gs - 1 >= gs0;
      const bool comp_now = pipe && gs - 2 >= gs0;  // compute wave's task: (ctq, cq) = gs-2
      const int cq = (p + 2 * P - 2) % (P > 0 ? P : 1);
      const int ctq = p >= 2 ? t : t - 1;
      // the update of this step's parameter lands during this step (P <= 2): priors
      // after the barrier
      const bool post_prior = P == 1 ? aux_now : (P == 2 && comp_now);
      // proposal (Parameter.propose :304-306): value + (proposalSd=1 * scale) * z
      const double v = th[p * 64];
      const double s = st[(NMC_ST_S * P + p) * 64];
      const double zc = lds[(L.zl + 2 * sp) * 64 + 2 * lane];
      const double prop = v + (1.0 * s) * zc;
      // this step's priors (:293-294) from the hyper-parameters in LDS -- by the wave that
      // has just updated them when that update lands during this step (post_prior)
      auto step_priors = [&]() {
        const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
        const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
        cwv[NMC_CW_LPC * 64] =
            t > 0 ? nmc_norm_logpdf_r(v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
        cwv[NMC_CW_LPP * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
      };
      // ---- control wave, before the barrier: next variates in flight, priors, and both
      //      outcomes of the decision -- accept (sA, naA, nrA, ta + 1) / reject (sR,
      //      naR, nrR, ta), tuned if due -- parked in LDS (no registers live across
      //      the likelihood region) ----
      if (ctl) {
        if constexpr (sync) {   // the previous step's value is stored; count it published
          if (pub_p >= 0) {
            nmc_drain_vm();
            if (lane == 0)
              __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            pub_p = -1;
          }
        }
        // P >= 2: the control wave is the loader, right after its own publish (the copies
        // stay in flight under the rest of its pre-barrier work): it waits for the chain
        // block's counter of task gs-1 (verdict word for the check after barrier A) and
        // copies the payload into LDS buffer (gs-1)&1 (sc1 LDS-DMA, drained with its other
        // copies before barrier A)
        if constexpr (hl) if (pipe && aux_now) {
          const bool r = nmc_poll_published(d, cb, aq, (unsigned)G * (unsigned)(atq - i0 + 1));
          if (lane == 0)
            __hip_atomic_store(lds + L.flag * 64 + 1, r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (p == 0) NMC_STAMP(t, 8);
          if (r) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double* src = (atq & 1) ? d.vb1 : d.vb0;
            if ((C & 1) == 0)
              nmc_hyper_dma(d, src, aq, cb, 0, G, lds, L, ((gs - 1) & 1) * (G + 1));
            else
              nmc_hyper_load(d, src, aq, cc, 0, G, lds, L, ((gs - 1) & 1) * (G + 1));
          }
        }
        if (pend_p >= 0) apply_pending();
        {
          const double na = st[(NMC_ST_NA * P + p) * 64], nr = st[(NMC_ST_NR * P + p) * 64];
          double sA = s, sR = s, naA = na + 1.0, nrA = nr, naR = na, nrR = nr + 1.0;
          if (tune) {
            nmc_tune(sA, naA, nrA);
            nmc_tune(sR, naR, nrR);
          }
          cwv[NMC_CW_SA * 64] = sA;
          cwv[NMC_CW_SR * 64] = sR;
          cwv[NMC_CW_NAA * 64] = naA;
          cwv[NMC_CW_NRA * 64] = nrA;
          cwv[NMC_CW_NAR * 64] = naR;
          cwv[NMC_CW_NRR * 64] = nrR;
          cwv[NMC_CW_TA * 64] = st[(NMC_ST_TA * P + p) * 64];
        }
        cwv[NMC_CW_LU * 64] = lds[(L.zl + 2 * sp) * 64 + 2 * lane + 1];
        cwv[NMC_CW_PROP * 64] = prop;
        cwv[NMC_CW_V * 64] = v;
        const int tn = p + 1 < P ? t : t + 1;
        const int pn = p + 1 < P ? p + 1 : 0;
        if (tn < i1) nmc_dma16(zl_src(tn, pn), lds + (L.zl + 2 * (sp ^ 1)) * 64);
        if (!hl && hyper_now) nmc_hyper_variates(d, cb, t - 1, lds, L, 0, 1);
        if (PARTIAL && !hl && p == (P > 1 ? 1 : 0)) nmc_hyper_sdm(d, lds, L, lane);
        if (!hyper_now && !(hl && post_prior)) {   // priors (:293-294)
          double lpc, lpp;
          if (PARTIAL) {
            const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
            const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
            lpc = t > 0 ? nmc_norm_logpdf_r(v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
            lpp = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
          } else {
            lpc = st[(NMC_ST_LP * P + p) * 64];
            lpp = nmc_prior_logpdf(d.pfam[p], d.ppar + 8 * p, prop);
          }
          cwv[NMC_CW_LPC * 64] = lpc;
          cwv[NMC_CW_LPP * 64] = lpp;
        }
      }
      // ---- auxiliary waves, overlapped with this step's likelihood: loader wave 1 waits
      //      for the chain block's counter of task gs-1, each loader copies its share of
      //      the groups' values into LDS (one batch of sc1 loads); P == 1: they join
      //      through LDS epoch words and wave 1 computes; P >= 2: the compute wave (the
      //      last auxiliary) updates task gs-2 from the buffer the loaders filled at the
      //      previous step ----
      const int nload = pipe ? 0 : naux;   // P >= 2: the control wave loads, waves 1-2 compute
      const bool aux = hl && w >= 1 && w <= naux && (w <= nload ? aux_now : comp_now);
      if constexpr (hl) if (aux) {
        const int a = w - 1;
        if (a < nload) {
          double hz = 0.0, hx = 0.0;
          if (!pipe && a == 0) {   // this lane's hyper variates of (atq, aq), issued early
            const size_t hvi = (((size_t)(atq - d.vbase) * P + aq) * C + cc) * 2;
            hz = d.vh[hvi];
            hx = d.vh[hvi + 1];
          }
          const double want = 2.0 * ((double)gs + 1);      // this step's epoch
          double* flagw = lds + L.flag * 64 + 1;
          if (a == 0) {
            const bool r = nmc_poll_published(d, cb, aq, (unsigned)G * (unsigned)(atq - i0 + 1));
            if (lane == 0)
              __hip_atomic_store(flagw, r ? want : -want, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          double f;
          while (true) {
            f = __hip_atomic_load(flagw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (f == want || f == -want) break;
            __builtin_amdgcn_s_sleep(1);
          }
          // keep the payload loads below the poll (no instruction: wavefront scope)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (p == 0) NMC_STAMP_AUX(t, 13);
          if (f == want) {
            const double* src = (atq & 1) ? d.vb1 : d.vb0;
            if (nload == 1 && (C & 1) == 0) {
              nmc_hyper_dma(d, src, aq, cb, 0, G, lds, L, ((gs - 1) & 1) * (G + 1));
              nmc_drain_vm();
            } else {
              nmc_hyper_load(d, src, aq, cc, (int)(((int64_t)G * a) / nload),
                             (int)(((int64_t)G * (a + 1)) / nload), lds, L, ((gs - 1) & 1) * (G + 1));
            }
            if (p == 0) NMC_STAMP_AUX(t, 14);
            if (!pipe) {
              // join: each loader stamps its LDS word with the epoch once its share has
              // landed; wave 1 waits for all of them (bounded)
              double* joinw = lds + L.flag * 64 + 8;
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              if (lane == 0)
                __hip_atomic_store(joinw + a, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (a == 0) {
                for (int k = 1; k < nload; ++k)
                  for (unsigned spins = 0;
                       __hip_atomic_load(joinw + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) !=
                           want &&
                       spins < NMC_SPIN_LIMIT;
                       ++spins)
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (p == 0) NMC_STAMP_AUX(t, 15);
                nmc_hyper_compute(d, cb, atq, aq, lds, L, g == 0, hz, hx, ((gs - 1) & 1) * (G + 1));
                if (post_prior) step_priors();
                if (p == 0) NMC_STAMP_AUX(t, 12);
              }
            }
          }
        } else {   // compute waves: task gs-2, loaded into buffer (gs-2)&1 at step gs-1
          const int half = w - nload - 1;
          const size_t hvi = (((size_t)(ctq - d.vbase) * P + cq) * C + cc) * 2;
          if (p == 0) NMC_STAMP_CMP(t, 13);
          if (G >= 8)
            nmc_hyper_compute2(d, cb, ctq, cq, lds, L, g == 0, d.vh[hvi], d.vh[hvi + 1],
                               (gs & 1) * (G + 1), half, (double)(gs + 1));
          else if (half == 0)
            nmc_hyper_compute(d, cb, ctq, cq, lds, L, g == 0, d.vh[hvi], d.vh[hvi + 1],
                              (gs & 1) * (G + 1));
          if (p == 0) NMC_STAMP_CMP(t, 14);
          if (post_prior && half == 0) step_priors();
          if (p == 0) NMC_STAMP_CMP(t, 15);
        }
      }
      // ---- likelihood of the proposal over this wave's rows (:615-635) ----
      if (w >= l0 && !aux) {
        const int k = w - l0;
        int64_t ra;
        int rn;
        nmc_chunk(0, nrow, k, nll, &ra, &rn);
        double thp[Fam::MAXP];
#pragma unroll
        for (int q = 0; q < Fam::MAXP; ++q) thp[q] = q < P ? (q == p ? prop : th[q * 64]) : 0.0;
        const typename Fam::Reg reg = fam.prepare(thp);
        double acc[Fam::NACC];
        if (d.rows_lds)   // wave-uniform LDS address: broadcast ds_reads, software-pipelined
          nmc_ll_rows_lds(fam, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc);
        else              // wave-uniform global address: scalar loads
          nmc_ll_rows(fam, reg, grows + (size_t)ra * Fam::NFIELDS, rn, acc);
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j) lds[(L.part + j * 16 + k) * 64 + lane] = acc[j];
      }
      NMC_STAMP(t, 1 + 3 * (p & 1));
      if (ctl) nmc_drain_vm();   // this wave's LDS-DMA has landed
      __syncthreads();
      NMC_STAMP(t, 2 + 3 * (p & 1));

      // ---- Gibbs update after iteration t-1 (needed by this iteration's priors) ----
      if constexpr (hl) {
        if (aux_now) {   // the loaders' verdict
          ok = lds[L.flag * 64 + 1] == 2.0 * ((double)gs + 1);
          if (!ok) break;
        }
      }
      if constexpr (PARTIAL && !hl) if (hyper_now) {
        if constexpr (sync) {   // every parameter of t-1 is published once P-1's count is full
          ok = nmc_wait_published(d, cb, P - 1, (unsigned)G * (unsigned)(t - i0), lds, L);
          if (!ok) break;
          nmc_hyper<NMC_SRC_SC1>(d, ((t - 1) & 1) ? d.vb1 : d.vb0, cb, t - 1, lds, L, g == 0);
        } else {
          nmc_hyper<NMC_SRC_GLOBAL>(d, ((t - 1) & 1) ? d.vb1 : d.vb0, cb, t - 1, lds, L, g == 0);
        }
        if (ctl) {
          const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
          const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
          const double vv = cwv[NMC_CW_V * 64], pp = cwv[NMC_CW_PROP * 64];
          cwv[NMC_CW_LPC * 64] = nmc_norm_logpdf_r(vv, m, sd, isd, lsd);   // t > 0 (setPrior :281)
          cwv[NMC_CW_LPP * 64] = nmc_norm_logpdf_r(pp, m, sd, isd, lsd);
        }
        NMC_STAMP(t, 9);
      }

      // ---- control wave: group log-likelihood of the proposal (tiles in order) and
      //      the Metropolis decision, one chain per lane (:334-383) ----
      if (ctl) {
        double acc[Fam::NACC];
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j) {
          // the likelihood waves' partials in a fixed order: wave k into accumulator
          // k % 4, combined (a0+a1)+(a2+a3); every LDS read in flight at once (slots
          // past the last likelihood wave hold -0.0)
          const double* pt = lds + (L.part + j * 16) * 64 + lane;
          double a4[4] = {0.0, 0.0, 0.0, 0.0};
          double v16[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v16[u] = pt[u * 64];
#pragma unroll
          for (int u = 0; u < 16; ++u)
            a4[u & 3] = u < 4 ? v16[u] : a4[u & 3] + v16[u];
          acc[j] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        }
        if (p == 0) NMC_STAMP(t, 10);
        const double prop = cwv[NMC_CW_PROP * 64], v = cwv[NMC_CW_V * 64];
        const double lpc = cwv[NMC_CW_LPC * 64], lpp = cwv[NMC_CW_LPP * 64];
        const double lu = cwv[NMC_CW_LU * 64];
        double thp[Fam::MAXP];
#pragma unroll
        for (int q = 0; q < Fam::MAXP; ++q) thp[q] = q < P ? (q == p ? prop : th[q * 64]) : 0.0;
        const typename Fam::Reg reg = fam.prepare(thp);
        const double llp = fam.finish_fast(reg, acc, (long)nrow, gcst);
        if (p == 0) NMC_STAMP(t, 11);
        const double postp = lpp + llp;
        const double post = lpc + LL;
        const double diff = postp - post;
        bool accept;
        if (!isfinite(post) && isfinite(postp)) accept = true;        // :347-352
        else if (!isfinite(llp)) accept = false;                      // :354-356
        else if (!isfinite(diff)) accept = false;                     // :358-360
        else accept = lu < diff;                                      // :362-364
        // :369-383, :608-610 (+ tune :385-437, prepared above)
        const double vn = accept ? prop : v;
        th[p * 64] = vn;
        if constexpr (sync) {   // publish write-through; counted at the next step's start
          if (live)
            __hip_atomic_store(((t & 1) ? d.vb1 : d.vb0) + (size_t)p * G * C + gc, vn,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pub_p = p;
        }
        st[(NMC_ST_S * P + p) * 64] = cwv[(accept ? NMC_CW_SA : NMC_CW_SR) * 64];
        cwv[NMC_CW_PAC * 64] = accept ? 1.0 : 0.0;
        cwv[NMC_CW_PLP * 64] = accept ? lpp : lpc;
        cwv[NMC_CW_PLL * 64] = llp;
        pend_p = p;
        pend_t = t;
        // the rest of the update waits for the next step's pre-barrier slack
        if (p == 0) NMC_STAMP(t, 12);
      }
      if (p == 0) NMC_STAMP(t, 3);
      __syncthreads();      // the new value is visible to every wave
    }
    NMC_STAMP(t, 6);
    if (!ok) break;
    NMC_STAMP(t, 7);
  }

  if constexpr (sync) if (ctl && pub_p >= 0) {   // the last parameter's count
    nmc_drain_vm();
    if (lane == 0)
      __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }

  if (ctl && pend_p >= 0) apply_pending();
  // ---- epilogue: state back to HBM (control wave) ----
  if (ctl && live && ok) {
    double* vo = ((i1 - 1) & 1) ? d.vb1 : d.vb0;
    for (int p = 0; p < P; ++p) {
      const size_t ip = (size_t)p * G * C + gc;
      if (!sync) vo[ip] = th[p * 64];
      d.lp[ip] = st[(NMC_ST_LP * P + p) * 64];
      d.scale[ip] = st[(NMC_ST_S * P + p) * 64];
      d.nacc[ip] = (int)st[(NMC_ST_NA * P + p) * 64];
      d.nrej[ip] = (int)st[(NMC_ST_NR * P + p) * 64];
      d.tacc[ip] = (long long)st[(NMC_ST_TA * P + p) * 64];
    }
    d.ll[gc] = LL;
  }
  // ---- closing Gibbs update after i1-1 (group-0 workgroups write and record it) ----
  if constexpr (hl) if (ok && g == 0) {
    const int ge = i1 * P;   // tasks ge-2 (loaded at the last step; P >= 2) and ge-1 are left
    const bool pipe = P >= 2;
    const int nload = 1;   // closing: wave 1 loads
    if (pipe && w == naux) {
      const size_t hvi = (((size_t)(i1 - 1 - d.vbase) * P + (P - 2)) * C + cc) * 2;
      nmc_hyper_compute(d, cb, i1 - 1, P - 2, lds, L, true, d.vh[hvi], d.vh[hvi + 1],
                        ((ge - 2) & 1) * (G + 1));
    }
    if (nmc_wait_published(d, cb, P - 1, (unsigned)G * (unsigned)(i1 - i0), lds, L)) {
      if (w >= 1 && w <= nload) {
        const double* src = ((i1 - 1) & 1) ? d.vb1 : d.vb0;
        if (nload == 1 && (C & 1) == 0) {
          nmc_hyper_dma(d, src, P - 1, cb, 0, G, lds, L, ((ge - 1) & 1) * (G + 1));
          nmc_drain_vm();
        } else {
          nmc_hyper_load(d, src, P - 1, cc, (int)(((int64_t)G * (w - 1)) / nload),
                         (int)(((int64_t)G * w) / nload), lds, L, ((ge - 1) & 1) * (G + 1));
        }
      }
      __syncthreads();
      if (w == 1) {
        const size_t hvi = (((size_t)(i1 - 1 - d.vbase) * P + (P - 1)) * C + cc) * 2;
        nmc_hyper_compute(d, cb, i1 - 1, P - 1, lds, L, true, d.vh[hvi], d.vh[hvi + 1],
                          ((ge - 1) & 1) * (G + 1));
      }
    }
  }
  if constexpr (sync && !hl) if (ok && g == 0) {
    nmc_hyper_sdm(d, lds, L, lane);
    nmc_hyper_variates(d, cb, i1 - 1, lds, L, 0, W);
    nmc_drain_vm();
    if (nmc_wait_published(d, cb, P - 1, (unsigned)G * (unsigned)(i1 - i0), lds, L))
      nmc_hyper<NMC_SRC_SC1>(d, ((i1 - 1) & 1) ? d.vb1 : d.vb0, cb, i1 - 1, lds, L, true);
  }
}

// Group sums for arbitrary theta [P][G][C] -> out [G][C] (all W waves stream rows).
template <class Fam>
__global__ void __launch_bounds__(1024)
nmc_k_group_ll(Dev d, Fam fam, const double* __restrict__ obs, const double* theta,
               double* out) {
  extern __shared__ __attribute__((aligned(16))) double red[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[Fam::MAXP];
  nmc_load_theta(d, theta, g, cc, th);
  const typename Fam::Reg reg = fam.prepare(th);
  const int64_t r0 = d.off[g], r1 = d.off[g + 1];
  int64_t a;
  int n;
  nmc_chunk(r0, r1, w, W, &a, &n);
  double acc[Fam::NACC];
  nmc_ll_rows(fam, reg, obs + a * Fam::NFIELDS, n, acc);
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j) red[(j * W + w) * 64 + lane] = acc[j];
  __syncthreads();
  if (w != 0 || c >= d.C) return;
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j) {
    double sum = red[(j * W) * 64 + lane];
    for (int u = 1; u < W; ++u) sum += red[(j * W + u) * 64 + lane];
    acc[j] = sum;
  }
  out[(size_t)g * d.C + c] = fam.finish(reg, acc, (long)(r1 - r0));
}

// Per-observation LL at the values in `value` [P][G][C] -> out [C][n_obs].
template <class Fam>
__global__ void __launch_bounds__(64)
nmc_k_obs_ll(Dev d, Fam fam, const double* value, double* out, int64_t n_obs) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[Fam::MAXP];
  nmc_load_theta(d, value, g, cc, th);
  const typename Fam::Reg reg = fam.prepare(th);
  const int nf = Fam::NFIELDS;
  for (int64_t r = d.off[g]; r < d.off[g + 1]; ++r) {
    const double v = fam.obs_ll(reg, d.obs + r * nf);
    if (c < d.C) out[(size_t)c * n_obs + r] = v;
  }
}

