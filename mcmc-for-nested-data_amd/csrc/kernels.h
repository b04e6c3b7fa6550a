// kernels.h -- the MCMC iteration kernel for gfx950 (CDNA4, wave64, fp64).
//
// One launch = one reference iteration (Sampler._loop body, posteriorSampling.py:
// 872-891) for every chain.  Layout: chain-on-lane.  A workgroup owns one (chain
// block of 64 chains, group g) pair:
//   * its group's observation rows (CSR off[g]..off[g+1]) are staged ONCE into LDS
//     and reused by all P parameter steps; lanes are chains, so every row is read
//     with a wave-uniform (broadcast) LDS address and one row feeds 64 chains, and
//     the group sum needs no cross-lane reduction;
//   * partial pooling: the Gibbs update of the previous iteration's hyper-parameters
//     (HyperParameter.update, :463-498) is recomputed, deterministically and in the
//     same order, by every workgroup of the chain block at launch start -- so one
//     kernel boundary per iteration is the only global synchronisation;
//   * then for p = 0..P-1 (StepMethod.step, :594-613): waves 1..W-1 split the rows
//     and accumulate the family log-likelihood with the proposal for p and the
//     current values of the others (:615-635); wave 0 meanwhile evaluates both
//     prior log-densities; after one barrier wave 0 runs the Metropolis decision
//     for its 64 chains (:334-383, branch order exact, IEEE isfinite), tuning
//     (:385-437), group-LL propagation (:608-610) and recording (:887-889), and
//     broadcasts the new value for the next parameter's step.
// Random variates are state-independent: nmc_k_fill draws a chunk of iterations at
// once (fully parallel Philox) into HBM; replay mode fills the same buffers from
// the reference's captured variates.
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
  int* nacc;             // [P][G][C]  since last tune
  int* nrej;
  long long* tacc;       // [P][G][C]  total accepted
  double* mu;            // [P][C]
  double* s2;
  double* hsd;           // sqrt(s2)
  double* hlsd;          // log(sqrt(s2))
  double ha, hlga;       // invgamma shape a = (G-1)/2 and gammaln(a)
  int stage_rows;        // LDS rows per workgroup (max group size) or 0: stream rows
  // variates of iterations [vbase, vbase + vcap): filled by nmc_k_fill
  double* vz;            // [t][P][G][C] proposal normal
  double* vlu;           // [t][P][G][C] log of the accept uniform
  double* vhz;           // [t][P][C]    hyper mean normal
  double* vhx;           // [t][P][C]    hyper Gamma(a) draw
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
  unsigned long long* stamps;   // diagnostic build only (-DNMC_STAMPS): [block][8]
};

#ifdef NMC_STAMPS
// Diagnostic build only (never the shipped library): lane 0 of wave `wv` drains
// its outstanding memory ops and writes a 100 MHz timestamp to stamps[block][slot].
#define NMC_STAMP(wv, slot)                                                           \
  do {                                                                                \
    if ((threadIdx.x >> 6) == (wv)) {                                                 \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                     \
      if ((threadIdx.x & 63) == 0 && d.stamps)                                        \
        d.stamps[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();         \
    }                                                                                 \
  } while (0)
#else
#define NMC_STAMP(wv, slot) do {} while (0)
#endif

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
// Variates for iterations [iter0, iter0 + T): one thread per (t, p, g, c) element
// of the step variates and per (t, p, c) of the hyper variates.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) nmc_k_fill(Dev d, int iter0, int T) {
  const size_t PGC = (size_t)d.P * d.G * d.C, PC = (size_t)d.P * d.C;
  const size_t n1 = (size_t)T * PGC;
  const size_t n2 = d.pooling == NMC_POOL_PARTIAL ? (size_t)T * PC : 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n1 + n2;
       i += (size_t)gridDim.x * blockDim.x) {
    if (i < n1) {
      const int t = (int)(i / PGC);
      const size_t r = i % PGC;
      const int c = (int)(r % d.C);
      const int g = (int)((r / d.C) % d.G);
      const int p = (int)(r / ((size_t)d.C * d.G));
      const int it = iter0 + t;
      double z, lu;
      if (d.rng_mode == NMC_RNG_REPLAY) {
        const size_t k = (size_t)it * PGC + r;
        z = it < d.replay_n ? d.rz[k] : nmc_nan();
        lu = it < d.replay_n ? log(d.ru[k]) : nmc_nan();
      } else {
        const uint32_t ch = (uint32_t)(d.chain_base + c);
        z = nmc_normal(it, g, p, NMC_PURPOSE_PROPOSAL, ch, d.seed);
        lu = log(nmc_uniform2(it, g, p, NMC_PURPOSE_ACCEPT, ch, d.seed).a);
      }
      d.vz[i] = z;
      d.vlu[i] = lu;
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
      d.vhz[j] = hz;
      d.vhx[j] = hx;
    }
  }
}

// ---------------------------------------------------------------------------
// Gibbs update of every parameter's hyper-parameters at iteration hiter for one
// chain block (HyperParameter._updateMean :481-487, _updateVar :489-498, setPrior
// :273-282), cooperatively by ALL threads of the workgroup (contains barriers).
// numpy's pairwise order: the 8 accumulator chains r_j = x_j + x_{j+8} + ... of each
// parameter are summed by different waves, wave 0 combines them as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) and adds the n%8 tail -- numpy-exact for
// G <= 128 (one leaf); larger G keeps this fixed single-level order.
// LDS: hx[8P][64] chain sums, hm[P][64] means, out: hmu/hsd/hlsd [P][64].
// write: store mu/s2/sd/log sd to global and record the row of hiter.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double nmc_combine8(const double* r) {
  return ((r[0] + r[64]) + (r[128] + r[192])) + ((r[256] + r[320]) + (r[384] + r[448]));
}

// r_j = f(x_j) + f(x_{j+8}) + ... over i < n8 (sequential, numpy's accumulator j),
// f = identity or (x - m)^2; loads issued 16 at a time before the adds.
template <bool SQ>
__device__ __forceinline__ double nmc_chain_sum(const double* xp, int j, int n8, int C,
                                                double m) {
  const int cnt = n8 >> 3;
  double r = 0.0;
  for (int base = 0; base < cnt; base += 16) {
    double t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = base + u < cnt ? base + u : cnt - 1;
      t[u] = xp[(size_t)(j + 8 * k) * C];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (base + u < cnt) {
        double v = t[u];
        if (SQ) { v = v - m; v = v * v; }
        r = (base + u == 0) ? v : r + v;
      }
    }
  }
  return r;
}

__device__ __forceinline__ void nmc_wg_hyper(const Dev& d, int cb, int hiter, double* hx,
                                             double* hm, double* hmu, double* hsd,
                                             double* hlsd, bool write) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int c = cb * 64 + lane;
  const int G = d.G, C = d.C, P = d.P;
  const int cc = c < C ? c : C - 1;
  const int n8 = G >= 8 ? G - G % 8 : 0;
  const double* x = d.value + cc;
  // pass 1: chain sums of the values
  for (int q = w; q < 8 * P; q += nw) {
    const int p = q >> 3, j = q & 7;
    hx[q * 64 + lane] = n8 ? nmc_chain_sum<false>(x + (size_t)p * G * C, j, n8, C, 0.0) : 0.0;
  }
  __syncthreads();
  if (w == 0) {
    for (int p = 0; p < P; ++p) {
      const double* xp = x + (size_t)p * G * C;
      double res = n8 ? nmc_combine8(hx + p * 8 * 64 + lane) : 0.0;
      for (int i = n8; i < G; ++i) res += xp[(size_t)i * C];
      const size_t hv = ((size_t)(hiter - d.vbase) * P + p) * C + cc;
      const double sd = sqrt(d.s2[p * C + cc] / G);
      hm[p * 64 + lane] = res / G + sd * d.vhz[hv];      // mu ~ N(mean(x), sqrt(s2/G))
    }
  }
  __syncthreads();
  // pass 2: chain sums of squared deviations from the new mean
  for (int q = w; q < 8 * P; q += nw) {
    const int p = q >> 3, j = q & 7;
    const double m = hm[p * 64 + lane];
    hx[q * 64 + lane] = n8 ? nmc_chain_sum<true>(x + (size_t)p * G * C, j, n8, C, m) : 0.0;
  }
  __syncthreads();
  if (w == 0) {
    const int row = write ? nmc_record_row(d, hiter) : -1;
    for (int p = 0; p < P; ++p) {
      const double* xp = x + (size_t)p * G * C;
      const double m = hm[p * 64 + lane];
      double ss = n8 ? nmc_combine8(hx + p * 8 * 64 + lane) : 0.0;
      for (int i = n8; i < G; ++i) {
        const double t = xp[(size_t)i * C] - m;
        ss += t * t;
      }
      const double hat = ss / (double)(G - 1);
      const double scale = d.ha * hat;
      const size_t hv = ((size_t)(hiter - d.vbase) * P + p) * C + cc;
      // scipy invgamma.rvs: (1/gammainccinv(a, U)) * scale + loc; loc when scale == 0
      const double s2n = scale == 0.0 ? 0.0 : (1.0 / d.vhx[hv]) * scale;
      const double sdn = sqrt(s2n);
      const double lsd = log(sdn);
      hmu[p * 64 + lane] = m;
      hsd[p * 64 + lane] = sdn;
      hlsd[p * 64 + lane] = lsd;
      if (write && c < C) {
        d.mu[p * C + c] = m;
        d.s2[p * C + c] = s2n;
        d.hsd[p * C + c] = sdn;
        d.hlsd[p * C + c] = lsd;
        if (row >= 0) {
          double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
          out[0] = m;
          out[C] = s2n;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// log-likelihood of one group over one wave's row chunk, chain-on-lane.
// n rows from p (wave-uniform address: LDS broadcast reads, or scalar loads when
// streaming from global); R rows (~16 doubles) per iteration, four accumulator
// sets to break the dependence chain.
// ---------------------------------------------------------------------------
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
  if (nb > 0) {
    // two register blocks: block b+1 is requested before block b is consumed
    double cur[R * NF];
#pragma unroll
    for (int j = 0; j < R * NF; ++j) cur[j] = p[j];
    for (int b = 0; b < nb; ++b) {
      const int bn = b + 1 < nb ? b + 1 : b;
      const double* q = p + (size_t)bn * (R * NF);
      double nxt[R * NF];
#pragma unroll
      for (int j = 0; j < R * NF; ++j) nxt[j] = q[j];
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

// theta[q] = src[q][g][c] for q < P (p >= 0: parameter p replaced by prop).
template <int MP>
__device__ __forceinline__ void nmc_load_theta(const Dev& d, const double* src, int g, int c,
                                               int p, double prop, double (&th)[MP]) {
#pragma unroll
  for (int q = 0; q < MP; ++q) {
    th[q] = 0.0;
    if (q < d.P) th[q] = q == p ? prop : src[((size_t)q * d.G + g) * d.C + c];
  }
}

// th[p] (runtime p) without dynamic register indexing
template <int MP>
__device__ __forceinline__ double nmc_get(const double (&th)[MP], int p) {
  double v = th[0];
#pragma unroll
  for (int q = 1; q < MP; ++q)
    if (q == p) v = th[q];
  return v;
}
template <int MP>
__device__ __forceinline__ void nmc_set(double (&th)[MP], int p, double v) {
#pragma unroll
  for (int q = 0; q < MP; ++q)
    if (q == p) th[q] = v;
}

// LDS carve (doubles) of the iteration kernel; host computes the same size.
struct nmc_lds_layout {
  int rows, part, bc, st, hx, hm, total;
};
__host__ __device__ inline nmc_lds_layout nmc_lds(int stage_rows, int nf, int W, int nacc,
                                                  int P) {
  nmc_lds_layout L;
  const int nll = W > 1 ? W - 1 : 1;
  L.rows = 0;
  L.part = ((stage_rows * nf + 1) / 2) * 2;                  // keep 16-byte alignment
  L.bc = L.part + nll * nacc * 64;
  L.st = L.bc + 64;
  L.hx = L.st + 10 * P * 64;                                 // 10 per-parameter columns
  L.hm = L.hx + 8 * P * 64;
  L.total = L.hm + P * 64;
  return L;
}
// per-parameter state columns in st: [k][p][64]
enum { NMC_ST_S = 0, NMC_ST_Z, NMC_ST_LU, NMC_ST_LP, NMC_ST_NA, NMC_ST_NR, NMC_ST_TA,
       NMC_ST_MU, NMC_ST_SD, NMC_ST_LSD };

// ---------------------------------------------------------------------------
// K_iter: one full iteration for every (chain, group); grid = CB*G workgroups of
// 64*W threads; dynamic LDS = nmc_lds(...).total doubles.
// ---------------------------------------------------------------------------
// Values are double-buffered: every workgroup reads iteration iter-1's values from
// vsrc (its own for the proposals, the whole chain block's for the redundant Gibbs
// update) and writes its new values to vdst, so no workgroup can observe another's
// update of the same launch.
// At most 8 waves (512 threads): the register budget is 256 VGPRs, enough for the
// double-buffered row blocks without spills (1-2 workgroups per CU).
template <class Fam, bool STAGE>
__global__ void __launch_bounds__(512)
nmc_k_iter(Dev d, Fam fam, const double* __restrict__ obs, const double* __restrict__ vsrc,
           double* __restrict__ vdst, int iter) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  d.value = const_cast<double*>(vsrc);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = d.W, P = d.P, G = d.G, C = d.C;
  const int b = blockIdx.x;
  const int g = b % G, cb = b / G;
  const int c = cb * 64 + lane;
  const bool live = c < C;
  const int cc = live ? c : C - 1;
  const nmc_lds_layout L = nmc_lds(d.stage_rows, Fam::NFIELDS, W, Fam::NACC, P);
  double* rows = lds + L.rows;
  double* part = lds + L.part;
  double* bc = lds + L.bc;
  double* st = lds + L.st;
  auto ST = [&](int k, int p) -> double& { return st[(k * P + p) * 64 + lane]; };
  const int64_t r0 = d.off[g], r1 = d.off[g + 1];
  const int nrow = (int)(r1 - r0);
  const bool partial = d.pooling == NMC_POOL_PARTIAL;
  NMC_STAMP(0, 0);
  NMC_STAMP(1, 4);

  // ---- prologue: every global load of the launch issued before it is consumed ----
  // rows -> LDS by all threads (8 loads in flight per thread per round), the
  // per-parameter state -> LDS with parameter p loaded by wave p % W.
  if (STAGE) {
    const double* src = obs + r0 * Fam::NFIELDS;
    const int nd = nrow * Fam::NFIELDS;
    const int bd = blockDim.x;
    for (int base = 0; base < nd; base += 8 * bd) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * bd + (int)threadIdx.x;
        t[u] = src[i < nd ? i : nd - 1];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * bd + (int)threadIdx.x;
        if (i < nd) rows[i] = t[u];
      }
    }
  }
  double th[Fam::MAXP];
  nmc_load_theta(d, d.value, g, cc, -1, 0.0, th);       // current values, every wave
  {
    const size_t tv = (size_t)(iter - d.vbase) * P * G * C;
    const bool hyp0 = partial && iter == d.vbase;
    for (int p = w; p < P; p += W) {
      const size_t ip = ((size_t)p * G + g) * C + cc;
      const double s = d.scale[ip], z = d.vz[tv + ip], lu = d.vlu[tv + ip], lp = d.lp[ip];
      const int na = d.nacc[ip], nr = d.nrej[ip];
      const long long ta = d.tacc[ip];
      double m = 0.0, sd = 0.0, lsd = 0.0;
      if (hyp0) {
        m = d.mu[p * C + cc];
        sd = d.hsd[p * C + cc];
        lsd = d.hlsd[p * C + cc];
      }
      ST(NMC_ST_S, p) = s;
      ST(NMC_ST_Z, p) = z;
      ST(NMC_ST_LU, p) = lu;
      ST(NMC_ST_LP, p) = lp;
      ST(NMC_ST_NA, p) = (double)na;
      ST(NMC_ST_NR, p) = (double)nr;
      ST(NMC_ST_TA, p) = (double)ta;
      if (hyp0) {
        ST(NMC_ST_MU, p) = m;
        ST(NMC_ST_SD, p) = sd;
        ST(NMC_ST_LSD, p) = lsd;
      }
    }
  }
  double LL = w == 0 ? d.ll[(size_t)g * C + cc] : 0.0;
  // ---- Gibbs update of iteration iter-1, redundantly per workgroup -----------------
  if (partial && iter > d.vbase)
    nmc_wg_hyper(d, cb, iter - 1, lds + L.hx, lds + L.hm, &st[(NMC_ST_MU * P) * 64],
                 &st[(NMC_ST_SD * P) * 64], &st[(NMC_ST_LSD * P) * 64], g == 0);
  __syncthreads();
  NMC_STAMP(0, 1);

  const int nll = W > 1 ? W - 1 : 1;
  const int k = W > 1 ? w - 1 : 0;
  int64_t ca;
  int cn;
  nmc_chunk(0, nrow, k, nll, &ca, &cn);
  const double* mine = STAGE ? rows + ca * Fam::NFIELDS : obs + (r0 + ca) * Fam::NFIELDS;
  const int row_rec = nmc_record_row(d, iter);

  for (int p = 0; p < P; ++p) {
    // proposal (Parameter.propose :304-306): value + (proposalSd=1 * scale) * z
    const double v = nmc_get(th, p);
    const double s = st[(NMC_ST_S * P + p) * 64 + lane];
    const double prop = v + (1.0 * s) * st[(NMC_ST_Z * P + p) * 64 + lane];
    double acc[Fam::NACC];
#pragma unroll
    for (int j = 0; j < Fam::NACC; ++j) acc[j] = 0.0;
    double thp[Fam::MAXP];
#pragma unroll
    for (int q = 0; q < Fam::MAXP; ++q) thp[q] = th[q];
    nmc_set(thp, p, prop);
    const typename Fam::Reg reg = fam.prepare(thp);
    if (W == 1 || w > 0) {
      nmc_ll_chunk(fam, reg, mine, cn, acc);
      if (W > 1) {
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j) part[(j * nll + k) * 64 + lane] = acc[j];
      }
    }
    double lpc = 0.0, lpp = 0.0;
    if (w == 0) {
      if (partial) {
        const double m = ST(NMC_ST_MU, p), sd = ST(NMC_ST_SD, p), lsd = ST(NMC_ST_LSD, p);
        lpc = iter > 0 ? nmc_norm_logpdf(v, m, sd, lsd) : ST(NMC_ST_LP, p);  // setPrior :281
        lpp = nmc_norm_logpdf(prop, m, sd, lsd);
      } else {
        lpc = ST(NMC_ST_LP, p);
        lpp = nmc_prior_logpdf(d.pfam[p], d.ppar + 8 * p, prop);
      }
    }
    if (p == 0) NMC_STAMP(1, 7);
    if (W > 1) __syncthreads();
    if (p == 0) NMC_STAMP(0, 4);
    if (w == 0) {
      if (W > 1) {
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j) {
          double sum = part[(j * nll) * 64 + lane];
          for (int u = 1; u < nll; ++u) sum += part[(j * nll + u) * 64 + lane];
          acc[j] = sum;
        }
      }
      const double llp = fam.finish(reg, acc, (long)nrow);
      // ---- Metropolis decision, one chain per lane (:334-367) ----
      const double postp = lpp + llp;
      const double post = lpc + LL;
      const double diff = postp - post;
      bool accept;
      if (!isfinite(post) && isfinite(postp)) accept = true;        // :347-352
      else if (!isfinite(llp)) accept = false;                      // :354-356
      else if (!isfinite(diff)) accept = false;                     // :358-360
      else accept = ST(NMC_ST_LU, p) < diff;                        // :362-364
      double na = ST(NMC_ST_NA, p), nr = ST(NMC_ST_NR, p), sn = s;
      double vn = v;
      if (accept) {                                                 // :369-378, :608-610
        vn = prop;
        ST(NMC_ST_LP, p) = lpp;
        LL = llp;
        na += 1.0;
        ST(NMC_ST_TA, p) += 1.0;
      } else {                                                      // :380-383
        ST(NMC_ST_LP, p) = lpc;
        nr += 1.0;
      }
      if (iter > 0 && iter < d.burn && iter % d.tune_interval == 0) nmc_tune(sn, na, nr);
      ST(NMC_ST_NA, p) = na;
      ST(NMC_ST_NR, p) = nr;
      ST(NMC_ST_S, p) = sn;
      bc[lane] = vn;
      if (live) {
        if (row_rec >= 0) {
          const int col = p * (G + (partial ? 2 : 0)) + (partial ? 2 : 0) + g;
          d.samples[((size_t)row_rec * d.cols + col) * C + c] = vn;
        }
        if (iter < d.trace_n) {
          const size_t it = (((size_t)iter * P + p) * G + g) * C + c;
          d.tflag[it] = accept ? 1 : 0;
          d.tllp[it] = llp;
        }
      }
    }
    // every wave reads bc before its next partial store; wave 0 rewrites bc only
    // after the next step's first barrier, so two barriers per step suffice.
    if (p == 0) NMC_STAMP(0, 5);
    if (W > 1) __syncthreads();
    if (p == 0) NMC_STAMP(0, 6);
    nmc_set(th, p, bc[lane]);
  }
  NMC_STAMP(0, 2);
  // ---- epilogue: state back to HBM (wave 0) ----
  if (w == 0 && live) {
    for (int p = 0; p < P; ++p) {
      const size_t ip = ((size_t)p * G + g) * C + c;
      vdst[ip] = nmc_get(th, p);
      d.lp[ip] = ST(NMC_ST_LP, p);
      d.scale[ip] = ST(NMC_ST_S, p);
      d.nacc[ip] = (int)ST(NMC_ST_NA, p);
      d.nrej[ip] = (int)ST(NMC_ST_NR, p);
      d.tacc[ip] = (long long)ST(NMC_ST_TA, p);
    }
    d.ll[(size_t)g * C + c] = LL;
  }
  NMC_STAMP(0, 3);
}

// Gibbs update alone, for the last iteration of each chunk (grid = CB workgroups).
__global__ void __launch_bounds__(1024) nmc_k_hyper(Dev d, int hiter) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int P = d.P;
  nmc_wg_hyper(d, blockIdx.x, hiter, lds, lds + 8 * P * 64, lds + 9 * P * 64,
               lds + 10 * P * 64, lds + 11 * P * 64, true);
}

// Group sums for arbitrary theta [P][G][C] -> out [G][C] (all W waves stream rows).
template <class Fam>
__global__ void __launch_bounds__(1024)
nmc_k_group_ll(Dev d, Fam fam, const double* __restrict__ obs, const double* theta,
               double* out) {
  extern __shared__ __attribute__((aligned(16))) double red[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[Fam::MAXP];
  nmc_load_theta(d, theta, g, cc, -1, 0.0, th);
  const typename Fam::Reg reg = fam.prepare(th);
  const int64_t r0 = d.off[g], r1 = d.off[g + 1];
  int64_t a;
  int n;
  nmc_chunk(r0, r1, w, d.W, &a, &n);
  double acc[Fam::NACC];
  nmc_ll_chunk(fam, reg, obs + a * Fam::NFIELDS, n, acc);
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j) red[(j * d.W + w) * 64 + lane] = acc[j];
  __syncthreads();
  if (w != 0 || c >= d.C) return;
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j) {
    double sum = red[(j * d.W) * 64 + lane];
    for (int u = 1; u < d.W; ++u) sum += red[(j * d.W + u) * 64 + lane];
    acc[j] = sum;
  }
  out[(size_t)g * d.C + c] = fam.finish(reg, acc, (long)(r1 - r0));
}

// Per-observation LL at the current state -> out [C][n_obs].
template <class Fam>
__global__ void __launch_bounds__(64) nmc_k_obs_ll(Dev d, Fam fam, double* out, int64_t n_obs) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x % d.G, cb = blockIdx.x / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[Fam::MAXP];
  nmc_load_theta(d, d.value, g, cc, -1, 0.0, th);
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
