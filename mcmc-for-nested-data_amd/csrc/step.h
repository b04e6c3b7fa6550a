// step.h -- the one-barrier step kernel: nmc_k_step<Fam, MODE>, an opt-in (NMC_STEP=1)
// alternative to nmc_k_run for groups whose rows fit LDS, none/complete pooling (NOPOOL)
// and partial pooling with the register Gibbs hand-off (SYNC_REG).  Measured slower on
// MI355X (cfg 3: 8.8-11.7 against 8.0 us/iter, profiles/r03_step_kernel_ab.json), kept
// bit-identical and tested.
//
// Same work, partition and summation orders as nmc_k_run (kernels.h) -- the two are
// bit-identical and the tests compare them -- but with ONE workgroup barrier per
// parameter step instead of two.  nmc_k_run lets the control wave alone sum the tile
// partials and decide (posteriorSampling.py:334-383) while the other waves wait at a
// second barrier for the decided value; here every wave sums the partials and makes the
// identical decision from the same LDS operands, so each wave holds the chain state it
// needs (values, proposal scales, group log-likelihood) in registers and walks straight
// into the next step's likelihood tiles:
//
//   per step k = (t, p), sp = k & 1 (every LDS hand-off double-buffered by step parity):
//     Gibbs wave  task k-lag of the register hand-off (poll, fetch, pairwise update,
//                 HyperParameter.update :463-498) and, when that update is the one this
//                 step's prior needs, the step's priors -> ops[sp]
//     control     the deferred state update of step k-1 (counters, log prior, sample and
//                 trace rows, :369-383), both outcomes of the counters and of the tuned
//                 scale (:385-437) -> ops[sp], priors (:293-294) -> ops[sp], the count of
//                 the last published value, the LDS-DMA of step k+1's {z, log u}
//     every wave proposal theta_p + scale_p * z (:304-306) from its registers and
//                 likelihood tiles (:615-635) taken from an LDS counter -> part[sp]
//     ---------- barrier ----------
//     every wave the 16 tile partials in the fixed order, the group LL, the Metropolis
//                 branches in the reference's order (:347-364); values, scale and LL
//                 registers updated (:369-383, :608-610); the control wave publishes
//
// A slow wave still reading step k's operands cannot be overtaken: the next writes to
// the same parity (step k+2) come after the barrier of step k+1, which it has not
// reached.  The z slot of step k+2 is written during step k+1, after every wave has read
// step k's z and log u (at the start of step k, before the barrier of step k).
#pragma once
#include "kernels.h"

// LDS carve of nmc_k_step, in columns of 64 doubles (one per lane); the host computes
// the same (ctx.h).
struct nmc_step_layout {
  int part;   // [2][NACC][NSLOT]  tile partial sums by step parity (unused slots: -0.0)
  int st;     // [5][P]            control wave: (unused), log prior, n acc, n rej, total acc
  int cw;     // [5]               control wave: counter outcomes of the pending step
  int hyp;    // [6][P]            hyper state (NMC_HY_*), partial pooling
  int zl;     // [4][2]            {z, log u} ring by step (LDS-DMA, two steps ahead)
  int ops;    // [2][4]            decision operands by step parity (NMC_OP_*)
  int hval;   // [G + 1]           Gibbs payload: the chain block's values of one parameter
  int flag;   // [1]               wait flag, Gibbs verdict, tile counters
  int rows;   // [nmax][NF]        the group's rows, staged once per launch
  int total;
};
__host__ __device__ inline nmc_step_layout nmc_step_lds(int nacc, int P, int partial,
                                                        int row_doubles, int G) {
  nmc_step_layout L;
  L.part = 0;
  L.st = L.part + 2 * nacc * NMC_NSLOT;
  L.cw = L.st + 5 * P;
  L.hyp = L.cw + 5;
  L.zl = L.hyp + (partial ? 6 * P : 0);
  L.ops = L.zl + 8;
  L.hval = L.ops + 8;
  L.flag = L.hval + (partial ? G + 1 : 0);   // (+1: the payload DMA moves group pairs)
  L.rows = L.flag + 1;
  // (+1 column: the pipelined row loops prefetch one block past a tile's rows)
  L.total = L.rows + (row_doubles > 0 ? (row_doubles + 63) / 64 + 1 : 0);
  return L;
}
// Diagnostic build only (make stamps, never shipped; tools/steptl.py reads them):
//   [0, 512)      workgroup 0, wave w, launch step si < 8: ((w * 8 + si) * 8 + slot) shader
//                 clocks; slots 0 step start, 1 role work done, 2 tiles done, 3 past the
//                 barrier, 4 decided
//   [512, 1024)   workgroup 0, tile k of launch step si < 8: (si * 16 + k) * 4 + {start,
//                 end, wave}
//   [1024, ...)   every workgroup b: 1024 + b * 4 + {entry, prologue done, loop done, exit},
//                 s_memrealtime (100 MHz, one clock for the whole chip)
#ifdef NMC_STAMPS
#define NMC_SW(si, slot)                                                                  \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) >= 0 && (si) < 8 && (threadIdx.x & 63) == 0)  \
      d.stamps[((w) * 8 + (si)) * 8 + (slot)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
#define NMC_SL(slot)                                                                      \
  do {                                                                                    \
    if (d.stamps && threadIdx.x == 0)                                                     \
      d.stamps[1024 + (size_t)blockIdx.x * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#ifdef NMC_STAMPS_TILES   // (tile stamps too: -DNMC_STAMPS_TILES; with every stamp in the
                          // linreg instance the backend fails with an illegal VGPR->SGPR copy)
#define NMC_ST(si, k, e, wv)                                                              \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) >= 0 && (si) < 8 && (k) < 16 &&               \
        (threadIdx.x & 63) == 0) {                                                        \
      d.stamps[512 + ((si) * 16 + (k)) * 4 + (e)] = __builtin_amdgcn_s_memtime();         \
      if (e) d.stamps[512 + ((si) * 16 + (k)) * 4 + 2] = (unsigned long long)(wv);        \
    }                                                                                     \
  } while (0)
#else
#define NMC_ST(si, k, e, wv) do {} while (0)
#endif
#else
#define NMC_SW(si, slot) do {} while (0)
#define NMC_SL(slot) do {} while (0)
#define NMC_ST(si, k, e, wv) do {} while (0)
#endif

// decision operands of a step: priors of the current value and of the proposal, the
// proposal scale after an accept / a reject (tuned when due)
enum { NMC_OP_LPC = 0, NMC_OP_LPP, NMC_OP_SA, NMC_OP_SR };
enum { NMC_CWS_NAA = 0, NMC_CWS_NRA, NMC_CWS_NAR, NMC_CWS_NRR, NMC_CWS_TA };

// The likelihood tiles of one step, taken from the step's LDS counter until none is
// left; tile k's partial sums -> part[j * NSLOT + k] (this lane's column).  The next
// tile is requested before the current one is computed (the atomic's return rides
// under the tile's row reads).
template <class Fam>
__device__ __forceinline__ void nmc_step_tiles(const Dev& d, const Fam& fam,
                                               const typename Fam::Reg& reg,
                                               const typename Fam::Reg& preg,
                                               const double* lrows, const nmc_tiling& TI,
                                               unsigned* tc, double* part, int si = 0) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  (void)si;
  (void)w;
  auto grab = [&]() -> unsigned {
    unsigned k = 0;
    if (lane == 0) k = __hip_atomic_fetch_add(tc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return k;
  };
  int k = (int)__builtin_amdgcn_readlane(grab(), 0);
  while (k < TI.nt) {
    const unsigned kn = grab();
    const int ra = TI.start(k);
    const int rn = TI.len(k);
    NMC_ST(si, k, 0, w);
    double acc[Fam::NACC];
    bool done = false;
    if constexpr (nmc_paired_rows_ok<Fam>()) if (d.paired) {
      nmc_ll_rows_lds<Fam, true>(fam, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc, &preg);
      done = true;
    }
    if (!done) nmc_ll_rows_lds(fam, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc);
#pragma unroll
    for (int j = 0; j < Fam::NACC; ++j) part[(j * NMC_NSLOT + k) * 64] = acc[j];
    NMC_ST(si, k, 1, w);
    k = (int)__builtin_amdgcn_readlane(kn, 0);
  }
}

// field-wise a ? x : y of a family's per-lane registers (a struct of doubles)
template <class R>
__device__ __forceinline__ R nmc_reg_select(bool a, const R& x, const R& y) {
  static_assert(sizeof(R) % sizeof(double) == 0, "Fam::Reg: doubles only");
  R r;
  const double* px = reinterpret_cast<const double*>(&x);
  const double* py = reinterpret_cast<const double*>(&y);
  double* pr = reinterpret_cast<double*>(&r);
#pragma unroll
  for (unsigned i = 0; i < sizeof(R) / sizeof(double); ++i) pr[i] = a ? px[i] : py[i];
  return r;
}

// (768 threads: up to three waves per SIMD -- the hand-written row loops keep below v168 --
//  so two likelihood waves per SIMD issue fp64 while the third plays a role; one wave alone
//  issues an fp64 instruction at most every ~7 cycles, two every ~3.4: tools/fp64lat.hip,
//  tools/llbench7.hip)
#ifndef NMC_STEP_THREADS
#define NMC_STEP_THREADS 512
#endif
template <class Fam, int MODE>
__global__ void __launch_bounds__(NMC_STEP_THREADS)
nmc_k_step(Dev d, Fam fam, const double* __restrict__ obs, int i0, int i1, int flags) {
  static_assert(MODE == NMC_MODE_NOPOOL || MODE == NMC_MODE_SYNC_REG,
                "nmc_k_step: none/complete pooling or the register Gibbs hand-off");
  constexpr bool PARTIAL = MODE == NMC_MODE_SYNC_REG;
  constexpr int MP = Fam::MAXP;
  constexpr bool PAIRED_OK = nmc_paired_rows_ok<Fam>();
  using Reg = typename Fam::Reg;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  (void)flags;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = d.P, G = d.G, C = d.C;
  const int g = blockIdx.x % G, cb = blockIdx.x / G;
  const int c = nmc_lane_chain(d, cb, lane);
  const bool live = nmc_lane_owns(d, c, lane);
  const bool g0w = g == 0;                 // writes (and records) the chain block's hyper state
  const int cc = c < C ? c : C - 1;
  const int ngrp = (int)(d.off[g + 1] - d.off[g]);
  const nmc_tiling TI = nmc_tiles(ngrp, d.tile);
  const nmc_step_layout L = nmc_step_lds(Fam::NACC, P, PARTIAL, d.nmax * Fam::NFIELDS, G);
  const size_t PGC = (size_t)P * G * C;
  const size_t gc = (size_t)g * C + cc;
  const bool ctl = w == 0;
  const bool gw = PARTIAL && w == 1;       // the Gibbs wave (host: W >= 3, G <= 64)
  nmc_lds_layout HL;                       // (the Gibbs helpers' view: payload, hyper state)
  HL.hval = L.hval;
  HL.hyp = L.hyp;
  const int lag = P >= 2 ? 2 : 1;          // Gibbs task of step gs: gs - lag
  const bool paired = PAIRED_OK && d.paired;
  double* st = lds + L.st * 64 + lane;     // st[(k * P + p) * 64]
  double* cw = lds + L.cw * 64 + lane;
  double* hy = lds + L.hyp * 64 + lane;
  double* ops = lds + L.ops * 64 + lane;   // ops[(sp * 4 + j) * 64]
  double* zl = lds + L.zl * 64;            // {z, log u} of step gs: zl + (2 * (gs & 3)) * 64
  unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);   // tile counters by step parity
  double* lrows = lds + L.rows * 64;
  const int gs0 = i0 * P, ge = i1 * P;

  NMC_SL(0);
  // ---- prologue: registers (every wave), control state and hyper state (LDS) ----
  const double* vin = ((i0 - 1) & 1) ? d.vb1 : d.vb0;
  double th[MP], sc[MP];
#pragma unroll
  for (int q = 0; q < MP; ++q) {
    th[q] = q < P ? vin[(size_t)q * G * C + gc] : 0.0;
    sc[q] = q < P ? d.scale[(size_t)q * G * C + gc] : 0.0;
  }
  double LL = d.ll[gc];
  const double gcst = fam.gconst((long)ngrp);
  // {z, log u} of global step k -> its ring slot (k & 3), by LDS-DMA: issued two steps ahead
  // by the control wave, landed (its vmcnt drain) before the barrier of the step before
  auto put_zl = [&](int k) {
    if (k < ge)
      nmc_dma16(d.vzl + ((size_t)(k / P - d.vbase) * PGC + (size_t)(k % P) * G * C + gc) * 2,
                zl + (2 * (k & 3)) * 64);
  };
  if (ctl) {
    for (int p = 0; p < P; ++p) {
      const size_t ip = (size_t)p * G * C + gc;
      st[(NMC_ST_LP * P + p) * 64] = d.lp[ip];
      st[(NMC_ST_NA * P + p) * 64] = (double)d.nacc[ip];
      st[(NMC_ST_NR * P + p) * 64] = (double)d.nrej[ip];
      st[(NMC_ST_TA * P + p) * 64] = (double)d.tacc[ip];
      if (PARTIAL) {   // hyper-parameters after iteration i0-1 (slot (i0-1) & 1)
        const size_t ho = nmc_hslot(d, i0 - 1) + (size_t)p * C + cc;
        const double s2 = d.s2[ho];
        hy[(NMC_HY_MU * P + p) * 64] = d.mu[ho];
        hy[(NMC_HY_SD * P + p) * 64] = d.hsd[ho];
        hy[(NMC_HY_LSD * P + p) * 64] = d.hlsd[ho];
        hy[(NMC_HY_S2 * P + p) * 64] = s2;
        hy[(NMC_HY_SDM * P + p) * 64] = sqrt(s2 / G);
        hy[(NMC_HY_ISD * P + p) * 64] = 1.0 / d.hsd[ho];
      }
    }
    put_zl(gs0);
    put_zl(gs0 + 1);
    for (int s = 0; s < 2; ++s)   // x + (-0.0) == x: the fixed slot sum
      for (int j = 0; j < Fam::NACC; ++j)
        for (int k = TI.nt; k < NMC_NSLOT; ++k)
          lds[(L.part + (s * Fam::NACC + j) * NMC_NSLOT + k) * 64 + lane] = -0.0;
    lds[L.flag * 64 + lane] = 0.0;   // (also zeroes both tile counters)
    nmc_drain_vm();
  }
  {   // this group's rows -> LDS, once for the whole launch
    const double* grows = obs + d.off[g] * Fam::NFIELDS;
    const int nd = ngrp * Fam::NFIELDS;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
  }
  __syncthreads();
  NMC_SL(1);

  // the proposal of step k (Parameter.propose :304-306) and its likelihood registers:
  // th with th[p] = prop (this lane's chain, and the partner lane's for the paired rows)
  auto proposal = [&](const double (&thv)[MP], int p, double prop, Reg& reg, Reg& preg) {
    double thp[MP];
#pragma unroll
    for (int q = 0; q < MP; ++q) thp[q] = q == p ? prop : thv[q];
    reg = fam.prepare(thp);
    preg = reg;
    if constexpr (PAIRED_OK) if (paired) {
      const bool hi = lane >= 32;
#pragma unroll
      for (int q = 0; q < MP; ++q) {
        const nmc_pair2 e = nmc_halves(thp[q]);
        thp[q] = hi ? e.lo : e.hi;
      }
      preg = fam.prepare(thp);
    }
  };
  auto sel = [](const double (&a)[MP], int p) {
    double v = a[0];
#pragma unroll
    for (int q = 1; q < MP; ++q)
      if (q == p) v = a[q];
    return v;
  };
  // step gs0's proposal
  double prop, lu;
  Reg reg, preg;
  {
    const double* z0 = zl + (2 * (gs0 & 3)) * 64 + 2 * lane;
    prop = th[0] + (1.0 * sc[0]) * z0[0];
    lu = z0[1];
    proposal(th, 0, prop, reg, preg);
  }

  bool ok = true;
  int pub_p = -1;                    // control wave: published value awaiting its count
  int pend_p = -1, pend_t = 0;       // control wave: decided step whose bookkeeping waits
  bool q_acc = false;
  double q_plp = 0, q_pll = 0, q_val = 0;
  // control wave: the rest of a decided step's update (:369-383): counters, log prior,
  // sample and trace rows
  auto apply_pending = [&]() {
    const int q = pend_p, tq = pend_t;
    st[(NMC_ST_LP * P + q) * 64] = q_plp;
    st[(NMC_ST_NA * P + q) * 64] = cw[(q_acc ? NMC_CWS_NAA : NMC_CWS_NAR) * 64];
    st[(NMC_ST_NR * P + q) * 64] = cw[(q_acc ? NMC_CWS_NRA : NMC_CWS_NRR) * 64];
    st[(NMC_ST_TA * P + q) * 64] = cw[NMC_CWS_TA * 64] + (q_acc ? 1.0 : 0.0);
    if (live) {
      const int row = nmc_record_row(d, tq);
      if (row >= 0) {
        const int col = q * (G + (PARTIAL ? 2 : 0)) + (PARTIAL ? 2 : 0) + g;
        d.samples[((size_t)row * d.cols + col) * C + c] = q_val;
      }
      if (tq < d.trace_n) {
        const size_t it = (((size_t)tq * P + q) * G + g) * C + c;
        d.tflag[it] = q_acc ? 1 : 0;
        d.tllp[it] = q_pll;
      }
    }
    pend_p = -1;
  };
  // the Gibbs update of parameter kq after iteration kt (HyperParameter.update :463-498) for
  // this wave's 64 chains: the chain block's published values -> LDS payload (sc1 LDS-DMA,
  // one round trip), numpy's pairwise sums read back from LDS (nmc_hyper_compute)
  auto gibbs_task = [&](int kt, int kq, bool write) {
    const size_t hvi = (((size_t)(kt - d.vbase) * P + kq) * C + cc) * 2;
    const double hz = d.vh[hvi], hx = d.vh[hvi + 1];
    const double* src = (kt & 1) ? d.vb1 : d.vb0;
    if ((C & 1) == 0) {
      nmc_hyper_dma(d, src, kq, cb, 0, G, lds, HL, 0);
      nmc_drain_vm();
    } else {
      nmc_hyper_load(d, src, kq, cc, 0, G, lds, HL, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    nmc_hyper_compute(d, cb, kt, kq, lds, HL, write, hz, hx, 0);
  };
  auto count_published = [&]() {
    if (pub_p >= 0) {
      nmc_drain_vm();
      if (lane == 0)
        __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      pub_p = -1;
    }
  };

  for (int t = i0; t < i1 && ok; ++t) {
    const bool tune = t > 0 && t < d.burn && t % d.tune_interval == 0;
    for (int p = 0; p < P; ++p) {
      const int gs = t * P + p, sp = gs & 1;
      double* opk = ops + sp * 4 * 64;
      const bool due = PARTIAL && gs - lag >= gs0;   // the Gibbs wave's task gs - lag
      const bool post_prior = due && P <= 2;         // ... is the update this step's prior needs
      const double thp_p = sel(th, p), scp = sel(sc, p);
      const int si = gs - gs0;   // (stamps)
      NMC_SW(si, 0);

      // ---- Gibbs wave: task gs - lag = (kt, kq), and this step's priors when due ----
      if constexpr (PARTIAL) if (gw && due) {
        if (!(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);
        const int k = gs - lag, kq = k % P, kt = k / P;
        const bool r = nmc_poll_published(d, cb, kq, (unsigned)G * (unsigned)(kt - i0 + 1));
        if (lane == 0)
          __hip_atomic_store(lds + L.flag * 64 + 1 + sp, r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (r) {
          // keep the payload loads below the poll (no instruction: wavefront scope)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (d.sflags & 1) {
            gibbs_task(kt, kq, g0w);
          } else {
            double xv[64], hz, hx;
            nmc_hyper_fetch_reg(d, kt, kq, cc, xv, hz, hx);
            nmc_hyper_compute_reg(d, cb, kt, kq, lds, L.hyp, g0w, hz, hx, xv);
          }
          if (post_prior) {
            const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
            const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
            opk[NMC_OP_LPC * 64] =
                t > 0 ? nmc_norm_logpdf_r(thp_p, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
            opk[NMC_OP_LPP * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
          }
        }
        __builtin_amdgcn_s_setprio(0);
      }
      // ---- control wave: bookkeeping of step gs-1, operands of this step, z of gs+2 ----
      if (ctl) {
        if (!(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);
        if (pend_p >= 0) apply_pending();
        {
          const double na = st[(NMC_ST_NA * P + p) * 64], nr = st[(NMC_ST_NR * P + p) * 64];
          double naA = na + 1.0, nrA = nr, naR = na, nrR = nr + 1.0;
          double sA = scp, sR = scp;
          if (tune) {
            nmc_tune(sA, naA, nrA);
            nmc_tune(sR, naR, nrR);
          }
          cw[NMC_CWS_NAA * 64] = naA;
          cw[NMC_CWS_NRA * 64] = nrA;
          cw[NMC_CWS_NAR * 64] = naR;
          cw[NMC_CWS_NRR * 64] = nrR;
          cw[NMC_CWS_TA * 64] = st[(NMC_ST_TA * P + p) * 64];
          opk[NMC_OP_SA * 64] = sA;
          opk[NMC_OP_SR * 64] = sR;
        }
        if (!post_prior) {   // priors (:293-294)
          double lpc, lpp;
          if constexpr (PARTIAL) {
            const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
            const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
            lpc = t > 0 ? nmc_norm_logpdf_r(thp_p, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
            lpp = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
          } else {
            lpc = st[(NMC_ST_LP * P + p) * 64];
            lpp = nmc_prior_logpdf(d.pfam[p], d.ppar + 8 * p, prop);
          }
          opk[NMC_OP_LPC * 64] = lpc;
          opk[NMC_OP_LPP * 64] = lpp;
        }
        // the previous step's published value has had the work above to drain
        if constexpr (PARTIAL) count_published();
        put_zl(gs + 2);
        __builtin_amdgcn_s_setprio(0);
      }

      // ---- every wave: the likelihood tiles of the proposal (:615-635) ----
      NMC_SW(si, 1);
      nmc_step_tiles(d, fam, reg, preg, lrows, TI, tcnt + sp,
                     lds + (L.part + sp * Fam::NACC * NMC_NSLOT) * 64 + lane, si);
      // ---- the next step's proposal for both outcomes of this decision (P >= 2: the
      //      next parameter's value and scale are already known; its z landed before the
      //      previous barrier) ----
      const int pn = p + 1 < P ? p + 1 : 0;
      double propn = 0.0, lun = 0.0;
      Reg regA = reg, regR = reg, pregA = preg, pregR = preg;
      const bool pre = (d.sflags & 2) && P >= 2;
      if (pre && gs + 1 < ge) {
        const double* zn = zl + (2 * ((gs + 1) & 3)) * 64 + 2 * lane;
        propn = sel(th, pn) + (1.0 * sel(sc, pn)) * zn[0];
        lun = zn[1];
        double thA[MP];
#pragma unroll
        for (int q = 0; q < MP; ++q) thA[q] = q == p ? prop : th[q];
        proposal(thA, pn, propn, regA, pregA);
        proposal(th, pn, propn, regR, pregR);
      }
      if (ctl) nmc_drain_vm();   // step gs+2's {z, log u} have landed
      NMC_SW(si, 2);
      __syncthreads();
      NMC_SW(si, 3);

      // ---- every wave: group log-likelihood and the Metropolis decision (:334-383) ----
      if (ctl && lane == 0) tcnt[sp] = 0u;   // all of this step's tiles are taken; reused at +2
      double acc[Fam::NACC];
#pragma unroll
      for (int j = 0; j < Fam::NACC; ++j)
        acc[j] = nmc_sum_slots(lds + (L.part + (sp * Fam::NACC + j) * NMC_NSLOT) * 64 + lane);
      // (one verdict word per step parity, flag words 1-2: the Gibbs wave may already be
      //  writing step gs+1's verdict while a slow wave reads this one)
      const double verdict = due ? lds[L.flag * 64 + 1 + sp] : 0.0;
      const double lpc = opk[NMC_OP_LPC * 64], lpp = opk[NMC_OP_LPP * 64];
      const double sA = opk[NMC_OP_SA * 64], sR = opk[NMC_OP_SR * 64];
      const double llp = fam.finish_fast(reg, acc, (long)ngrp, gcst);
      const double postp = lpp + llp;
      const double post = lpc + LL;
      const double diff = postp - post;
      bool accept;
      if (!isfinite(post) && isfinite(postp)) accept = true;        // :347-352
      else if (!isfinite(llp)) accept = false;                      // :354-356
      else if (!isfinite(diff)) accept = false;                     // :358-360
      else accept = lu < diff;                                      // :362-364
      const double vn = accept ? prop : thp_p;
#pragma unroll
      for (int q = 0; q < MP; ++q)
        if (q == p) {
          th[q] = vn;
          sc[q] = accept ? sA : sR;
        }
      if (accept) LL = llp;                                         // :608-610
      if (ctl) {
        if constexpr (PARTIAL) {   // publish write-through; counted at the next step
          if (live)
            __hip_atomic_store(((t & 1) ? d.vb1 : d.vb0) + (size_t)p * G * C + gc, vn,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pub_p = p;
        }
        q_acc = accept;
        q_plp = accept ? lpp : lpc;
        q_pll = llp;
        q_val = vn;
        pend_p = p;
        pend_t = t;
      }
      // the next step's proposal: selected (P >= 2) or formed now (P == 1: it depends on
      // this decision's value and scale)
      if (pre) {
        prop = propn;
        lu = lun;
        reg = nmc_reg_select(accept, regA, regR);
        if constexpr (PAIRED_OK) if (paired) {   // the partner lane's (lane ^ 32) outcome
          const unsigned a = accept ? 1u : 0u;
          const auto sw = __builtin_amdgcn_permlane32_swap(a, a, false, false);
          preg = nmc_reg_select((lane >= 32 ? sw[0] : sw[1]) != 0u, pregA, pregR);
        }
      } else if (gs + 1 < ge) {
        const double* zn = zl + (2 * ((gs + 1) & 3)) * 64 + 2 * lane;
        prop = sel(th, pn) + (1.0 * sel(sc, pn)) * zn[0];
        lu = zn[1];
        proposal(th, pn, prop, reg, preg);
      }
      NMC_SW(si, 4);
      if (due) {
        ok = verdict == 2.0 * ((double)gs + 1);
        if (!ok) break;
      }
    }
  }

  NMC_SL(2);
  if (ctl) {
    if constexpr (PARTIAL) count_published();   // the last parameter's count
    if (pend_p >= 0) apply_pending();
  }
  // ---- epilogue: state back to HBM (control wave) ----
  if (ctl && live && ok) {
    double* vo = ((i1 - 1) & 1) ? d.vb1 : d.vb0;
#pragma unroll
    for (int q = 0; q < MP; ++q) {
      if (q >= P) break;
      const size_t ip = (size_t)q * G * C + gc;
      if (!PARTIAL) vo[ip] = th[q];   // (partial: published write-through)
      d.lp[ip] = st[(NMC_ST_LP * P + q) * 64];
      d.scale[ip] = sc[q];
      d.nacc[ip] = (int)st[(NMC_ST_NA * P + q) * 64];
      d.nrej[ip] = (int)st[(NMC_ST_NR * P + q) * 64];
      d.tacc[ip] = (long long)st[(NMC_ST_TA * P + q) * 64];
    }
    d.ll[gc] = LL;
  }
  // ---- closing Gibbs updates, tasks ge-lag .. ge-1 (group-0 workgroups write and record
  //      them), once every workgroup of the chain block has published its last value ----
  if constexpr (PARTIAL) if (ok && g0w) {
    if (nmc_wait_published_col(d, cb, P - 1, (unsigned)G * (unsigned)(i1 - i0), lds, L.flag) &&
        gw) {
      for (int k = ge - lag > gs0 ? ge - lag : gs0; k < ge; ++k) {
        if (d.sflags & 1) {
          gibbs_task(k / P, k % P, true);
        } else {
          double xv[64], hz, hx;
          nmc_hyper_fetch_reg(d, k / P, k % P, cc, xv, hz, hx);
          nmc_hyper_compute_reg(d, cb, k / P, k % P, lds, L.hyp, true, hz, hx, xv);
        }
      }
    }
  }
  nmc_drain_vm();
  NMC_SL(3);
}
