// sweep.h -- nmc_k_sweep<Fam, MODE>: the step kernel for groups whose rows fit LDS and need
// no row split, in three waves per SIMD.
//
// Same work, tile partition, summation orders, variates and outputs as nmc_k_run
// (kernels.h) -- the two are bit-identical and the tests compare them -- built around what
// MI355X measurements say bounds the loop (profiles/r04_fp64issue.jsonl): one wave issues an
// fp64 VALU instruction at most every ~5.8 cycles, two waves on a SIMD every ~4.7, three
// every ~4.5 (the paired row loop with its LDS reads: 7.0 / 5.3 / 4.9).  nmc_k_run's eight
// waves leave the SIMDs of its control and Gibbs waves with one likelihood wave for most
// of a step; here 12 waves (768 threads, <= 168 VGPRs) keep two or three likelihood waves
// on every SIMD while the roles run.  The kernel holds few values across its persistent
// loop: Dev is read through a pointer laundered at the top of every step (nmc_kdev), and
// each role's values live in its own branch (the Gibbs wave's 64-value payload never shares
// registers with the row loop).  The variates come from nmc_k_fill's ring (the control wave
// LDS-DMAs each next step's {z, log u}; the Gibbs wave reads its task's pair), or, with
// Dev.zin, are drawn inside the kernel (the fill's own functions, so the same bits):
//   * {z, log u} of step (t, p) (Parameter.propose :304-306, the accept uniform :362):
//     entries 0-2 of the previous step's tile queue (radius, cosine, log u);
//   * {hyper z, Gamma((G-1)/2)} of a Gibbs task (HyperParameter.update :481-498): drawn by
//     the Gibbs wave for its own task.
//
// MODE (kernels.h NMC_MODE_*):
//   NOPOOL    none / complete pooling, 64 chains per workgroup
//   HALF      none / complete pooling, 32 chains per workgroup (lanes l, l + 32: one chain)
//   SYNC_REG  partial pooling, G <= 64: the Gibbs wave fetches a task's G published values
//             into registers (one sc1 round trip) -- nmc_k_run's register hand-off
//   SYNC_LDS  partial pooling, 64 < G <= 128 (one numpy leaf): the same hand-off with the
//             payload moved to LDS by LDS-DMA, updated from there (nmc_hyper_compute)
//   SYNC_OWN  partial pooling, G > 128 (up to four numpy leaves): RB * P extra workgroups in
//             the grid, one per (chain block, parameter), compute each Gibbs task ONCE for the
//             chain block (every wave streaming its numpy streams' values with sc1 loads, all
//             in flight; nmc_hyper) and publish the four hyper values write-through with a
//             ready count; each likelihood workgroup's Gibbs wave only polls that count and
//             reads the four values (nmc_hyper_read) -- instead of every one of the G
//             workgroups streaming the chain block's G values itself
// Wave roles per step k = (t, p):
//   wave 0   control: the deferred state update of step k-1, the decision's operands (both
//            counter outcomes, tuned scales, priors), the count of the last published value;
//            then likelihood tiles; after barrier A the slot sum, finish and the Metropolis
//            decision (:334-383), published write-through (partial pooling)
//   wave 1   (partial) Gibbs: task k - lag (poll, fetch, pairwise update, this step's priors
//            when they need it), then barrier A / B with the others
//   others   likelihood tiles from the step's LDS queue (entry 0: the next step's variates)
#pragma once
#include "kernels.h"

#ifndef NMC_SWEEP_THREADS
#define NMC_SWEEP_THREADS 768
#endif

// LDS carve of nmc_k_sweep, in columns of 64 doubles (one per lane); the host computes the
// same (ctx.h).
struct nmc_sweep_layout {
  int th;     // [P]            current values
  int part;   // [NACC][NSLOT]  tile partial sums (unused slots: -0.0)
  int st;     // [5][P]         scale, log prior, n acc, n rej, total acc (NMC_ST_*)
  int hyp;    // [6][P]         hyper state (NMC_HY_*), partial pooling
  int hval;   // [G + 1]        SYNC_LDS: the Gibbs payload (+1: the DMA moves group pairs)
  int zl;     // [2][2]         {z, log u} of this and the next step (step parity)
  int zm;     // [2]            the proposal normal's second factor by step parity: z is
              //                zl's z times zm (1.0 with the fill's ring; with Dev.zin the
              //                Box-Muller radius and cosine are two queue jobs)
  int cw;     // [8]            control values across the barriers (NMC_CW_*)
  int flag;   // [1]            column 0: word 0 wait flag, words 1-2 Gibbs verdict by step
              //                parity, uint32 words 8-9 the tile queues by step parity,
              //                uint32 words 32.. the step constants (NMC_SWK_AT)
  int rows;   // [nrows][NF]    the group's rows, staged once per launch
  int total;  // columns
};
__host__ __device__ inline nmc_sweep_layout nmc_sweep_lds(int nacc, int P, int partial,
                                                          int hlds, int G, int row_doubles) {
  nmc_sweep_layout L;
  L.flag = 0;   // (first: its step constants, NMC_SWK_*, sit at a fixed address)
  L.th = 1;
  L.part = L.th + P;
  L.st = L.part + nacc * NMC_NSLOT;
  L.hyp = L.st + 5 * P;
  L.hval = L.hyp + (partial ? 6 * P : 0);
  L.zl = L.hval + (partial && hlds ? G + 1 : 0);
  L.zm = L.zl + 4;
  L.cw = L.zm + 2;
  L.rows = L.cw + 8;
  // (+1 column: the pipelined likelihood loop prefetches one block past a wave's rows)
  L.total = L.rows + (row_doubles > 0 ? (row_doubles + 63) / 64 + 1 : 0);
  return L;
}

// Out-of-line helpers: the variate draws and the none/complete-pooling priors run once per
// step on one wave; kept out of the step loop's body so their many polynomial constants are
// materialized where they are used rather than hoisted into registers for the whole launch.
// The step constants: ints at word NMC_SWK_AT of LDS column 0 (the flag column), written
// once by the prologue (after the column is zeroed) -- the problem
// sizes, the group's row count and tiling and the carve's offsets -- so a step derives its
// view with a few broadcast LDS reads at a fixed address (no kernel-argument or global load
// on the step's critical path)
enum { NMC_SWK_P = 0, NMC_SWK_G, NMC_SWK_C, NMC_SWK_NGRP, NMC_SWK_N, NMC_SWK_NT, NMC_SWK_H,
       NMC_SWK_A, NMC_SWK_B, NMC_SWK_TH, NMC_SWK_PART, NMC_SWK_ST, NMC_SWK_HYP, NMC_SWK_HVAL,
       NMC_SWK_ZL, NMC_SWK_ZM, NMC_SWK_CW, NMC_SWK_FLAG, NMC_SWK_ROWS, NMC_SWK_TOTAL,
       NMC_SWK_COUNT = 20, NMC_SWK_AT = 32 };

// Part j of the variates of step (it, p) of group g, chain c, nmc_step_variate's values
// split three ways so three waves draw them side by side (each ~1/3 of the ~460 VALU
// instructions): j = 0 the Box-Muller radius sqrt(-2 log(1 - ua)), j = 1 its cosine
// cos(2 pi ub) -- the normal is their product, rounded exactly as nmc_box_muller rounds it --
// and j = 2 log u of the accept uniform.  Replay: the reference's z, 1.0 and log u.
__device__ __noinline__ double nmc_sweep_variate_part(const double* rz, const double* ru,
                                                      int replay_n, int rng_mode, int P, int G,
                                                      int C, uint32_t ch, uint32_t seed, int it,
                                                      int p, int g, int c, int j) {
  if (rng_mode == NMC_RNG_MODE_REPLAY) {
    const size_t k = (((size_t)it * P + p) * G + g) * C + c;
    if (j == 1) return 1.0;
    if (!(it < replay_n)) return nmc_nan();
    return j == 0 ? rz[k] : log(ru[k]);
  }
  const nmc_d2 u = nmc_uniform2(it, g, p, j == 2 ? NMC_PURPOSE_ACCEPT : NMC_PURPOSE_PROPOSAL,
                                ch, seed);
  if (j == 0) return sqrt(-2.0 * nmc_log_unit(1.0 - u.a));
  if (j == 1) return nmc_cos2pi(u.b);
  return nmc_log_unit(u.a);
}
// {hyper z, Gamma(a) draw} of the Gibbs update of parameter q after iteration t for chain c
// (nmc_k_fill's values: Philox normal and Marsaglia-Tsang, or the replayed reference draws
// through scipy's inverse-CDF path).
__device__ __noinline__ nmc_d2 nmc_sweep_hyper_variate(const double* rhz, const double* rhu,
                                                       int replay_n, int rng_mode, int P, int C,
                                                       uint32_t ch, uint32_t seed, double ha,
                                                       double hlga, int t, int q, int c) {
  nmc_d2 r;
  if (rng_mode == NMC_RNG_MODE_REPLAY) {
    const size_t k = ((size_t)t * P + q) * C + c;
    r.a = t < replay_n ? rhz[k] : nmc_nan();
    r.b = t < replay_n ? nmc_igamci(ha, rhu[k], hlga) : nmc_nan();
  } else {
    r.a = nmc_normal(t, 0, q, NMC_PURPOSE_HYPER_NORMAL, ch, seed);
    r.b = nmc_gamma_mt(ha, t, q, ch, seed);
  }
  return r;
}
__device__ __noinline__ double nmc_sweep_prior(int fam, const double* prm, double x) {
  return nmc_prior_logpdf(fam, prm, x);
}

// The kernel's only argument (one struct, so the kernarg segment holds it at offset 0 and
// every field is read through the laundered pointer of nmc_sweep_args_at).
template <class Fam>
struct nmc_sweep_args {
  Dev d;
  Fam fam;
  int i0, i1;
};
template <class Fam>
__device__ __forceinline__ const nmc_sweep_args<Fam>* nmc_sweep_args_at() {
  typedef __attribute__((address_space(4))) const nmc_sweep_args<Fam>* kp;
  kp q = (kp)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return (const nmc_sweep_args<Fam>*)q;
}

// HyperParameter.update (:463-498) of parameter q for one chain block, as nmc_hyper<SC1, NS,
// true> (the same streams, sums and order, so the same bits) but loading the G values once:
// each wave keeps its NS streams' values in registers for the second pass (sum of squares
// about the new mean) instead of fetching them again -- one device-scope round trip per
// task instead of two.  The tail stream's raw values wait in LDS (pass 1 writes them).
template <int NS>
__device__ __forceinline__ void nmc_hyper_once(const Dev& d, const double* src, int cb, int t,
                                               double* lds, const nmc_lds_layout& L, int q) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C, nl = d.nleaf, ncol = 8 + d.ntail;
  const int per = 8 + (d.ntail ? 1 : 0);
  const int c = nmc_lane_chain(d, cb, lane);
  const int cc = c < C ? c : C - 1;
  const int sbeg = q * nl * per, nst = (q + 1) * nl * per;
  struct Strm {
    int j, pl, m, m8;
    const double* xp;
  };
  auto strm = [&](int s) {
    Strm r;
    r.j = s % per;
    r.pl = s / per;
    const int lf = r.pl % nl;
    const int a = nl == 1 ? 0 : d.leaf[lf];
    r.m = nl == 1 ? G : d.leaf[lf + 1] - a;
    r.m8 = r.m >= 8 ? r.m - r.m % 8 : 0;
    r.xp = src + ((size_t)q * G + a) * C + cc;
    return r;
  };
  // one round: this wave's streams w, w + W, ..., w + (NS-1) W of [sbeg, nst)
  static_assert(NS >= 1, "streams per wave");
  double v[NS][16];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int s = sbeg + w + k * W;
    const Strm r = strm(s < nst ? s : sbeg);
    const int cnt = s < nst && r.j < 8 ? r.m8 >> 3 : 0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[k][u] = u < cnt ? nmc_ldv<NMC_SRC_SC1>(r.xp + (size_t)(r.j + 8 * u) * C) : 0.0;
  }
  auto pass = [&](bool sq) {
    const double mu = sq ? lds[(L.hyp + NMC_HY_MU * P + q) * 64 + lane] : 0.0;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int s = sbeg + w + k * W;
      if (s >= nst) continue;
      const Strm r = strm(s);
      double* out = lds + (size_t)(L.hst + r.pl * ncol) * 64 + lane;
      if (r.j < 8) {
        const int cnt = r.m8 >> 3;
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (u < cnt) {
            double x = v[k][u];
            if (sq) {
              x = x - mu;
              x = x * x;
            }
            acc = u == 0 ? x : acc + x;
          }
        }
        out[r.j * 64] = acc;
      } else {   // the tail: raw values in pass 1, their squares about mu in pass 2
        for (int u = r.m8; u < r.m; ++u) {
          double x = sq ? out[(8 + u - r.m8) * 64] : nmc_ldv<NMC_SRC_SC1>(r.xp + (size_t)u * C);
          if (sq) {
            x = x - mu;
            x = x * x;
          }
          out[(8 + u - r.m8) * 64] = x;
        }
      }
    }
  };
  // (a wave holds NS streams: the whole parameter's streams in one round)
  pass(false);
  __syncthreads();
  if (w == 0) {
    const double tot = nmc_hyper_combine(d, lds, L, q, lane);
    const double sdm = lds[(L.hyp + NMC_HY_SDM * P + q) * 64 + lane];
    const double hz = lds[L.hv * 64 + (q * 64 + lane) * 2];
    lds[(L.hyp + NMC_HY_MU * P + q) * 64 + lane] = tot / G + sdm * hz;   // mu ~ N(mean, s2/G)
  }
  __syncthreads();
  pass(true);
  __syncthreads();
  if (w == 0) {
    const bool own = nmc_lane_owns(d, c, lane);
    const int row = nmc_record_row(d, t);
    const double ss = nmc_hyper_combine(d, lds, L, q, lane);
    const double hat = ss / (double)(G - 1);
    const double scale = d.ha * hat;
    const double hx = lds[L.hv * 64 + (q * 64 + lane) * 2 + 1];
    // scipy invgamma.rvs: (1/gammainccinv(a, U)) * scale + loc; loc when scale == 0
    const double s2n = scale == 0.0 ? 0.0 : (1.0 / hx) * scale;
    const double sdn = sqrt(s2n);
    const double lsd = log(sdn);
    const double m = lds[(L.hyp + NMC_HY_MU * P + q) * 64 + lane];
    lds[(L.hyp + NMC_HY_SD * P + q) * 64 + lane] = sdn;
    lds[(L.hyp + NMC_HY_LSD * P + q) * 64 + lane] = lsd;
    lds[(L.hyp + NMC_HY_S2 * P + q) * 64 + lane] = s2n;
    lds[(L.hyp + NMC_HY_ISD * P + q) * 64 + lane] = 1.0 / sdn;
    if (own) {
      const size_t ho = nmc_hslot(d, t) + (size_t)q * C + c;
      __hip_atomic_store(d.mu + ho, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.s2 + ho, s2n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.hsd + ho, sdn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.hlsd + ho, lsd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (row >= 0) {
        double* out = d.samples + ((size_t)row * d.cols + (size_t)q * (G + 2)) * C + c;
        out[0] = m;
        out[C] = s2n;
      }
    }
  }
}

// ---- Dev.gsep without co-scheduling ----
// The two kernels of the gsep path each wait on counters only the other advances, and HIP
// does not promise that kernels on two streams run at the same time (a profiler's PMC pass,
// AMD_SERIALIZE_KERNEL or a shared hardware queue serialize them).  So each chain block of a
// launch has a role word (Dev.grole, epoch = Dev.gep): a Gibbs workgroup marks itself
// started once its first task's values are published; if no Gibbs workgroup of the chain
// block has started within Dev.gpat ticks, whichever side notices first sets the fallback
// bit.  Then the Gibbs workgroups leave, and the likelihood workgroups' Gibbs waves update
// every task of the launch themselves (nmc_hyper_update_stream: the same sums, draws and
// outputs, so the same bits), group 0's writing and counting them as the Gibbs workgroup
// would.  Either every task of a (launch, chain block) comes from the Gibbs kernel or every
// one from the fallback: the bit is only set while no Gibbs workgroup has started.
__device__ __forceinline__ unsigned long long* nmc_grole(const Dev& d, int cb) {
  return d.grole + (size_t)cb * 16;
}
__device__ __forceinline__ bool nmc_grole_is_fallback(const Dev& d, unsigned long long v) {
  return (unsigned)(v >> 32) == d.gep && (v & 1ull);
}
// (one lane) set the fallback bit of this launch; false: a Gibbs workgroup has started
__device__ __forceinline__ bool nmc_grole_fallback(const Dev& d, int cb) {
  unsigned long long* r = nmc_grole(d, cb);
  const unsigned long long ep = (unsigned long long)d.gep << 32;
  unsigned long long v = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if ((unsigned)(v >> 32) == d.gep) {
      if (v & 1ull) return true;
      if (v != ep) return false;   // started
    }
    if (__hip_atomic_compare_exchange_strong(r, &v, ep | 1ull, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      __hip_atomic_fetch_add(d.gfb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
  }
}
// (one lane) a Gibbs workgroup starts its first task; false: the fallback is set, leave
__device__ __forceinline__ bool nmc_grole_start(const Dev& d, int cb) {
  unsigned long long* r = nmc_grole(d, cb);
  const unsigned long long ep = (unsigned long long)d.gep << 32;
  unsigned long long v = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    unsigned long long nv = ep + 2ull;
    if ((unsigned)(v >> 32) == d.gep) {
      if (v & 1ull) return false;
      nv = v + 2ull;
    }
    if (__hip_atomic_compare_exchange_strong(r, &v, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return true;
  }
}
// The calling wave's patience clock (s_memrealtime: 100 MHz, one clock for the chip).
__device__ __forceinline__ bool nmc_grole_patience_over(const Dev& d, unsigned long long t0) {
  return __builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)d.gpat;
}
// A Gibbs workgroup's wait for its FIRST task's publications (wave 0; wave-uniform result):
// 1 go on (started), 0 leave (the fallback is set, or a timeout recorded in d.tmo).
__device__ __forceinline__ int nmc_grole_first_wait(const Dev& d, int cb, int q, unsigned target) {
  const int lane = threadIdx.x & 63;
  target += (unsigned)d.G * d.pbase;
  unsigned* ctr = nmc_counter(d, cb, q, lane & 7);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool patient = true;
  for (unsigned spins = 0;; ++spins) {
    const unsigned v =
        lane < 8 ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += __builtin_amdgcn_readlane(v, k);
    if (tot >= target) {
      const bool go = lane == 0 ? nmc_grole_start(d, cb) : false;
      return __builtin_amdgcn_readlane((int)go, 0);
    }
    if ((spins & 63) == 63) {
      const unsigned long long rv =
          __hip_atomic_load(nmc_grole(d, cb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nmc_grole_is_fallback(d, rv)) return 0;
      if (patient && nmc_grole_patience_over(d, t0)) {
        const bool fb = lane == 0 ? nmc_grole_fallback(d, cb) : false;
        if (__builtin_amdgcn_readlane((int)fb, 0)) return 0;
        patient = false;   // a sibling has started: the likelihood kernel runs, wait for it
      }
    }
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
      return 0;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
// A likelihood workgroup's Gibbs wave waiting for task (cb, q)'s ready count (wave-uniform):
// 1 ready, -1 fallback (update it here), 0 timeout (d.tmo).
__device__ __forceinline__ int nmc_grole_own_wait(const Dev& d, int cb, int q, unsigned target) {
  const int lane = threadIdx.x & 63;
  const unsigned* ctr = nmc_hrd(d, cb, q);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool patient = true;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return 1;
    if ((spins & 63) == 63) {
      const unsigned long long rv =
          __hip_atomic_load(nmc_grole(d, cb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nmc_grole_is_fallback(d, rv)) return -1;
      if (patient && nmc_grole_patience_over(d, t0)) {
        const bool fb = lane == 0 ? nmc_grole_fallback(d, cb) : false;
        if (__builtin_amdgcn_readlane((int)fb, 0)) return -1;
        patient = false;   // a Gibbs workgroup has started: wait as long as it takes
      }
    }
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
      return 0;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
// The fallback's update of task (tq, q) by one wave: HyperParameter.update (:463-498) with
// the values streamed from global memory (sc1) in 8-value chunks -- nmc_pairwise_stream,
// the order of nmc_hyper / nmc_hyper_once -- and the task's variates from the fill's ring or
// drawn here (Dev.zin).  write: the global slot of tq and the sample row (group 0's wave).
// Inlined, with short chunks: a rare path (the Gibbs kernel did not run beside the sweep)
// whose registers must not cost the likelihood loop -- as a call it added 58 SGPR spills and
// 128 B of scratch to the cfg-4 instance; inlined with 32-value chunks, one VGPR spill.
__device__ __forceinline__ void nmc_hyper_update_stream(const Dev& d, int cb, int tq, int q,
                                                     int cc, double* lds, int hyp, bool write) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G, C = d.C;
  const double* src = ((tq & 1) ? d.vb1 : d.vb0) + (size_t)q * G * C + cc;
  nmc_d2 hv;
  if (d.zin) {
    hv = nmc_sweep_hyper_variate(d.rhz, d.rhu, d.replay_n, d.rng_mode, P, C,
                                 (uint32_t)(d.chain_base + cc), d.seed, d.ha, d.hlga, tq, q, cc);
  } else {
    const size_t hvi = (((size_t)(tq - d.vbase) * P + q) * C + cc) * 2;
    hv.a = d.vh[hvi];
    hv.b = d.vh[hvi + 1];
  }
  const double sdm = sqrt(lds[(hyp + NMC_HY_S2 * P + q) * 64 + lane] / G);
  const double tot = nmc_pairwise_stream<8>(d, src, false, 0.0);
  const double mu = tot / G + sdm * hv.a;                        // mu ~ N(mean(x), sqrt(s2/G))
  const double ss = nmc_pairwise_stream<8>(d, src, true, mu);
  nmc_hyper_finish(d, cb, tq, q, lds, hyp, write, mu, ss, hv.b);
}

// SYNC_OWN's Gibbs workgroup kb = (chain block, parameter q), four waves: every task (t, q)
// of the launch in order, once its publication is complete -- HyperParameter.update
// (:463-498) computed once per chain block, written through and counted ready (nmc_hrd)
// for the likelihood workgroups' Gibbs waves.
// GW: the waves of the Gibbs kernel of its own (nmc_k_sweep_gibbs: the one-load update, four
// streams per wave on 4 waves, two on 8); 0: inside nmc_k_sweep, where the update streams its
// values twice (168-VGPR budget shared with the likelihood code).
template <class Fam, int GW>
__device__ __forceinline__ void nmc_sweep_gibbs_wg(int kb, double* lds) {
  const nmc_sweep_args<Fam>* A = nmc_sweep_args_at<Fam>();
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int i0 = A->i0, i1 = A->i1;
#define d (A->d)
  const int P = d.P, G = d.G, C = d.C;
  const int hcb = d.cb0 + kb / P, q = kb % P;
  const int c = hcb * 64 + lane;
  const int cc = c < C ? c : C - 1;
  const nmc_lds_layout H = nmc_lds(0, P, 1, d.nleaf, d.ntail, W, G, 0, 0);
  double* hy = lds + H.hyp * 64 + lane;
  if (w == 0) {   // the state of q after iteration i0-1 (slot (i0-1) & 1)
    const size_t ho = nmc_hslot(d, i0 - 1) + (size_t)q * C + cc;
    hy[(NMC_HY_MU * P + q) * 64] = d.mu[ho];
    hy[(NMC_HY_SD * P + q) * 64] = d.hsd[ho];
    hy[(NMC_HY_LSD * P + q) * 64] = d.hlsd[ho];
    hy[(NMC_HY_S2 * P + q) * 64] = d.s2[ho];
  }
#ifdef NMC_STAMPS   // chain block 0's Gibbs workgroups, iterations < 8 of the launch:
                    // stamps[1024 + 4*4096 + ((t - i0) * 16 + 12 + q) * 4 + k]
#define NMC_GSTAMP(k)                                                                        \
  do {                                                                                       \
    if (d.stamps && hcb == 0 && q < 4 && t - i0 < 8 && threadIdx.x == 0)                      \
      d.stamps[1024 + 4 * 4096 + ((t - i0) * 16 + 12 + q) * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define NMC_GSTAMP(k) do {} while (0)
#endif
  for (int t = i0; t < i1; ++t) {
    A = nmc_sweep_args_at<Fam>();
    NMC_GSTAMP(3);
    if (GW > 0 && t == i0) {   // (Dev.gsep: the first task starts this workgroup, or the
                               //  likelihood workgroups have taken the launch over)
      if (threadIdx.x < 64) {
        const int r = nmc_grole_first_wait(d, hcb, q, (unsigned)d.G);
        if (threadIdx.x == 0) lds[H.flag * 64] = r ? 1.0 : 0.0;
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lds[H.flag * 64] == 0.0) break;
    } else if (!nmc_wait_published(d, hcb, q, (unsigned)d.G * (unsigned)(t - i0 + 1), lds, H)) {
      break;
    }
    NMC_GSTAMP(0);
    if (w == 0) {   // the task's variates and sqrt(s2 / G) of the previous update
      nmc_d2 hv;
      if (d.zin) {
        hv = nmc_sweep_hyper_variate(d.rhz, d.rhu, d.replay_n, d.rng_mode, d.P, d.C,
                                     (uint32_t)(d.chain_base + cc), d.seed, d.ha, d.hlga, t, q,
                                     cc);
      } else {
        const size_t hvi = (((size_t)(t - d.vbase) * d.P + q) * d.C + cc) * 2;
        hv.a = d.vh[hvi];
        hv.b = d.vh[hvi + 1];
      }
      lds[H.hv * 64 + (q * 64 + lane) * 2] = hv.a;
      lds[H.hv * 64 + (q * 64 + lane) * 2 + 1] = hv.b;
      hy[(NMC_HY_SDM * d.P + q) * 64] = sqrt(hy[(NMC_HY_S2 * d.P + q) * 64] / d.G);
    }
    __syncthreads();
    // HyperParameter.update (:463-498) for the chain block, written through to the global
    // slot of t (and the sample row); wave 0 stored it and counts it ready
#ifdef NMC_STAMPS   // the update's phases (entry 14 + q): pass 1, mean, pass 2
    {
      const double* src = (t & 1) ? d.vb1 : d.vb0;
      auto gs2 = [&](int k) {
        if (d.stamps && hcb == 0 && q < 2 && t - i0 < 8 && threadIdx.x == 0)
          d.stamps[1024 + 4 * 4096 + ((t - i0) * 16 + 14 + q) * 4 + k] = __builtin_amdgcn_s_memtime();
      };
      nmc_hyper_streams<NMC_SRC_SC1, false, 4>(d, src, cc, lds, H, q);
      __syncthreads();
      gs2(0);
      if (w == 0) {
        const double tot = nmc_hyper_combine(d, lds, H, q, lane);
        const double sdm = lds[(H.hyp + NMC_HY_SDM * P + q) * 64 + lane];
        const double hz = lds[H.hv * 64 + (q * 64 + lane) * 2];
        lds[(H.hyp + NMC_HY_MU * P + q) * 64 + lane] = tot / G + sdm * hz;
      }
      __syncthreads();
      gs2(1);
      nmc_hyper_streams<NMC_SRC_SC1, true, 4>(d, src, cc, lds, H, q);
      __syncthreads();
      gs2(2);
      // (diagnostics only: the full update below runs on the same inputs)
    }
#endif
    if (GW > 0 && d.nleaf * (8 + (d.ntail ? 1 : 0)) <= 16)   // every stream in one round
      nmc_hyper_once<GW == 8 ? 2 : 4>(d, (t & 1) ? d.vb1 : d.vb0, hcb, t, lds, H, q);
    else
      nmc_hyper<NMC_SRC_SC1, GW == 8 ? 1 : 4, true>(d, (t & 1) ? d.vb1 : d.vb0, hcb, t, lds, H,
                                                    true, q);
    NMC_GSTAMP(1);
    if (w == 0) {
      nmc_drain_vm();
      if (lane == 0)
        __hip_atomic_fetch_add(nmc_hrd(d, hcb, q), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    NMC_GSTAMP(2);
  }
#undef NMC_GSTAMP
  nmc_drain_vm();
#undef d
}

// Dev.gsep: the Gibbs workgroups of SYNC_OWN as a kernel of their own (RB * P workgroups
// of four waves, the small nmc_lds carve), launched on a second stream beside
// nmc_k_sweep's RB * G likelihood workgroups: co-resident with two 61-KB likelihood
// workgroups per CU where one kernel with a single LDS size would not be.
// GW: its waves (4: four streams per wave, every stream of a 256-group update in one round)
template <class Fam, int GW>
__global__ void __launch_bounds__(64 * GW) nmc_k_sweep_gibbs(nmc_sweep_args<Fam> a_arg) {
  (void)a_arg;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  // (its waves share a CU with two likelihood workgroups: issue ahead of their tile waves,
  //  the update is on every step's critical path; NMC_NOPRIO bit 2 drops it)
  if (!(a_arg.d.noprio & 2)) __builtin_amdgcn_s_setprio(3);
  nmc_sweep_gibbs_wg<Fam, GW>((int)blockIdx.x, lds);
}

template <class Fam, int MODE>
__global__ void __launch_bounds__(NMC_SWEEP_THREADS)
nmc_k_sweep(nmc_sweep_args<Fam> a_arg) {
  (void)a_arg;   // (read through nmc_sweep_args_at(): the same bytes)
  constexpr bool OWN = MODE == NMC_MODE_SYNC_OWN;
  constexpr bool PARTIAL = MODE == NMC_MODE_SYNC_REG || MODE == NMC_MODE_SYNC_LDS || OWN;
  constexpr bool HREG = MODE == NMC_MODE_SYNC_REG;
  constexpr bool HALF = MODE == NMC_MODE_HALF;
  constexpr int NF = Fam::NFIELDS;
  constexpr int MP = Fam::MAXP;
  static_assert(MODE == NMC_MODE_NOPOOL || MODE == NMC_MODE_HALF || PARTIAL, "sweep modes");
  (void)OWN;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const nmc_sweep_args<Fam>* A = nmc_sweep_args_at<Fam>();
#define d (A->d)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int i0 = A->i0, i1 = A->i1;

  // ---- SYNC_OWN: the Gibbs workgroups (blocks RB * G .., unless Dev.gsep puts them in
  //      their own kernel, nmc_k_sweep_gibbs) ----
  if constexpr (OWN) if (!d.gsep && (int)blockIdx.x >= d.RB * d.G) {
    nmc_sweep_gibbs_wg<Fam, 0>((int)blockIdx.x - d.RB * d.G, lds);
    return;
  }

  // (Dev.cb0: the first chain block of this launch -- resident batches of chain blocks)
  const int g = blockIdx.x % d.G, cb = d.cb0 + (int)blockIdx.x / d.G;
  const int c = HALF ? cb * 32 + (lane & 31) : cb * 64 + lane;
  const bool live = c < d.C && (!HALF || lane < 32);   // writes this lane's outputs
  const int cc = c < d.C ? c : d.C - 1;
  const bool ctl = w == 0;
  const bool gw = PARTIAL && w == 1;                    // the Gibbs wave
  const bool g0w = g == 0;                              // writes the chain block's hyper state
  // Everything else is re-derived from the laundered arguments where a step needs it, so the
  // persistent loop holds few values in registers: the step's view of the problem.
  struct View {
    int P, G, C, lag, gs0, ge, ngrp;
    size_t gc;
    nmc_sweep_layout L;
    nmc_tiling TI;
  };
  // (pro: the prologue's view, from the group offsets in HBM; the steps read the group's
  // row count and tiling from the LDS words the prologue stored, NMC_SWK_*)
  auto view = [&](bool pro = false) {
    View v;
    if (pro) {
      v.P = d.P; v.G = d.G; v.C = d.C;
      v.ngrp = (int)(d.off[g + 1] - d.off[g]);
      v.L = nmc_sweep_lds(Fam::NACC, v.P, PARTIAL, MODE == NMC_MODE_SYNC_LDS, v.G, d.nmax * NF);
      v.TI = nmc_tiles(v.ngrp, d.tile);
    } else {
      int k[NMC_SWK_COUNT];
      const int* kw = (const int*)lds + NMC_SWK_AT;
#pragma unroll
      for (int j = 0; j < NMC_SWK_COUNT; ++j) k[j] = __builtin_amdgcn_readfirstlane(kw[j]);
      v.P = k[NMC_SWK_P]; v.G = k[NMC_SWK_G]; v.C = k[NMC_SWK_C]; v.ngrp = k[NMC_SWK_NGRP];
      v.TI.n = k[NMC_SWK_N]; v.TI.nt = k[NMC_SWK_NT]; v.TI.h = k[NMC_SWK_H];
      v.TI.a = k[NMC_SWK_A]; v.TI.b = k[NMC_SWK_B];
      v.L.th = k[NMC_SWK_TH]; v.L.part = k[NMC_SWK_PART]; v.L.st = k[NMC_SWK_ST];
      v.L.hyp = k[NMC_SWK_HYP]; v.L.hval = k[NMC_SWK_HVAL]; v.L.zl = k[NMC_SWK_ZL];
      v.L.zm = k[NMC_SWK_ZM]; v.L.cw = k[NMC_SWK_CW]; v.L.flag = k[NMC_SWK_FLAG];
      v.L.rows = k[NMC_SWK_ROWS]; v.L.total = k[NMC_SWK_TOTAL];
    }
    v.lag = v.P >= 2 ? 2 : 1;                           // Gibbs task of step gs: gs - lag
    v.gs0 = i0 * v.P; v.ge = i1 * v.P;
    v.gc = (size_t)g * v.C + cc;
    return v;
  };
  auto hl_view = [](const nmc_sweep_layout& L) {   // the Gibbs helpers' view of the carve
    nmc_lds_layout H;
    H.hval = L.hval;
    H.hyp = L.hyp;
    H.flag = L.flag;
    return H;
  };
  // the task this workgroup closes after the loop: ge-lag+g (groups 0 .. lag-1), -1: none
  auto close_task = [&](const View& v) {
    const int k0 = v.ge - v.lag > v.gs0 ? v.ge - v.lag : v.gs0;
    return PARTIAL && !OWN && k0 + g < v.ge ? k0 + g : -1;
  };
  // {z, log u} of step (tn, pn) -> LDS slot `slot` (this lane's chain)
  // {z, log u} of step (tn, pn) -> LDS slot `slot`: part j of the draw (Dev.zin; j = 3: all
  // three), or the LDS-DMA of the pair nmc_k_fill wrote to the ring vzl (the issuing wave
  // drains its vmcnt before the next barrier; zm holds 1.0)
  auto put_variates = [&](const View& v, int tn, int pn, int slot, int j) {
    if (d.zin) {
      for (int jj = j == 3 ? 0 : j; jj <= (j == 3 ? 2 : j); ++jj) {
        const double x = nmc_sweep_variate_part(d.rz, d.ru, d.replay_n, d.rng_mode, v.P, v.G,
                                                v.C, (uint32_t)(d.chain_base + cc), d.seed, tn,
                                                pn, g, cc, jj);
        if (jj == 1) lds[(v.L.zm + slot) * 64 + lane] = x;
        else lds[(v.L.zl + 2 * slot) * 64 + 2 * lane + (jj == 2 ? 1 : 0)] = x;
      }
    } else {
      nmc_dma16(d.vzl + ((size_t)(tn - d.vbase) * v.P * v.G * v.C + (size_t)pn * v.G * v.C +
                         v.gc) * 2,
                lds + (v.L.zl + 2 * slot) * 64);
    }
  };
  // this lane's proposal normal and log u of the step in slot sp
  auto zval = [&](const nmc_sweep_layout& L, int sp) {
    return lds[(L.zl + 2 * sp) * 64 + 2 * lane] * lds[(L.zm + sp) * 64 + lane];
  };

  NMC_RUN_SL(0);
  // ---- prologue: the group's rows -> LDS (LDS-DMA, 1 KiB per wave-instruction), values and
  //      state -> LDS (parameter p by wave p % W) ----
  {
    const View v = view(true);
    const nmc_sweep_layout& L = v.L;
    double* lrows = lds + L.rows * 64;
    const int64_t ra0 = d.off[g];
    const double* grows = d.obs + ra0 * NF;
    const int nd = v.ngrp * NF;
    if (((ra0 * NF) & 1) == 0) {   // 16-byte pieces; an odd nd copies one double of slack
      const int npc = (nd + 1) / 2;
      for (int b0 = w * 64; b0 < npc; b0 += W * 64)
        if (b0 + lane < npc) nmc_dma16(grows + 2 * (b0 + lane), lrows + 2 * b0);
    } else {
      for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
    }
    const int P = v.P, G = v.G, C = v.C;
    double* th = lds + L.th * 64 + lane;
    double* st = lds + L.st * 64 + lane;
    double* hy = lds + L.hyp * 64 + lane;
    const double* vin = ((i0 - 1) & 1) ? d.vb1 : d.vb0;
    for (int p = w; p < P; p += W) {
      const size_t ip = (size_t)p * G * C + v.gc;
      th[p * 64] = vin[ip];
      st[(NMC_ST_S * P + p) * 64] = d.scale[ip];
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
    if (ctl) {
      put_variates(v, i0, 0, v.gs0 & 1, 3);   // {z, log u} of the launch's first step
      if (!d.zin)   // (the fill's ring holds z itself)
        for (int k = 0; k < 2; ++k) lds[(L.zm + k) * 64 + lane] = 1.0;
      for (int j = 0; j < Fam::NACC; ++j)   // x + (-0.0) == x: the fixed slot sum
        for (int k = v.TI.nt; k < NMC_NSLOT; ++k)
          lds[(L.part + j * NMC_NSLOT + k) * 64 + lane] = -0.0;
      lds[L.flag * 64 + lane] = 0.0;
      if (lane < 2)   // both tile queues: the first nq entries go by rank
        ((unsigned*)(lds + L.flag * 64 + 4))[lane] = (unsigned)(W - 1 - (PARTIAL ? 1 : 0));
      if (lane == 0) {                     // the step constants (view())
        int* kw = (int*)lds + NMC_SWK_AT;
        kw[NMC_SWK_P] = v.P; kw[NMC_SWK_G] = v.G; kw[NMC_SWK_C] = v.C;
        kw[NMC_SWK_NGRP] = v.ngrp;
        kw[NMC_SWK_N] = v.TI.n; kw[NMC_SWK_NT] = v.TI.nt; kw[NMC_SWK_H] = v.TI.h;
        kw[NMC_SWK_A] = v.TI.a; kw[NMC_SWK_B] = v.TI.b;
        kw[NMC_SWK_TH] = L.th; kw[NMC_SWK_PART] = L.part; kw[NMC_SWK_ST] = L.st;
        kw[NMC_SWK_HYP] = L.hyp; kw[NMC_SWK_HVAL] = L.hval; kw[NMC_SWK_ZL] = L.zl;
        kw[NMC_SWK_ZM] = L.zm; kw[NMC_SWK_CW] = L.cw; kw[NMC_SWK_FLAG] = L.flag;
        kw[NMC_SWK_ROWS] = L.rows; kw[NMC_SWK_TOTAL] = L.total;
      }
    }
    nmc_drain_vm();                        // this wave's row DMA has landed
  }
  __syncthreads();
  NMC_RUN_SL(1);

  // ---- the likelihood of the proposal (:615-635), tile by tile from the step's LDS queue;
  //      with Dev.zin its first entries draw the next step's variates.  role 0: a queue wave,
  //      1: the control wave, 2: the Gibbs wave ----
  auto run_tiles = [&](const View& v, int t, int p, int role, auto&& after_first) {
    const int P = v.P;
    const nmc_sweep_layout& L = v.L;
    const double* th = lds + L.th * 64 + lane;
    const double* st = lds + L.st * 64 + lane;
    unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);   // tile queues by step parity
    const Fam& fam = A->fam;
    const int sp = (t * P + p) & 1;
        double thp[MP];
#pragma unroll
        for (int q = 0; q < MP; ++q) thp[q] = q < P ? th[q * 64] : 0.0;
        const double prop = thp[p] + (1.0 * st[(NMC_ST_S * P + p) * 64]) * zval(L, sp);
#pragma unroll
        for (int q = 0; q < MP; ++q)
          if (q == p) thp[q] = prop;
        const typename Fam::Reg reg = fam.prepare(thp);
        // quad rows ({x, y}, kernels.h nmc_ll_rows_lds_quad): intercept and slope of the four
        // chains of this lane's quarter position
        const bool quad = Fam::ASM_ROWS && !HALF && d.quad;
        double q4c[4], q4d[4];
        if constexpr (Fam::ASM_ROWS && !HALF) if (quad) {
          nmc_quarters(reg.b0, q4c);
          nmc_quarters(reg.b[0], q4d);
        }
        typename Fam::Reg preg = reg;   // paired rows: the partner lane's (lane ^ 32) values
        if constexpr (nmc_paired_rows_ok<Fam>() && !HALF) if (d.paired && !quad) {
          const bool hi = lane >= 32;
#pragma unroll
          for (int q = 0; q < MP; ++q) {
            const nmc_pair2 e = nmc_halves(thp[q]);
            thp[q] = hi ? e.lo : e.hi;
          }
          preg = fam.prepare(thp);
        }
        const double* lrows = lds + L.rows * 64;
        const int tn = p + 1 < P ? t : t + 1, pn = p + 1 < P ? p + 1 : 0;
        const int zj = tn < i1 && d.zin ? 3 : 0;   // (the fill's ring: the control wave's DMA)
        const int nt = v.TI.nt;
        // The step's entries [0, ne): the zj variate jobs, then the nt tiles, in one LDS
        // queue.  The nq queue waves (all but the control and the Gibbs wave) start on
        // entries 0 .. nq-1 by rank, without a take (the counter starts at nq); further
        // entries go to whichever wave asks first, the next take in flight during the entry.
        // The control wave arrives after its pre-work and takes only while the others have
        // more than a round left (Dev.ctiles), so it never ends the step last.  Entry ->
        // partial slot is fixed: the sums stay in order.
        const int ne = nt + zj;
        unsigned* qc = tcnt + sp;
        const int nq = W - 1 - (PARTIAL ? 1 : 0);
        auto issue = [&]() -> unsigned {   // lane 0: a take
          return lane == 0 ? __hip_atomic_fetch_add(qc, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP)
                           : 0u;
        };
        auto resolve = [&](unsigned i) -> int {   // the entry, -1: the queue is empty
          const int e = (int)__builtin_amdgcn_readlane(i, 0);
          return e < ne ? e : -1;
        };
        // role 1: the control wave (Dev.ctiles), 2: the Gibbs wave (Dev.gtiles) -- both take
        // only while the queue waves have more than a round left
        const int pol = role == 1 ? d.ctiles : role == 2 ? d.gtiles : 2;
        const bool cpick = role != 0 && pol != 2;
        auto ctake = [&]() -> int {   // control: only while the others have a round left
          if (pol != 1) return -1;
          const unsigned i = lane == 0 ? __hip_atomic_load(qc, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP)
                                       : 0u;
          return ne - (int)__builtin_amdgcn_readlane(i, 0) > nq ? resolve(issue()) : -1;
        };
        const int rank = w - 1 - (PARTIAL ? 1 : 0);   // (control: -1)
        NMC_RS_STAMP((t - i0) * P + p, 2);
        int kq = cpick ? ctake() : role != 0 ? resolve(issue()) : (rank < ne ? rank : -1);
        NMC_RS_STAMP((t - i0) * P + p, 3);
        // after_first: once, after this wave's first queue entry (or with none) -- the
        // control's count of the previous step's published value waits for its store there,
        // off the step's critical path
        bool first = true;
        if (d.pubearly) {   // (Dev.pubearly: before this wave's first entry)
          after_first();
          first = false;
        }
        while (kq >= 0) {
          const unsigned kn = cpick ? 0u : issue();
          NMC_TILE_STAMP(kq, 0);
          if (kq < zj) {
            put_variates(v, tn, pn, sp ^ 1, kq);
          } else {
            const int k = kq - zj;
            const int ra = v.TI.start(k), rn = v.TI.len(k);
            double acc[Fam::NACC];
            bool done = false;
            if constexpr (Fam::ASM_ROWS && !HALF) if (quad) {
              nmc_ll_rows_lds_quad(fam, reg, lrows + (size_t)ra * NF, rn, acc, q4c, q4d);
              done = true;
            }
            if constexpr (nmc_paired_rows_ok<Fam>()) if (!done && (HALF || d.paired)) {
              nmc_ll_rows_lds<Fam, true, HALF>(fam, reg, lrows + (size_t)ra * NF, rn, acc, &preg);
              done = true;
            }
            if (!done) nmc_ll_rows_lds(fam, reg, lrows + (size_t)ra * NF, rn, acc);
#pragma unroll
            for (int j = 0; j < Fam::NACC; ++j) lds[(L.part + j * NMC_NSLOT + k) * 64 + lane] = acc[j];
          }
          NMC_TILE_STAMP(kq, 1);
          if (first) {
            after_first();
            first = false;
          }
          kq = cpick ? ctake() : resolve(kn);
        }
        if (first) after_first();   // (no entry was left)
  };

  bool ok = true;
  // ---- the Gibbs wave: its own loop, meeting the others at both barriers of every step ----
  if constexpr (PARTIAL) if (gw) {
    if (!(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);
    bool gfall = false;   // (SYNC_OWN, Dev.gsep: this launch's tasks are updated here)
    // task k = (kt, kq): poll its publication, update (HyperParameter.update :463-498),
    // write (the global slot of kt and the sample row); priors: this step's priors from the
    // update (p, sp, t: the step); returns the poll's verdict
    auto task = [&](const View& v, int k, bool write, bool priors, int p, int sp, int t) -> bool {
      const int P = v.P, G = v.G, C = v.C;
      const nmc_sweep_layout& L = v.L;
      const int kq = k % P, kt = k / P;
      if constexpr (OWN) {   // the Gibbs workgroup of (cb, kq) has counted task k ready
        const unsigned target = (unsigned)(kt - i0 + 1) + d.pbase;
        if (!d.gsep) {
          if (!nmc_poll_count(d, nmc_hrd(d, cb, kq), target)) return false;
        } else if (!gfall) {   // (its own kernel: or nobody has started it, nmc_grole_*)
          const int r = nmc_grole_own_wait(d, cb, kq, target);
          if (r == 0) return false;
          gfall = r < 0;
        }
        if (gfall) {   // the fallback: this wave updates task k (group 0's writes, counts it)
          if (!nmc_poll_published(d, cb, kq, (unsigned)G * (unsigned)(kt - i0 + 1))) return false;
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          nmc_hyper_update_stream(d, cb, kt, kq, cc, lds, L.hyp, write);
          if (write) {
            nmc_drain_vm();   // (stored before counted, as the Gibbs workgroup does)
            if (lane == 0)
              __hip_atomic_fetch_add(nmc_hrd(d, cb, kq), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      } else {
        if (!nmc_poll_published(d, cb, kq, (unsigned)G * (unsigned)(kt - i0 + 1))) return false;
      }
      // keep the payload loads below the poll (no instruction: wavefront scope)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if constexpr (OWN) {
        if (!gfall) nmc_hyper_read(d, kt, kq, cc, lds, L.hyp);
      } else {
        nmc_d2 hv;
        if (d.zin) {
          hv = nmc_sweep_hyper_variate(d.rhz, d.rhu, d.replay_n, d.rng_mode, P, C,
                                       (uint32_t)(d.chain_base + cc), d.seed, d.ha, d.hlga, kt, kq,
                                       cc);
        } else {   // the fill kernel's pair
          const size_t hvi = (((size_t)(kt - d.vbase) * P + kq) * C + cc) * 2;
          hv.a = d.vh[hvi];
          hv.b = d.vh[hvi + 1];
        }
        if constexpr (HREG) {
          double xv[64];
          const double* src = ((kt & 1) ? d.vb1 : d.vb0) + (size_t)kq * G * C + cc;
#pragma unroll
          for (int u = 0; u < 64; ++u) xv[u] = nmc_ldv<NMC_SRC_SC1>(src + (size_t)u * C);
          nmc_hyper_compute_reg(d, cb, kt, kq, lds, L.hyp, write, hv.a, hv.b, xv);
        } else {
          const nmc_lds_layout H = hl_view(L);
          const double* src = (kt & 1) ? d.vb1 : d.vb0;
          if ((C & 1) == 0) {
            nmc_hyper_dma(d, src, kq, cb, 0, G, lds, H, 0);
            nmc_drain_vm();
          } else {
            nmc_hyper_load(d, src, kq, cc, 0, G, lds, H, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          nmc_hyper_compute(d, cb, kt, kq, lds, H, write, hv.a, hv.b, 0);
        }
      }
      if (priors) {   // the update lands in the step that needs it: this step's priors
        const double* th = lds + L.th * 64 + lane;
        const double* st = lds + L.st * 64 + lane;
        const double* hy = lds + L.hyp * 64 + lane;
        double* cwv = lds + L.cw * 64 + lane;
        const double x = th[p * 64];
        const double prop = x + (1.0 * st[(NMC_ST_S * P + p) * 64]) * zval(L, sp);
        const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
        const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
        cwv[NMC_CW_LPC * 64] =
            t > 0 ? nmc_norm_logpdf_r(x, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
        cwv[NMC_CW_LPP * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
      }
      return true;
    };
    for (int t = i0; t < i1 && ok; ++t) {
      for (int p = 0; p < d.P; ++p) {
        A = nmc_sweep_args_at<Fam>();
        const View v = view();
        const int gs = t * v.P + p, sp = gs & 1;
        const bool due = gs - v.lag >= v.gs0;
        if (p == 0) NMC_STAMP_AUX(t, 13);
        if (due) {
          const bool r = task(v, gs - v.lag, g0w, v.P <= 2, p, sp, t);
          if (p == 0) NMC_STAMP_AUX(t, 14);
          if (lane == 0)
            __hip_atomic_store(lds + v.L.flag * 64 + 1 + sp,
                               r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // then the step's tiles while the queue waves have more than a round left
        if (d.gtiles) run_tiles(v, t, p, 2, []() {});
        NMC_ARRIVE_STAMP((t - i0) * v.P + p);
        nmc_step_barrier();   // A
        if (due) {
          ok = lds[v.L.flag * 64 + 1 + sp] == 2.0 * ((double)gs + 1);
          if (!ok) break;
        }
        nmc_step_barrier();   // B
      }
    }
    // closing: task close_k (the matching barrier of the other waves' nmc_wait_published)
    A = nmc_sweep_args_at<Fam>();
    const View v = view();
    const int close_k = close_task(v);
    if (ok && close_k >= 0) {
      if (nmc_wait_published(d, cb, close_k % v.P,
                             (unsigned)v.G * (unsigned)(close_k / v.P - i0 + 1), lds,
                             hl_view(v.L)))
        task(v, close_k, true, false, 0, 0, 0);
    }
    // SYNC_OWN, Dev.gsep: group 0's wave sees the launch's last tasks done -- by the Gibbs
    // kernel (ready counts), or by itself when nobody started them (the fallback; also when
    // the launch is too short for any task to fall due in the loop)
    if constexpr (OWN) if (ok && d.gsep && g0w) {
      for (int k = v.ge - v.lag > v.gs0 ? v.ge - v.lag : v.gs0; k < v.ge && ok; ++k)
        ok = task(v, k, true, false, 0, 0, 0);
    }
    nmc_drain_vm();
    return;
  }

  // ---- control wave and likelihood waves ----
  if (ctl && W > 1 && !(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);
  int pub_p = -1;                  // control: parameter whose sc1 value store awaits its count
  int pend_p = -1, pend_t = 0;     // control: decided step whose state update is pending
  double c_LL = 0.0;               // control: the group LL of the current state
  if (ctl) {
    const View v = view();
    c_LL = d.ll[v.gc];
  }
  bool q_acc = false;
  double q_plp = 0, q_pll = 0;
  // the rest of a decided step's update (:369-383, :608-610): counters, log prior, LL,
  // sample and trace rows
  auto apply_pending = [&](const View& v) {
    const int P = v.P, G = v.G, C = v.C;
    const nmc_sweep_layout& L = v.L;
    double* th = lds + L.th * 64 + lane;
    double* st = lds + L.st * 64 + lane;
    const double* cwv = lds + L.cw * 64 + lane;
    const int q = pend_p, tq = pend_t;
    st[(NMC_ST_LP * P + q) * 64] = q_plp;
    st[(NMC_ST_NA * P + q) * 64] = cwv[(q_acc ? NMC_CW_NAA : NMC_CW_NAR) * 64];
    st[(NMC_ST_NR * P + q) * 64] = cwv[(q_acc ? NMC_CW_NRA : NMC_CW_NRR) * 64];
    st[(NMC_ST_TA * P + q) * 64] = cwv[NMC_CW_TA * 64] + (q_acc ? 1.0 : 0.0);
    if (q_acc) c_LL = q_pll;
    if (live) {
      const int row = nmc_record_row(d, tq);
      if (row >= 0) {
        const int col = q * (G + (PARTIAL ? 2 : 0)) + (PARTIAL ? 2 : 0) + g;
        d.samples[((size_t)row * d.cols + col) * C + c] = th[q * 64];
      }
      if (tq < d.trace_n) {
        const size_t it = (((size_t)tq * P + q) * G + g) * C + c;
        d.tflag[it] = q_acc ? 1 : 0;
        d.tllp[it] = q_pll;
      }
    }
    pend_p = -1;
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
    NMC_STAMP(t, 0);
    for (int p = 0; p < d.P; ++p) {
      NMC_RS_STAMP((t - i0) * d.P + p, 0);
      A = nmc_sweep_args_at<Fam>();
      const View v = view();
      const int P = v.P, G = v.G, C = v.C;
#ifdef NMC_STAMPS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      NMC_RS_STAMP((t - i0) * P + p, 1);
#endif
      const nmc_sweep_layout& L = v.L;
      double* th = lds + L.th * 64 + lane;
      double* st = lds + L.st * 64 + lane;
      double* hy = lds + L.hyp * 64 + lane;
      double* cwv = lds + L.cw * 64 + lane;
      unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);   // tile queues by step parity
      (void)G; (void)C; (void)tcnt;   // (not every instance uses them)
      const Fam& fam = A->fam;
      const int gs = t * P + p, sp = gs & 1;
      const bool due = PARTIAL && gs - v.lag >= v.gs0;   // the Gibbs wave has a task this step
      const bool post_prior = due && P <= 2;             // ... whose update this step's prior needs
      // ---- control: the pending update of step gs-1 and this step's decision operands:
      //      the proposal, both outcomes of the counters and of the (tuned) scale, priors ----
      double c_prop = 0, c_v = 0, c_lu = 0, c_lpc = 0, c_lpp = 0, c_sA = 0, c_sR = 0;
      typename Fam::Reg c_reg{};
      if (ctl) {
        {   // the next step's {z, log u} from the fill's ring, in flight first: its latency
            // overlaps everything below (d.zin: a queue job instead).  The slot held step
            // gs-1's pair, read by every wave before barrier B of gs-1.
          const int tn = p + 1 < P ? t : t + 1, pn = p + 1 < P ? p + 1 : 0;
          if (tn < i1 && !d.zin) put_variates(v, tn, pn, sp ^ 1, 3);
        }
        if (pend_p >= 0) apply_pending(v);
        c_v = th[p * 64];
        const double s = st[(NMC_ST_S * P + p) * 64];
        c_prop = c_v + (1.0 * s) * zval(L, sp);                              // propose (:304-306)
        c_lu = lds[(L.zl + 2 * sp) * 64 + 2 * lane + 1];
        {
          double thp[MP];
#pragma unroll
          for (int q = 0; q < MP; ++q) thp[q] = q < P ? (q == p ? c_prop : th[q * 64]) : 0.0;
          c_reg = fam.prepare(thp);
        }
        const double na = st[(NMC_ST_NA * P + p) * 64], nr = st[(NMC_ST_NR * P + p) * 64];
        double naA = na + 1.0, nrA = nr, naR = na, nrR = nr + 1.0;
        c_sA = s;
        c_sR = s;
        // (the control wave's alone: the burn-in / interval loads and the division stay off
        //  the other waves' restart)
        const bool tune = t > 0 && t < d.burn && t % d.tune_interval == 0;
        if (tune) {
          nmc_tune(c_sA, naA, nrA);
          nmc_tune(c_sR, naR, nrR);
        }
        cwv[NMC_CW_NAA * 64] = naA;
        cwv[NMC_CW_NRA * 64] = nrA;
        cwv[NMC_CW_NAR * 64] = naR;
        cwv[NMC_CW_NRR * 64] = nrR;
        cwv[NMC_CW_TA * 64] = st[(NMC_ST_TA * P + p) * 64];
        if (!post_prior) {   // priors (:293-294)
          if constexpr (PARTIAL) {
            const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
            const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
            c_lpc = t > 0 ? nmc_norm_logpdf_r(c_v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
            c_lpp = nmc_norm_logpdf_r(c_prop, m, sd, isd, lsd);
          } else {
            c_lpc = st[(NMC_ST_LP * P + p) * 64];
            c_lpp = nmc_sweep_prior(d.pfam[p], d.ppar + 8 * p, c_prop);
          }
        }
      }

      if (p == 0) NMC_STAMP(t, 8);   // (control: its pre-work done)
      // ---- every wave: the likelihood of the proposal (:615-635), tile by tile from the
      //      step's LDS queue; entry 0 (when there is a next step) draws its variates ----
      run_tiles(v, t, p, ctl ? 1 : 0, [&]() {
        if constexpr (PARTIAL) if (ctl) count_published();
      });
      if (p == 0) NMC_STAMP(t, 9);
      if (ctl) nmc_drain_vm();   // (its variate DMA has landed)
      if (p == 0) NMC_STAMP(t, 10);
      NMC_STAMP(t, 1 + 3 * (p & 1));
      NMC_ARRIVE_STAMP((t - i0) * P + p);
      nmc_step_barrier();   // A: every tile partial, the next step's variates, the Gibbs priors
      NMC_STAMP(t, 2 + 3 * (p & 1));
      NMC_CTL_STAMP((t - i0) * P + p, 0);
      {   // the view re-derived after the tile loop (nothing of it stays live across the loop)
      A = nmc_sweep_args_at<Fam>();
      const View v = view();
      const nmc_sweep_layout& L = v.L;
      double* th = lds + L.th * 64 + lane;
      double* st = lds + L.st * 64 + lane;
      double* cwv = lds + L.cw * 64 + lane;
      unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);
      const Fam& fam = A->fam;
      const int G = v.G, C = v.C;

      // (partial pooling: the Gibbs wave's verdict is read in the same batch as the operands
      // and checked after the decision; an aborted step's decision is never used)
      const double verdict = due ? lds[L.flag * 64 + 1 + sp] : 0.0;
      // ---- control: group log-likelihood of the proposal (tiles in order) and the
      //      Metropolis decision, one chain per lane (:334-383) ----
      if (ctl) {
        // every entry is taken; the queue is reused at step gs + 2 (its first nq entries
        // by rank)
        if (lane == 0) tcnt[sp] = (unsigned)(W - 1 - (PARTIAL ? 1 : 0));
        if (post_prior) {   // the Gibbs wave evaluated this step's priors (read in the slot
                            // sums' LDS round trip)
          c_lpc = cwv[NMC_CW_LPC * 64];
          c_lpp = cwv[NMC_CW_LPP * 64];
        }
        double acc[Fam::NACC];
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j)
          acc[j] = nmc_sum_slots(lds + (L.part + j * NMC_NSLOT) * 64 + lane);
        const double llp = fam.finish_fast(c_reg, acc, (long)v.ngrp, fam.gconst((long)v.ngrp));
        const double postp = c_lpp + llp;
        const double post = c_lpc + c_LL;
        const double diff = postp - post;
        bool accept;
        if (!isfinite(post) && isfinite(postp)) accept = true;        // :347-352
        else if (!isfinite(llp)) accept = false;                      // :354-356
        else if (!isfinite(diff)) accept = false;                     // :358-360
        else accept = c_lu < diff;                                    // :362-364
        // :369-383, :608-610 (+ tune :385-437, prepared above)
        const double vn = accept ? c_prop : c_v;
        th[p * 64] = vn;
        if constexpr (PARTIAL) {   // publish write-through; counted at the next step's start
          if (live)
            __hip_atomic_store(((t & 1) ? d.vb1 : d.vb0) + (size_t)p * G * C + v.gc, vn,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pub_p = p;
        }
        st[(NMC_ST_S * P + p) * 64] = accept ? c_sA : c_sR;
        q_acc = accept;
        q_plp = accept ? c_lpp : c_lpc;
        q_pll = llp;
        pend_p = p;
        pend_t = t;
      }
      if (due) {
        ok = verdict == 2.0 * ((double)gs + 1);
        if (!ok) break;
      }
      }
      if (p == 0) NMC_STAMP(t, 3);
      NMC_CTL_STAMP((t - i0) * P + p, 1);
      nmc_step_barrier();   // B: the decided value is visible to every wave
      NMC_CTL_STAMP((t - i0) * P + p, 2);
    }
    NMC_STAMP(t, 6);
  }

  NMC_RUN_SL(2);
  A = nmc_sweep_args_at<Fam>();
  const View v = view();
  if (ctl) {
    if constexpr (PARTIAL) count_published();   // the last parameter's count
    if (pend_p >= 0) apply_pending(v);
  }
  // ---- epilogue: state back to HBM (control wave) ----
  if (ctl && live && ok) {
    const int P = v.P, G = v.G, C = v.C;
    const double* th = lds + v.L.th * 64 + lane;
    const double* st = lds + v.L.st * 64 + lane;
    double* vo = ((i1 - 1) & 1) ? d.vb1 : d.vb0;
    for (int p = 0; p < P; ++p) {
      const size_t ip = (size_t)p * G * C + v.gc;
      if (!PARTIAL) vo[ip] = th[p * 64];   // (partial pooling: published write-through)
      d.lp[ip] = st[(NMC_ST_LP * P + p) * 64];
      d.scale[ip] = st[(NMC_ST_S * P + p) * 64];
      d.nacc[ip] = (int)st[(NMC_ST_NA * P + p) * 64];
      d.nrej[ip] = (int)st[(NMC_ST_NR * P + p) * 64];
      d.tacc[ip] = (long long)st[(NMC_ST_TA * P + p) * 64];
    }
    d.ll[v.gc] = c_LL;
  }
  // ---- closing Gibbs task (partial pooling): the Gibbs wave computes it; this is the
  //      matching barrier of its nmc_wait_published ----
  if constexpr (PARTIAL) {
    const int close_k = close_task(v);
    if (ok && close_k >= 0)
      nmc_wait_published(d, cb, close_k % v.P, (unsigned)v.G * (unsigned)(close_k / v.P - i0 + 1),
                         lds, hl_view(v.L));
  }
  nmc_drain_vm();
  NMC_RUN_SL(3);
#undef d
}
