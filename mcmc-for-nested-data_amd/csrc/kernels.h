// kernels.h -- the MCMC sampling kernels for gfx950 (CDNA4, wave64, fp64).
//
// Layout: chain-on-lane.  A workgroup owns one (chain block of 64 chains, group g)
// pair (none/complete pooling on few workgroups: 32 chains, NMC_MODE_HALF); its W waves
// split the group's CSR rows obs[off[g]..off[g+1]), staged once per launch in LDS.
// Every lane holds one chain's parameters in registers while the wave walks the same
// rows, so one broadcast ds_read feeds 64 chains (the paired loop: two chains per lane,
// one row pair per read) -- the cross-chain reuse that keeps the dataset on chip.
//
// nmc_k_run runs the reference's Sampler._loop body (posteriorSampling.py:872-891)
// for iterations [i0, i1) of every (chain, group).  Per parameter step p
// (StepMethod.step :594-613):
//   1. every wave proposes theta_p' = theta_p + scale*z (Parameter.propose :304-306)
//      and takes likelihood row tiles of the group from an LDS queue (:615-635); the
//      tile partition depends on the rows alone, so every sum is fixed;
//   2. barrier A: the control wave (wave 0) adds the tile partials in a fixed order and
//      makes the Metropolis decision (:334-383, branch order exact, IEEE isfinite),
//      tuning (:385-437) and group-LL propagation (:608-610);
//   3. barrier B: the decided value is visible; the rest of the state update is
//      deferred into the next step's slack.
// The step's {z, log u} are drawn by a job in the previous step's tile queue (Philox,
// or the replayed reference variates).
//
// Partial pooling couples the G groups of a chain through the Gibbs update of the
// hyper-parameters (HyperParameter.update :463-498).  The update of parameter q after
// iteration t is needed first by the decision of step (t + 1, q), not by any
// likelihood, so it is pipelined behind the steps in between:
//   * persistent modes (every workgroup resident): decided values are published
//     write-through (sc1 stores, vmcnt drain, one agent-scope counter add per
//     workgroup and step); the Gibbs wave (wave 1) polls the chain block's counter two
//     steps later, reads the values with sc1 loads (MI355X_MICROARCH.md, inter-workgroup
//     visibility) and updates in numpy's pairwise order (exact mean/variance parity);
//   * launch-per-iteration mode (grid too large to be resident): the kernel boundary
//     publishes, plain loads read.
// Every spin is bounded: a timeout sets d.tmo (pinned host memory) and every
// workgroup drains.
#pragma once
#ifndef __HIPCC_RTC__   // (hiprtc, user families: the runtime provides these)
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "families.h"
#include "rng.h"
#include "special.h"

struct Dev {
  int C, G, P, pooling, nf, chain_base, rng_mode, W, CB;
  // step kernel: chains per workgroup CL (64, one per lane; reported by
  // nmc_launch_config) and its chain blocks RB = ceil(C / CL).  (A 32-chain half-lane
  // layout -- two workgroups per CU -- measured 11.5 against 8.5 us per iteration at
  // cfg 3 and was removed.)
  int CL, RB;
  int paired;            // likelihood rows: two chains per lane (nmc_ll_rows_lds<Fam, true>)
  int quad;              // nmc_k_run, {x, y} rows in LDS: four chains per lane
                         // (nmc_ll_rows_lds_quad; NMC_ROWS=pair keeps the paired loop)
  // Row split (none/complete pooling with large groups): S workgroups ("members") share
  // one (chain block, group), member m owning the m-th contiguous chunk of the group's
  // rows (nmc_chunk); each step they exchange their partial sums through xbuf
  // ([2 step parity][RB][G][S][NACC][64], sc1 stores + the unit's counter xcnt[RB*G][32])
  // and all make the same decision.  S depends on the rows, the group count and the CU
  // count only, never on the chain count: results are shard- and batch-invariant.
  // cb0: first chain block of this launch (chain blocks are launched in resident batches).
  int S, cb0;
  // publish / exchange counters are never reset between launches: they already hold
  // G * pbase publishes per (chain block, parameter) and S * xbase arrivals per unit from
  // the context's earlier launches (the host advances both; no memset per launch)
  unsigned pbase, xbase;
  double* xbuf;
  unsigned* xcnt;
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
  int hreg;              // persistent partial, G <= 64: Gibbs payload in registers (SYNC_REG)
  int xpc;               // nmc_k_run, persistent partial pooling, RB | 8: XCDs per chain block
                         // (workgroup placement, nmc_k_run; 0: chain-block-major)
  unsigned* hrd;         // [RB][P][32] hyper-ready counts of nmc_k_sweep's Gibbs workgroups
                         // (SYNC_OWN; pbase tasks per parameter before)
  int noprio;            // diagnostics: no issue priority for the latency-bound waves
  int pubearly;          // nmc_k_sweep: the control counts the previous step's publication
                         // before taking a tile (its store drained first), not after one
  int gwaves;            // waves of nmc_k_sweep_gibbs (4)
  int nstatic;           // nmc_k_run: waves 2.. start on static tile entries (W - 2; 0 off,
                         // NMC_STATIC_TILES=0)
  int gsep;              // nmc_k_sweep SYNC_OWN: the Gibbs workgroups run as their own kernel
                         // (nmc_k_sweep_gibbs) on a second stream
  // gsep progress without co-scheduling (sweep.h nmc_grole_*): per chain block a role word
  // [63:32] launch epoch, [31:1] Gibbs workgroups started, [0] fallback -- if the Gibbs
  // kernel has not started within gpat ticks (s_memrealtime, 100 MHz), the likelihood
  // workgroups update every task themselves (bit-identical) and the Gibbs kernel leaves
  unsigned long long* grole;   // [RB][16] (one 128-B line per chain block)
  unsigned* gfb;         // chain-block launches that fell back, since create
  unsigned gep, gpat;    // this launch's epoch (the host counts gsep launches), patience
  int ctiles;            // nmc_k_sweep, the control wave in the tile queue (NMC_CTL_TILES):
                         // 0 never, 1 only while the other waves have more than a round of
                         // entries left (default), 2 like every other wave
  int gtiles;            // nmc_k_sweep, the Gibbs wave after its task (NMC_GIBBS_TILES): 0 no
                         // tiles, 1 as ctiles 1 (default)
  int rows_lds;          // 1: each workgroup stages its group's rows in LDS once per launch
  int tile;              // target rows per likelihood tile (nmc_tiles)
  unsigned* cnt;         // [CB][P][32] publish counters (persistent partial): zeroed at create,
                         // then they keep counting across launches (targets offset by pbase);
                         // reset only before pbase would overflow (nestmc.hip nmc_run)
  unsigned* tmo;         // timeout word: pinned host memory, mapped (host reads it directly)
  // variates of iterations [vbase, vbase + vcap): filled by nmc_k_fill
  double* vzl;           // [t][P][G][C][2] {proposal normal, log accept uniform}
  // zin: the step's {z, log u} are drawn inside the step kernel (jobs in the step's tile
  // queue) and nmc_k_fill is not launched (nmc_k_sweep: every variate, NMC_ZIN=1; nmc_k_run:
  // build option NMC_ZIN_BUILD=1 only, the fill still writes vh); 0: nmc_k_fill writes vzl
  // (+ vh) and the control wave DMAs each step's pair into LDS
  int zin;
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
  // Resident launch (nmc_k_run<..., RES = true>; nestmc.hip nmc_set_resident): one launch
  // serves consecutive nmc_run calls of a sampling loop.  At the end of a call every
  // workgroup completes its results as a launch does (the last Gibbs tasks, sample rows),
  // counts itself done and waits for the host's next command; workgroup 0 alone reads the
  // command word in pinned host memory and relays it (rsync) to the others, so all take the
  // same decision -- a new end, or the park after ridle ticks of s_memrealtime (100 MHz)
  // without one.  The groups' rows and the chain state stay in LDS between calls; the state
  // goes to HBM when the launch parks.
  unsigned long long* rcmd;   // pinned host, mapped: (end << 32) | seq; end 0xffffffff = park
  unsigned* rsync;       // device, zeroed per launch: the relay (end << 32) | seq, one copy
                         // per XCD line (NMC_RSYNC_REL + 32 k), the done count (NMC_RSYNC_CNT)
                         // and the calls' start / loop-end clock maxima (NMC_RSYNC_MAX, u64)
  unsigned* rack;        // pinned host: [0] last seq taken, [1] 0x80000000 | seq when parked,
                         // [2], [3] s_memrealtime when it was taken (lo, hi)
  unsigned* rdone;       // pinned host, written by the last workgroup done: {seq done, 0, then
                         // the s_memrealtime (lo, hi) of: done, the latest loop end, the
                         // latest start of the call}
  unsigned rseq;         // the latest seq the host issued before this launch
  unsigned ridle;        // idle ticks before workgroup 0 parks the launch
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
// tile k of the step (t, p), workgroup 0, first 8 steps of a launch: start/end clock
// and the wave that ran it, stamps[512 + ((step * 16 + k) * 4 + {0, 1, 2})]
#define NMC_TILE_STAMP(k, e)                                                              \
  do {                                                                                    \
    const int si_ = (t - i0) * P + p;                                                     \
    if (d.stamps && blockIdx.x == 0 && si_ < 8 && (k) < 16 && lane == 0) {               \
      d.stamps[512 + (si_ * 16 + (k)) * 4 + (e)] = __builtin_amdgcn_s_memtime();         \
      if (e) d.stamps[512 + (si_ * 16 + (k)) * 4 + 2] = (unsigned long long)w;           \
    }                                                                                     \
  } while (0)
// wave w of workgroup 0 arriving at barrier A of step si (< 8): stamps[512 + (si * 16 + w) * 4 + 3]
#define NMC_ARRIVE_STAMP(si)                                                              \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) < 8 && w < 16 && lane == 0)                   \
      d.stamps[512 + ((si) * 16 + w) * 4 + 3] = __builtin_amdgcn_s_memtime();              \
  } while (0)
// wave w of workgroup 0 at step si (< 8): stamps[1024 + 4 * 4096 + (si * 16 + w) * 4 + k],
// k = 0 step top, 1 before the first take, 2 first take resolved
#define NMC_RS_STAMP(si, k)                                                               \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) < 8 && w < 16 && lane == 0)                   \
      d.stamps[1024 + 4 * 4096 + ((si) * 16 + w) * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// the control wave of workgroup 0 at step si: stamps[512 + (si * 16 + 12 + k) * 4 + 3],
// k = 0 barrier A passed, 1 decided, 2 barrier B passed (W <= 12)
#define NMC_CTL_STAMP(si, k)                                                              \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) < 8 && w == 0 && lane == 0)                   \
      d.stamps[512 + ((si) * 16 + 12 + (k)) * 4 + 3] = __builtin_amdgcn_s_memtime();       \
  } while (0)
// every workgroup b: stamps[1024 + b * 4 + {entry, prologue done, loop done, exit}],
// s_memrealtime (100 MHz, one clock for the whole chip; tools/launchtl.py)
#define NMC_RUN_SL(slot)                                                                  \
  do {                                                                                    \
    if (d.stamps && threadIdx.x == 0)                                                     \
      d.stamps[1024 + (size_t)blockIdx.x * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define NMC_RUN_SL(slot) do {} while (0)
#define NMC_TILE_STAMP(k, e) do {} while (0)
#define NMC_ARRIVE_STAMP(si) do {} while (0)
#define NMC_RS_STAMP(si, k) do {} while (0)
#define NMC_CTL_STAMP(si, k) do {} while (0)
#define NMC_STAMP_CMP(t, slot) do {} while (0)
#define NMC_STAMP_AUX(t, slot) do {} while (0)
#define NMC_STAMP(t, slot) do {} while (0)
#define NMC_STAMP_AT(k, slot) do {} while (0)
#endif

// Diagnostic build only (make cstamps -> libnestmc_cst.so, never shipped): shader clock of
// workgroup 0's waves at the step loop's phase points, steps 0..15 of a launch:
// stamps[step * 32 + slot], slot = w (wave w arrives at barrier A), 8 (barrier A passed,
// control), 9 (decided), 10 (barrier B passed), 16 + w (wave w's first tile starts); wave 2:
// 11 (barrier B passed, the step before), 12 (the step's likelihood entered), 13 (proposal
// prepared); control: 14 (slot sums done), 15 (log-likelihood finished).  Every
// lane of the wave stores the same value (no lane-divergent store: the kernel's laundered
// argument pointer stays scalar).
#ifdef NMC_CSTAMPS
#define NMC_CS(si, slot)                                                                  \
  do {                                                                                    \
    if (d.stamps && blockIdx.x == 0 && (si) >= 0 && (si) < 16)                            \
      d.stamps[(si) * 32 + (slot)] = __builtin_amdgcn_s_memtime();                        \
  } while (0)
#else
#define NMC_CS(si, slot) do {} while (0)
#endif

// The chain of this lane in step-kernel chain block cb (64 chains per workgroup, one per
// lane), and whether the lane's chain exists.
__device__ __forceinline__ int nmc_lane_chain(const Dev&, int cb, int lane) {
  return cb * 64 + lane;
}
__device__ __forceinline__ bool nmc_lane_owns(const Dev& d, int c, int) { return c < d.C; }

// Both halves' values of v in every lane (v_permlane32_swap, gfx950): lo = lanes 0-31's
// value of the lane's pair, hi = lanes 32-63's.
struct nmc_pair2 { double lo, hi; };
__device__ __forceinline__ nmc_pair2 nmc_halves(double v) {
  const unsigned l = (unsigned)__double2loint(v), h = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(h, h, false, false);
  nmc_pair2 r;
  r.lo = __hiloint2double((int)b[0], (int)a[0]);
  r.hi = __hiloint2double((int)b[1], (int)a[1]);
  return r;
}

enum { NMC_RUN_HYPER_LOAD = 1 };
template <bool B> struct nmc_bool_c { static constexpr bool value = B; };
// Dev.rsync word offsets (u32): relay lines, done counter, clock maxima; 512 words in all
enum { NMC_RSYNC_REL = 0, NMC_RSYNC_CNT = 256, NMC_RSYNC_MAX = 288, NMC_RSYNC_WORDS = 512 };
// Largest step-kernel workgroup (build option): 512 threads = 8 waves, 256 VGPRs per lane;
// 768 = 12 waves (three per SIMD) caps the kernel at 168 VGPRs.
#ifndef NMC_RUN_THREADS
#define NMC_RUN_THREADS 512
#endif
#ifndef NMC_GIBBS_TILES
#define NMC_GIBBS_TILES 0
#endif
// nmc_k_run: the control wave takes its likelihood tiles at priority 0 (1), or keeps its
// priority 3 throughout (0)
#ifndef NMC_CTL_TILE_PRIO
#define NMC_CTL_TILE_PRIO 1
#endif
#ifndef NMC_TILE_TAPER
#define NMC_TILE_TAPER 0
#endif
// All-wave Gibbs modes (SYNC, LAUNCH): update every parameter after iteration t-1 at
// step 0 of t (1), or parameter p at step (t, p) (0: waits for a publication one step old,
// but runs two updates per iteration; measured 53.8-53.9 against 51.8-52.2 us/iter at the
// cfg-4 shard, profiles/r03j_ab_allp.json)
#ifndef NMC_HYPER_ALLP
#define NMC_HYPER_ALLP 1
#endif
// Likelihood tiles per group (nmc_tiles) = partial-sum slots per accumulator.
#ifndef NMC_NSLOT_N
#define NMC_NSLOT_N 16
#endif
enum { NMC_NSLOT = NMC_NSLOT_N };
enum { NMC_SPIN_LIMIT = 1 << 22 };
// diagnostic stamps buffer (make stamps): 1024 phase / tile words + 4 per workgroup
enum { NMC_STAMP_WORDS = 1024 + 4 * 4096 + 512 };
// CU count the row split is sized for (a full MI355X), whatever the device reports
enum { NMC_SPLIT_CU_BASIS = 256 };

// Offset of the hyper-parameter slot holding the state after iteration t ([2][P][C]:
// slot t & 1, like the values vb[t & 1]); a launch reads one slot and writes the other.
__device__ __forceinline__ size_t nmc_hslot(const Dev& d, int t) {
  return (size_t)(t & 1) * d.P * d.C;
}

__device__ __forceinline__ int nmc_record_row(const Dev& d, int iter) {
  if (iter < d.burn) return -1;
  if (d.thin == 1) {   // (every post-burn iteration: no integer divisions on the step's path)
    const int row = iter - d.burn;
    return row < d.n_rows ? row : -1;
  }
  if ((iter % d.thin) != 0) return -1;
  const int first = ((d.burn + d.thin - 1) / d.thin) * d.thin;
  const int row = (iter - first) / d.thin;
  return row < d.n_rows ? row : -1;
}

// {z, log u} of step (it, p) of group g, chain c (the chain's global id is chain_base +
// c): Philox4x32-10 normal and log of a 53-bit uniform, or the replayed reference
// variates.  nmc_k_fill and nmc_k_run's variate job both call this, so a step's variates
// never depend on which kernel drew them.
enum { NMC_RNG_MODE_REPLAY = 1 };   // (include/nestmc.h NMC_RNG_REPLAY)
#ifndef NMC_ZIN_BUILD
#define NMC_ZIN_BUILD 0
#endif
__device__ __forceinline__ void nmc_step_variate(const Dev& d, int it, int p, int g, int c,
                                                 double& z, double& lu) {
  if (d.rng_mode == NMC_RNG_MODE_REPLAY) {
    const size_t k = (((size_t)it * d.P + p) * d.G + g) * d.C + c;
    z = it < d.replay_n ? d.rz[k] : nmc_nan();
    lu = it < d.replay_n ? log(d.ru[k]) : nmc_nan();
  } else {
    const uint32_t ch = (uint32_t)(d.chain_base + c);
    z = nmc_normal(it, g, p, NMC_PURPOSE_PROPOSAL, ch, d.seed);
    lu = nmc_log_unit(nmc_uniform2(it, g, p, NMC_PURPOSE_ACCEPT, ch, d.seed).a);
  }
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
  int part;    // [NACC][NSLOT]  per-tile likelihood partial sums (unused slots: -0.0)
  int st;      // [5][P]         scale, log prior, n acc, n rej, total acc (control wave)
  int hyp;     // [6][P]         mu, sd, log sd, sigma2, sqrt(sigma2/G), 1/sd of the hyper-prior
  int hval;    // [2][G + 1]     Gibbs payload of two tasks (persistent Gibbs-wave mode)
  int hst;     // [P][nleaf][8 + ntail]  stream sums / tail elements (pairwise sum)
  int hleaf;   // [P][nleaf]     leaf sums
  int zl;      // [2][2]         {z, log u} of this and the next step (LDS-DMA, step parity)
  int hv;      // [2P]           {hyper z, gamma} of the Gibbs update (LDS-DMA)
  int cw;      // [8]            control-wave values across the step barriers
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
  L.st = L.part + nacc * NMC_NSLOT;   // partial slots per accumulator (unused: -0.0)
  L.hyp = L.st + 5 * P;
  L.hval = L.hyp + (partial ? 6 * P : 0);
  L.hst = L.hval + (partial && hlds ? 2 * (G + 1) : 0);   // two payload buffers (+1 DMA pad)
  L.hleaf = L.hst + (partial ? P * nleaf * (8 + ntail) : 0);
  L.zl = L.hleaf + (partial ? P * nleaf : 0);
  L.hv = L.zl + 4;
  L.cw = L.hv + (partial ? 2 * P : 0);
  L.flag = L.cw + 8;    // (NMC_CW_* uses 7 columns)
  L.xchg = L.flag + 1;
  L.rows = L.xchg;
  // (+1 column: the pipelined likelihood loop prefetches one block past a wave's rows)
  L.total = L.rows + (row_doubles > 0 ? (row_doubles + 63) / 64 + 1 : 0);
  return L;
}
enum { NMC_ST_S = 0, NMC_ST_LP, NMC_ST_NA, NMC_ST_NR, NMC_ST_TA };
enum { NMC_HY_MU = 0, NMC_HY_SD, NMC_HY_LSD, NMC_HY_S2, NMC_HY_SDM, NMC_HY_ISD };
// control-wave columns of the LDS carve (cw): LPC/LPP: priors of the step made by the
// Gibbs wave; NAA..TA: counter outcomes of the decided step
enum { NMC_CW_LPC = 0, NMC_CW_LPP, NMC_CW_NAA, NMC_CW_NRA, NMC_CW_NAR, NMC_CW_NRR, NMC_CW_TA };

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
// Write-through store of v to global memory -- what __hip_atomic_store(relaxed, agent scope)
// emits for a global pointer (global_store_dwordx2 ... sc1) -- for an address held in VGPRs
// whose address space the compiler no longer sees: it would emit a flat store, which counts
// in lgkmcnt as well, and the LDS-only step barrier would then wait for its write-through.
__device__ __forceinline__ void nmc_store_wt(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

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
#ifndef NMC_HYPER_NS
#define NMC_HYPER_NS 1   // streams per wave-iteration (2 and 4 measured slower at cfg 4)
#endif
template <int SRC, bool SQ, int NS = NMC_HYPER_NS>
__device__ __forceinline__ void nmc_hyper_streams(const Dev& d, const double* src, int cc,
                                                  double* lds, const nmc_lds_layout& L,
                                                  int ponly = -1) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C, nl = d.nleaf, ncol = 8 + d.ntail;
  const int per = 8 + (d.ntail ? 1 : 0);
  // the streams of every parameter, or of parameter ponly only
  const int sbeg = ponly < 0 ? 0 : ponly * nl * per;
  const int nst = ponly < 0 ? P * nl * per : (ponly + 1) * nl * per;
  // NS streams per wave-iteration, their loads in flight together
  struct Strm {
    int j, pl, p, m, m8;
    const double* xp;
  };
  auto strm = [&](int s) {
    Strm q;
    q.j = s % per;
    q.pl = s / per;   // pl = p * nleaf + leaf
    const int lf = q.pl % nl;
    q.p = q.pl / nl;
    const int a = nl == 1 ? 0 : d.leaf[lf];
    q.m = nl == 1 ? G : d.leaf[lf + 1] - a;
    q.m8 = q.m >= 8 ? q.m - q.m % 8 : 0;
    // element k of the leaf for this lane's chain
    q.xp = SRC == NMC_SRC_LDS ? lds + (size_t)(L.hval + q.p * G + a) * 64 + lane
                              : src + ((size_t)q.p * G + a) * C + cc;
    return q;
  };
  const size_t xs = SRC == NMC_SRC_LDS ? 64 : (size_t)C;
  for (int s0 = sbeg + w; s0 < nst; s0 += W * NS) {
    double t[NS][16];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int s = s0 + k * W;
      const Strm q = strm(s < nst ? s : s0);
      const int cnt = s < nst && q.j < 8 ? q.m8 >> 3 : 0;   // <= 16
#pragma unroll
      for (int u = 0; u < 16; ++u)
        t[k][u] = u < cnt ? nmc_ldv<SRC>(q.xp + (size_t)(q.j + 8 * u) * xs) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int s = s0 + k * W;
      if (s >= nst) continue;
      const Strm q = strm(s);
      double* out = lds + (size_t)(L.hst + q.pl * ncol) * 64 + lane;
      const double mu = SQ ? lds[(L.hyp + NMC_HY_MU * P + q.p) * 64 + lane] : 0.0;
      if (q.j < 8) {
        const int cnt = q.m8 >> 3;
        double r = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (u < cnt) {
            double v = t[k][u];
            if (SQ) {
              v = v - mu;
              v = v * v;
            }
            r = u == 0 ? v : r + v;
          }
        }
        out[q.j * 64] = r;
      } else {
        for (int u = q.m8; u < q.m; ++u) {
          double v = nmc_ldv<SRC>(q.xp + (size_t)u * xs);
          if (SQ) {
            v = v - mu;
            v = v * v;
          }
          out[(8 + u - q.m8) * 64] = v;
        }
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
  const int c = nmc_lane_chain(d, cb, lane);
  const int cc = c < d.C ? c : d.C - 1;
  for (int p = w - w0; p >= 0 && p < d.P; p += nw)
    nmc_dma16(d.vh + (((size_t)(t - d.vbase) * d.P + p) * d.C + cc) * 2,
              lds + L.hv * 64 + p * 128);
}

// ponly >= 0: the update of that parameter alone (the persistent all-wave mode updates
// parameter p at step (t + 1, p), one step after the last publication it needs).
// NS: streams per wave-iteration with their loads in flight together; WT: the global hyper
// state is stored write-through (agent scope: other workgroups read it inside the launch).
template <int SRC, int NS = NMC_HYPER_NS, bool WT = false>
__device__ __forceinline__ void nmc_hyper(const Dev& d, const double* src, int cb, int t,
                                          double* lds, const nmc_lds_layout& L, bool write,
                                          int ponly = -1) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C;
  const int c = nmc_lane_chain(d, cb, lane);
  const int cc = c < C ? c : C - 1;
  const bool own = nmc_lane_owns(d, c, lane);
  const int pb = ponly < 0 ? 0 : ponly, pe = ponly < 0 ? P : ponly + 1;
  nmc_hyper_streams<SRC, false, NS>(d, src, cc, lds, L, ponly);
  __syncthreads();
  for (int p = pb + w; p < pe; p += W) {
    const double tot = nmc_hyper_combine(d, lds, L, p, lane);
    const double sdm = lds[(L.hyp + NMC_HY_SDM * P + p) * 64 + lane];
    const double hz = lds[L.hv * 64 + (p * 64 + lane) * 2];
    lds[(L.hyp + NMC_HY_MU * P + p) * 64 + lane] = tot / G + sdm * hz;   // mu ~ N(mean(x), sqrt(s2/G))
  }
  __syncthreads();
  nmc_hyper_streams<SRC, true, NS>(d, src, cc, lds, L, ponly);
  __syncthreads();
  const int row = write ? nmc_record_row(d, t) : -1;
  for (int p = pb + w; p < pe; p += W) {
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
    if (write && own) {
      const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
      if constexpr (WT) {
        __hip_atomic_store(d.mu + ho, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d.s2 + ho, s2n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d.hsd + ho, sdn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d.hlsd + ho, lsd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        d.mu[ho] = m;
        d.s2[ho] = s2n;
        d.hsd[ho] = sdn;
        d.hlsd[ho] = lsd;
      }
      if (row >= 0) {
        double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
        out[0] = m;
        out[C] = s2n;
      }
    }
  }
  __syncthreads();
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
  target += (unsigned)d.G * d.pbase;   // (counts of the context's earlier launches)
  unsigned* ctr = nmc_counter(d, cb, p, lane & 7);
  for (unsigned spins = 0;; ++spins) {
    const unsigned v =
        lane < 8 ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += __builtin_amdgcn_readlane(v, k);
    if (tot >= target) return true;
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
      return false;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// The hyper-ready count of (cb, q) (nmc_k_sweep's Gibbs workgroups, SYNC_OWN) and the
// calling wave's bounded poll of such a count.
__device__ __forceinline__ unsigned* nmc_hrd(const Dev& d, int cb, int q) {
  return d.hrd + ((size_t)cb * d.P + q) * 32;
}
__device__ __forceinline__ bool nmc_poll_count(const Dev& d, const unsigned* ctr,
                                               unsigned target) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v >= target) return true;
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
      return false;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Whole-workgroup wait (thread 0 polls, result broadcast through LDS).
__device__ __forceinline__ bool nmc_wait_published_col(const Dev& d, int cb, int p,
                                                       unsigned target, double* lds, int flagcol) {
  if (threadIdx.x < 64) {
    const bool r = nmc_poll_published(d, cb, p, target);
    if (threadIdx.x == 0) lds[flagcol * 64] = r ? 1.0 : 0.0;
  }
  __syncthreads();
  // keep the payload loads below the poll (no instruction: wavefront scope)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return lds[flagcol * 64] != 0.0;
}
__device__ __forceinline__ bool nmc_wait_published(const Dev& d, int cb, int p, unsigned target,
                                                   double* lds, const nmc_lds_layout& L) {
  return nmc_wait_published_col(d, cb, p, target, lds, L.flag);
}

// ---------------------------------------------------------------------------
// log-likelihood of one group over one row range, chain-on-lane: n rows from p
// (wave-uniform address: scalar loads from global memory, broadcast ds_reads from
// LDS), R rows (~BLK doubles) per block, four accumulator sets to break the
// dependence chain.
// ---------------------------------------------------------------------------
// rows per block of the global-memory / staged row loops: >= 4 rows of narrow rows (the
// scalar-load loop runs ahead in the scalar cache), 4 rows of 5-8 fields (four independent
// per-row chains -- e.g. logistic's exp / log1p -- in flight per lane), fewer for wider rows
// (registers)
__host__ __device__ constexpr int nmc_row_block(int nf) {
  return nf <= 4 ? 16 / nf : (32 / nf >= 4 ? 4 : (32 / nf > 0 ? 32 / nf : 1));
}
template <class Fam>
__device__ __forceinline__ void nmc_ll_rows(const Fam& fam, const typename Fam::Reg& reg,
                                            const double* __restrict__ p, int n,
                                            double (&acc)[Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  constexpr int R = nmc_row_block(NF);
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

// The regression row loop (FamLinreg<2>: rows {x, y}, e = fma(x, b1, b0 - y),
// acc[i & 3] = fma(e, e, acc[i & 3]) for row i of each 8-row block) written by hand:
// two fixed register sets v[104:135] / v[136:167] (below 168, so the step kernel can run
// three waves per SIMD), block b+1's eight broadcast
// ds_read_b128 in flight while block b is consumed (counted lgkmcnt(8)).  The compiler
// does not keep this prefetch (it sinks the reads below the arithmetic and copies the
// register sets); measured at the LDS-broadcast floor, ~5 cycles per row per CU
// (tools/llbench4.hip).  Same operations in the same order as FamLinreg::accumN, so
// the sums are bit-identical to the C++ loop.  nb: even number of 8-row blocks >= 2.
#define NMC_L8(b, off)                                                     \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"         \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+16\n"        \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+32\n"       \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+48\n"      \
  "ds_read_b128 v[" #b "+16:" #b "+19], %[addr] offset:" #off "+64\n"      \
  "ds_read_b128 v[" #b "+20:" #b "+23], %[addr] offset:" #off "+80\n"      \
  "ds_read_b128 v[" #b "+24:" #b "+27], %[addr] offset:" #off "+96\n"      \
  "ds_read_b128 v[" #b "+28:" #b "+31], %[addr] offset:" #off "+112\n"
#define NMC_E(b, k)                                                                  \
  "v_fma_f64 v[" #b "+" #k ":" #b "+" #k "+1], v[" #b "+" #k ":" #b "+" #k "+1], %[b1], v[" #b \
  "+" #k "+2:" #b "+" #k "+3]\n"
#define NMC_D(b, k)                                                                  \
  "v_add_f64 v[" #b "+" #k "+2:" #b "+" #k "+3], %[b0], -v[" #b "+" #k "+2:" #b "+" #k "+3]\n"
#define NMC_S(b, k, a) \
  "v_fma_f64 %[" #a "], v[" #b "+" #k ":" #b "+" #k "+1], v[" #b "+" #k ":" #b "+" #k "+1], %[" #a "]\n"
#define NMC_B8(b)                                                                       \
  NMC_D(b, 0) NMC_D(b, 4) NMC_D(b, 8) NMC_D(b, 12) NMC_D(b, 16) NMC_D(b, 20) NMC_D(b, 24)  \
  NMC_D(b, 28) NMC_E(b, 0) NMC_E(b, 4) NMC_E(b, 8) NMC_E(b, 12) NMC_E(b, 16) NMC_E(b, 20)  \
  NMC_E(b, 24) NMC_E(b, 28) NMC_S(b, 0, a0) NMC_S(b, 4, a1) NMC_S(b, 8, a2)               \
  NMC_S(b, 12, a3) NMC_S(b, 16, a0) NMC_S(b, 20, a1) NMC_S(b, 24, a2) NMC_S(b, 28, a3)
typedef __attribute__((address_space(3))) const double* nmc_lds_cptr;
__device__ __forceinline__ void nmc_rows_lds_linreg2(const double* p, int nb, double b0,
                                                     double b1, double& a0, double& a1,
                                                     double& a2, double& a3) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nb;
  asm volatile(
      NMC_L8(104, 0)
      "L_nmc_rows_%=:\n"
      NMC_L8(136, 128)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_B8(104)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_nmc_last_%=\n"
      NMC_L8(104, 0)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_B8(136)
      "s_branch L_nmc_rows_%=\n"
      "L_nmc_last_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_B8(136)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2),
        [a3] "+v"(a3)
      : [b0] "v"(b0), [b1] "v"(b1)
      : "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114",
        "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125",
        "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136",
        "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147",
        "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158",
        "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "scc", "memory");
}

// The paired-chain form of the same loop (NMC_ROWS_PAIRED): lanes 0-31 read row 2m and
// lanes 32-63 row 2m+1 of every row pair m, and each lane evaluates its row for TWO
// chains -- its own and its partner lane's (lane ^ 32) -- so one ds_read_b128 feeds 128
// (chain, row) terms instead of 64: half the LDS instructions for the same fp64 work.
// An 8-row block is four reads (rows v[b:b+15], residual temporaries v[t:t+7]); row pair
// m feeds the own chain's u0/u1 and the partner's w0/w1 (m even / odd).  In half h those
// are the full loop's a[h] / a[2 + h] of the respective chain, with the same rows in the
// same order, and nmc_ll_rows_lds<Fam, true> reassembles them (one lane swap), so the
// sums are bit-identical to the broadcast loop.  p: this half's first row (tile start +
// h rows); nb: even number of 8-row blocks >= 2.
#define NMC_P4(b, off)                                                     \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"         \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+32\n"        \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+64\n"       \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+96\n"
// partner residual seed c0 - y into t, own b0 - y in place of y, then both fmas with x
#define NMC_PDX(b, t, k4, k2) \
  "v_add_f64 v[" #t "+" #k2 ":" #t "+" #k2 "+1], %[c0], -v[" #b "+" #k4 "+2:" #b "+" #k4 "+3]\n"
#define NMC_PDO(b, k4) \
  "v_add_f64 v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], %[b0], -v[" #b "+" #k4 "+2:" #b "+" #k4 "+3]\n"
#define NMC_PEO(b, k4)                                                                      \
  "v_fma_f64 v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], v[" #b "+" #k4 ":" #b "+" #k4 "+1], %[b1], v[" \
  #b "+" #k4 "+2:" #b "+" #k4 "+3]\n"
#define NMC_PEX(b, t, k4, k2)                                                               \
  "v_fma_f64 v[" #t "+" #k2 ":" #t "+" #k2 "+1], v[" #b "+" #k4 ":" #b "+" #k4 "+1], %[c1], v[" \
  #t "+" #k2 ":" #t "+" #k2 "+1]\n"
#define NMC_PSO(b, k4, a) \
  "v_fma_f64 %[" #a "], v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], %[" #a "]\n"
#define NMC_PSX(t, k2, a) \
  "v_fma_f64 %[" #a "], v[" #t "+" #k2 ":" #t "+" #k2 "+1], v[" #t "+" #k2 ":" #t "+" #k2 "+1], %[" #a "]\n"
#define NMC_PB(b, t)                                                                        \
  NMC_PDX(b, t, 0, 0) NMC_PDX(b, t, 4, 2) NMC_PDX(b, t, 8, 4) NMC_PDX(b, t, 12, 6)           \
  NMC_PDO(b, 0) NMC_PDO(b, 4) NMC_PDO(b, 8) NMC_PDO(b, 12)                                   \
  NMC_PEO(b, 0) NMC_PEO(b, 4) NMC_PEO(b, 8) NMC_PEO(b, 12)                                   \
  NMC_PEX(b, t, 0, 0) NMC_PEX(b, t, 4, 2) NMC_PEX(b, t, 8, 4) NMC_PEX(b, t, 12, 6)           \
  NMC_PSO(b, 0, u0) NMC_PSX(t, 0, w0) NMC_PSO(b, 4, u1) NMC_PSX(t, 2, w1)                   \
  NMC_PSO(b, 8, u0) NMC_PSX(t, 4, w0) NMC_PSO(b, 12, u1) NMC_PSX(t, 6, w1)
__device__ __forceinline__ void nmc_rows_lds_linreg2_paired(const double* p, int nb, double b0,
                                                            double b1, double c0, double c1,
                                                            double& u0, double& u1, double& w0,
                                                            double& w1) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nb;
  asm volatile(
      NMC_P4(120, 0)
      "L_nmc_prows_%=:\n"
      NMC_P4(144, 128)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_PB(120, 136)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_nmc_plast_%=\n"
      NMC_P4(120, 0)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_PB(144, 160)
      "s_branch L_nmc_prows_%=\n"
      "L_nmc_plast_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_PB(144, 160)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0),
        [w1] "+v"(w1)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130",
        "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141",
        "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152",
        "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163",
        "v164", "v165", "v166", "v167", "scc", "memory");
}

// The quad-chain form (Dev.quad, the default for {x, y} rows): a wave's four quarters (rows
// of 16 lanes) read rows 4m+q of every 16-row block, q = the lane's quarter, and every lane
// evaluates its row for FOUR chains -- those of lanes (lane & 15) + 16j, j = 0..3, the same
// position in each quarter -- so one ds_read_b128 feeds 256 (chain, row) terms: a quarter
// of the broadcast loop's LDS reads and half the paired loop's, and 48 fp64 instructions
// per four reads, which keeps one wave's issue off the LDS latency.  Chain slot j's
// accumulator a[j] in quarter q sums rows = q (mod 4) in row order: exactly the broadcast
// loop's a[q] of chain (lane & 15) + 16j (its 8-row blocks put row i into a[i & 3]), so a
// 4 x 4 transpose across the quarters (nmc_transpose4) hands every lane its own chain's
// a[0..3] and the sums are bit-identical to the broadcast and paired loops.
// Registers: row sets v[120:135] / v[136:151] (block b+1's four reads in flight while block
// b is consumed), residual temporaries v[152:167] -- the paired loop's range, so the kernel's
// register budget is unchanged.  p: this quarter's first row (tile start + q rows);
// nb: 16-row blocks >= 1, any count.
#define NMC_Q4(b, off)                                                     \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"         \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+64\n"        \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+128\n"      \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+192\n"
// chain slot j of a row (x at v[xr], y at v[yr]) into temporary t: t = c_j - y, then
// t = fma(x, d_j, t), then a_j = fma(t, t, a_j) -- FamLinreg::accum's operations
#define NMC_QD(t, yr, j) "v_add_f64 v[" #t ":" #t "+1], %[c" #j "], -v[" #yr ":" #yr "+1]\n"
#define NMC_QE(t, xr, j) \
  "v_fma_f64 v[" #t ":" #t "+1], v[" #xr ":" #xr "+1], %[d" #j "], v[" #t ":" #t "+1]\n"
#define NMC_QS(t, j) "v_fma_f64 %[a" #j "], v[" #t ":" #t "+1], v[" #t ":" #t "+1], %[a" #j "]\n"
// two rows (x0/y0, then x1/y1) for the four chain slots: 8 adds, 8 fmas, 8 accumulations
// (slot j gets row x0 before row x1, the row order)
#define NMC_QH(x0, y0, x1, y1)                                                               \
  NMC_QD(152, y0, 0) NMC_QD(154, y0, 1) NMC_QD(156, y0, 2) NMC_QD(158, y0, 3)                \
  NMC_QD(160, y1, 0) NMC_QD(162, y1, 1) NMC_QD(164, y1, 2) NMC_QD(166, y1, 3)                \
  NMC_QE(152, x0, 0) NMC_QE(154, x0, 1) NMC_QE(156, x0, 2) NMC_QE(158, x0, 3)                \
  NMC_QE(160, x1, 0) NMC_QE(162, x1, 1) NMC_QE(164, x1, 2) NMC_QE(166, x1, 3)                \
  NMC_QS(152, 0) NMC_QS(154, 1) NMC_QS(156, 2) NMC_QS(158, 3)                                \
  NMC_QS(160, 0) NMC_QS(162, 1) NMC_QS(164, 2) NMC_QS(166, 3)
// a 16-row block from register set A (v[120:135]) / B (v[136:151]): its rows 4m+q, m = 0..3
#define NMC_QBA NMC_QH(120, 122, 124, 126) NMC_QH(128, 130, 132, 134)
#define NMC_QBB NMC_QH(136, 138, 140, 142) NMC_QH(144, 146, 148, 150)
__device__ __forceinline__ void nmc_rows_lds_linreg2_quad(const double* p, int nb,
                                                          const double (&c)[4],
                                                          const double (&dd)[4],
                                                          double (&a)[4]) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nb;
  asm volatile(
      NMC_Q4(120, 0)
      "L_nmc_q_%=:\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_nmc_qla_%=\n"
      NMC_Q4(136, 256)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_QBA
      "v_add_u32 %[addr], 0x200, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_nmc_qlb_%=\n"
      NMC_Q4(120, 0)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_QBB
      "s_branch L_nmc_q_%=\n"
      "L_nmc_qla_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QBA
      "s_branch L_nmc_qend_%=\n"
      "L_nmc_qlb_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QBB
      "L_nmc_qend_%=:\n"
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]),
        [a3] "+v"(a[3])
      : [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [d0] "v"(dd[0]),
        [d1] "v"(dd[1]), [d2] "v"(dd[2]), [d3] "v"(dd[3])
      : "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130",
        "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141",
        "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152",
        "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163",
        "v164", "v165", "v166", "v167", "scc", "memory");
}

// v of the four lanes (lane & 15) + 16j, j = 0..3 (the lane's position in each quarter):
// v_permlane16_swap exchanges odd rows of its first operand with even rows of its second
// (rows of 16 lanes), v_permlane32_swap the upper half of the first with the lower half of
// the second (gfx950); swapping a value with itself yields its row pair / half pair
__device__ __forceinline__ void nmc_quarters(double v, double (&o)[4]) {
  const unsigned l = (unsigned)__double2loint(v), h = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(l, l, false, false);   // [0]: row 2k, [1]: 2k+1
  const auto b = __builtin_amdgcn_permlane16_swap(h, h, false, false);
  const nmc_pair2 ev = nmc_halves(__hiloint2double((int)b[0], (int)a[0]));   // rows 0, 2
  const nmc_pair2 od = nmc_halves(__hiloint2double((int)b[1], (int)a[1]));   // rows 1, 3
  o[0] = ev.lo;
  o[1] = od.lo;
  o[2] = ev.hi;
  o[3] = od.hi;
}
template <bool R16>
__device__ __forceinline__ void nmc_swap_rows(double& x, double& y) {
  const unsigned xl = (unsigned)__double2loint(x), xh = (unsigned)__double2hiint(x);
  const unsigned yl = (unsigned)__double2loint(y), yh = (unsigned)__double2hiint(y);
  const auto l = R16 ? __builtin_amdgcn_permlane16_swap(xl, yl, false, false)
                     : __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
  const auto h = R16 ? __builtin_amdgcn_permlane16_swap(xh, yh, false, false)
                     : __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
  x = __hiloint2double((int)h[0], (int)l[0]);
  y = __hiloint2double((int)h[1], (int)l[1]);
}
// a[j] of quarter q -> a[q] of quarter j (4 x 4 transpose over the quarters): half swaps of
// (a0, a2), (a1, a3), then row swaps of (a0, a1), (a2, a3)
__device__ __forceinline__ void nmc_transpose4(double (&a)[4]) {
  nmc_swap_rows<false>(a[0], a[2]);
  nmc_swap_rows<false>(a[1], a[3]);
  nmc_swap_rows<true>(a[0], a[1]);
  nmc_swap_rows<true>(a[2], a[3]);
}

// The same over rows staged in LDS: blocks of R rows read with wave-uniform
// (broadcast) ds_reads; block b+1 is requested before block b is consumed (LDS
// returns in order, so the wait covers only block b).
#ifndef NMC_LDS_ROW_DOUBLES
#define NMC_LDS_ROW_DOUBLES 16   // doubles per software-pipelined LDS block (8 regression rows)
#endif
// PAIRED (NMC_ROWS_PAIRED): the R-row blocks are split by row parity between the two
// lane halves and every lane evaluates its rows for its own chain (reg) and its partner
// lane's (preg); one lane swap hands each chain the other parity's accumulators, then
// the tail rows are added in order per chain -- bit-identical to PAIRED == false.
template <class Fam>
constexpr bool nmc_paired_rows_ok() {
  constexpr int NF = Fam::NFIELDS;
  constexpr int BD = NF <= 2 ? 16 : 8;
  constexpr int R = (BD / NF) > 0 ? (BD / NF) : 1;
  return R % 2 == 0;
}
// SAME (half layout): lanes l and l + 32 hold the same chain -- each evaluates its row
// parity for that chain only, and the partner's own accumulators are this chain's other
// parity (no partner evaluation).
template <class Fam, bool PAIRED = false, bool SAME = false>
__device__ __forceinline__ void nmc_ll_rows_lds(const Fam& fam, const typename Fam::Reg& reg,
                                                const double* __restrict__ p, int n,
                                                double (&acc)[Fam::NACC],
                                                const typename Fam::Reg* preg = nullptr) {
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
  // two register sets A/B over an even number of R-row blocks: block b+1's reads are
  // issued before block b is consumed, pinned by scheduling barriers (left alone the
  // compiler sinks the reads below the arithmetic and every block pays the full LDS
  // latency).  No condition inside the loop (a conditional load costs register
  // copies): the last prefetch reads one block past the range, which the LDS row
  // area is padded for (nmc_lds) and which is never consumed.
  const int nb2 = (n / R) & ~1;
  if constexpr (PAIRED) {
    static_assert(R % 2 == 0, "the paired split needs row pairs in every block");
    constexpr int RH = R / 2;
    const int h = (threadIdx.x >> 5) & 1;
    const double* ph = p + (size_t)h * NF;   // row 2m + h of pair m
    double u[2][Fam::NACC], v[2][Fam::NACC];   // own chain / partner chain, m even / odd
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int k = 0; k < Fam::NACC; ++k) u[s][k] = v[s][k] = 0.0;
    if constexpr (Fam::ASM_ROWS && !SAME) {
      static_assert(R == 8 && NF == 2, "the asm row loop is the 8-row {x, y} block");
      if (nb2 > 0)
        nmc_rows_lds_linreg2_paired(ph, nb2, reg.b0, reg.b[0], preg->b0, preg->b[0], u[0][0],
                                    u[1][0], v[0][0], v[1][0]);
    } else if (nb2 > 0) {
      double A[RH * NF], B[RH * NF];
#pragma unroll
      for (int m = 0; m < RH; ++m)
#pragma unroll
        for (int f = 0; f < NF; ++f) A[m * NF + f] = ph[(size_t)2 * m * NF + f];
      for (int b = 0; b < nb2; b += 2) {
        const double* q = ph + (size_t)b * (R * NF);
#pragma unroll
        for (int m = 0; m < RH; ++m)
#pragma unroll
          for (int f = 0; f < NF; ++f) B[m * NF + f] = q[R * NF + (size_t)2 * m * NF + f];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < RH; ++m) {
          fam.accum(reg, A + m * NF, u[m & 1]);
          if constexpr (!SAME) fam.accum(*preg, A + m * NF, v[m & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < RH; ++m)
#pragma unroll
          for (int f = 0; f < NF; ++f) A[m * NF + f] = q[2 * R * NF + (size_t)2 * m * NF + f];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < RH; ++m) {
          fam.accum(reg, B + m * NF, u[m & 1]);
          if constexpr (!SAME) fam.accum(*preg, B + m * NF, v[m & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // own chain: a[2k + h] = u[k]; a[2k + 1 - h] = the partner lane's v[k] (the partner's
    // partner chain is this lane's chain)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) {
      // (SAME: the other parity of this chain is the partner lane's own accumulators)
      const nmc_pair2 e = nmc_halves(SAME ? u[0][k] : v[0][k]);
      const nmc_pair2 o = nmc_halves(SAME ? u[1][k] : v[1][k]);
      const double p0 = h ? e.lo : e.hi, p1 = h ? o.lo : o.hi;
      a[0][k] = h ? p0 : u[0][k];
      a[1][k] = h ? u[0][k] : p0;
      a[2][k] = h ? p1 : u[1][k];
      a[3][k] = h ? u[1][k] : p1;
    }
  } else if constexpr (Fam::ASM_ROWS) {
    static_assert(R == 8 && NF == 2, "the asm row loop is the 8-row {x, y} block");
    if (nb2 > 0) nmc_rows_lds_linreg2(p, nb2, reg.b0, reg.b[0], a[0][0], a[1][0], a[2][0], a[3][0]);
  } else if (nb2 > 0) {
    double A[R * NF], B[R * NF];
#pragma unroll
    for (int j = 0; j < R * NF; ++j) A[j] = p[j];
    for (int b = 0; b < nb2; b += 2) {
      const double* q = p + (size_t)b * (R * NF);
#pragma unroll
      for (int j = 0; j < R * NF; ++j) B[j] = q[R * NF + j];
      __builtin_amdgcn_sched_barrier(0);
      fam.template accumN<R>(reg, A, a);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < R * NF; ++j) A[j] = q[2 * R * NF + j];
      __builtin_amdgcn_sched_barrier(0);
      fam.template accumN<R>(reg, B, a);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the remaining (< 2R) rows into a[0], in order; their reads are issued in batches of
  // TB rows (one LDS round trip per batch, not per row)
  constexpr int TB = (16 / NF) > 0 ? (16 / NF) : 1;
  for (int r0 = nb2 * R; r0 < n; r0 += TB) {
    double tv[TB * NF];
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int rr = r0 + i < n ? r0 + i : n - 1;
#pragma unroll
      for (int f = 0; f < NF; ++f) tv[i * NF + f] = p[(size_t)rr * NF + f];
    }
#pragma unroll
    for (int i = 0; i < TB; ++i)
      if (r0 + i < n) fam.accum(reg, tv + i * NF, a[0]);
  }
#pragma unroll
  for (int k = 0; k < Fam::NACC; ++k) acc[k] = (a[0][k] + a[1][k]) + (a[2][k] + a[3][k]);
}

// The quad-chain row loop (nmc_rows_lds_linreg2_quad) over one tile of n rows at p: c / dd
// hold the intercept and slope of the four chains of the lane's quarter position
// (nmc_quarters).  The 16-row blocks cover the broadcast loop's even number of 8-row blocks;
// after the transpose the lane's own chain's four accumulators take the remaining rows in
// order into a[0], as in nmc_ll_rows_lds -- every sum bit-identical to it.
template <class Fam>
__device__ __forceinline__ void nmc_ll_rows_lds_quad(const Fam& fam, const typename Fam::Reg& reg,
                                                     const double* __restrict__ p, int n,
                                                     double (&acc)[Fam::NACC],
                                                     const double (&c)[4], const double (&dd)[4]) {
  static_assert(Fam::ASM_ROWS && Fam::NFIELDS == 2 && Fam::NACC == 1, "{x, y} rows only");
  constexpr int NF = Fam::NFIELDS;
  const int q = (threadIdx.x >> 4) & 3;
  const int nb16 = (n / 8) >> 1;      // = the broadcast loop's (n / 8) & ~1 8-row blocks / 2
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (nb16 > 0) {
    nmc_rows_lds_linreg2_quad(p + (size_t)q * NF, nb16, c, dd, a);
    nmc_transpose4(a);
  }
  double at[1] = {a[0]};
  constexpr int TB = 8;
  for (int r0 = nb16 * 16; r0 < n; r0 += TB) {
    double tv[TB * NF];
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int rr = r0 + i < n ? r0 + i : n - 1;
#pragma unroll
      for (int f = 0; f < NF; ++f) tv[i * NF + f] = p[(size_t)rr * NF + f];
    }
#pragma unroll
    for (int i = 0; i < TB; ++i)
      if (r0 + i < n) fam.accum(reg, tv + i * NF, at);
  }
  acc[0] = (at[0] + a[1]) + (a[2] + a[3]);
}

// ---------------------------------------------------------------------------
// Rows that do not fit LDS (groups over 64 KiB): each wave stages its tile through two
// private LDS buffers of NMC_SR(NF) rows, copied by LDS-DMA (global_load_lds_dwordx4, no
// registers) one chunk ahead of the chunk it computes, so the row fetch -- an L2 / MALL
// round trip per row for the scalar-load loop it replaces -- hides behind the arithmetic.
// Same R-row blocks, accumulators and order as nmc_ll_rows (bit-identical sums).
// ---------------------------------------------------------------------------
// rows per chunk: as many whole row blocks as one 1 KiB DMA instruction carries beside
// 16 B of alignment slack (n_fields <= 64: at least one row)
__host__ __device__ constexpr int nmc_stage_rows(int nf) {
  return (1008 / (nf * 8)) / nmc_row_block(nf) > 0
             ? nmc_row_block(nf) * ((1008 / (nf * 8)) / nmc_row_block(nf))
             : nmc_row_block(nf);
}
// one buffer: the chunk's doubles plus 16 B of alignment slack, in whole 1 KiB DMAs
__host__ __device__ constexpr int nmc_stage_buf(int nf) {
  return ((nmc_stage_rows(nf) * nf + 2) * 8 + 1023) / 1024 * 128;
}
__host__ __device__ constexpr int nmc_stage_doubles(int nf, int W) { return W * 2 * nmc_stage_buf(nf); }

template <class Fam>
__device__ __forceinline__ void nmc_ll_rows_staged(const Fam& fam, const typename Fam::Reg& reg,
                                                   const double* __restrict__ p, int n,
                                                   const double* lim, double* stage,
                                                   double (&acc)[Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  constexpr int R = nmc_row_block(NF);
  constexpr int SR = nmc_stage_rows(NF);
  constexpr int BUF = nmc_stage_buf(NF);        // doubles per buffer
  constexpr int K = BUF / 128;                  // 1 KiB DMA instructions per chunk
  static_assert(K >= 1 && K <= 15, "vmcnt immediate");
  const int lane = threadIdx.x & 63;
  double a[4][Fam::NACC];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k) a[s][k] = 0.0;
  const uintptr_t last = ((uintptr_t)lim - 16) & ~(uintptr_t)15;   // last whole 16 B of the group
  auto issue = [&](int c, double* buf) -> int {   // chunk c -> buf; returns its offset (doubles)
    const uintptr_t src = (uintptr_t)(p + (size_t)c * SR * NF);
    const uintptr_t a16 = src & ~(uintptr_t)15;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the buffer's last reads are done
#pragma unroll
    for (int q = 0; q < K; ++q) {
      uintptr_t g = a16 + (uintptr_t)(q * 64 + lane) * 16;
      g = g > last ? (last > a16 ? last : a16) : g;      // never past the group's rows
      __builtin_amdgcn_global_load_lds((nmc_glb_ptr)g, (nmc_lds_ptr)(buf + q * 128), 16, 0, 0);
    }
    return (int)((src - a16) / 8);
  };
  const int nch = (n + SR - 1) / SR;
  int off_cur = nch > 0 ? issue(0, stage) : 0;
  for (int c = 0; c < nch; ++c) {
    double* cur = stage + (c & 1) * BUF;
    int off_next = 0;
    if (c + 1 < nch) {
      off_next = issue(c + 1, stage + ((c + 1) & 1) * BUF);
      // chunk c has landed once at most chunk c+1's K copies are outstanding (loads return
      // in order); vmcnt field [3:0], expcnt / lgkmcnt left unconstrained
      __builtin_amdgcn_s_waitcnt((K & 15) | (7 << 4) | (15 << 8));
    } else {
      __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
    }
    __builtin_amdgcn_sched_barrier(0);
    const double* q = cur + off_cur;
    const int rows = n - c * SR < SR ? n - c * SR : SR;
    const int nb = rows / R;
    for (int b = 0; b < nb; ++b) {
      double v[R * NF];
#pragma unroll
      for (int j = 0; j < R * NF; ++j) v[j] = q[(size_t)b * (R * NF) + j];
      fam.template accumN<R>(reg, v, a);
    }
    for (int r = nb * R; r < rows; ++r) fam.accum(reg, q + (size_t)r * NF, a[0]);
    __builtin_amdgcn_sched_barrier(0);
    off_cur = off_next;
  }
#pragma unroll
  for (int k = 0; k < Fam::NACC; ++k) acc[k] = (a[0][k] + a[1][k]) + (a[2][k] + a[3][k]);
}

// The tile partials of one sum in a fixed order: tile k into accumulator k % 4, combined
// (a0+a1)+(a2+a3); every LDS read in flight at once (slots past the last tile hold -0.0,
// and x + (-0.0) == x).
typedef double nmc_v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double nmc_sum_slots(const double* pt) {
  double v[NMC_NSLOT];
#if NMC_NSLOT_N == 16
  // the 16 slots (512 B apart) as eight ds_read2st64_b64, all in flight, one wait: left to
  // itself the scheduler splits them over two LDS round trips on the decision's path
  {
    const unsigned a = (unsigned)(uintptr_t)(nmc_lds_cptr)pt;
    nmc_v2d r[8];
    asm volatile(
        "ds_read2st64_b64 %0, %8 offset1:1\n\t"
        "ds_read2st64_b64 %1, %8 offset0:2 offset1:3\n\t"
        "ds_read2st64_b64 %2, %8 offset0:4 offset1:5\n\t"
        "ds_read2st64_b64 %3, %8 offset0:6 offset1:7\n\t"
        "ds_read2st64_b64 %4, %8 offset0:8 offset1:9\n\t"
        "ds_read2st64_b64 %5, %8 offset0:10 offset1:11\n\t"
        "ds_read2st64_b64 %6, %8 offset0:12 offset1:13\n\t"
        "ds_read2st64_b64 %7, %8 offset0:14 offset1:15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
          "=&v"(r[6]),
          "=&v"(r[7])
        : "v"(a)
        : "memory");
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      v[2 * u] = r[u].x;
      v[2 * u + 1] = r[u].y;
    }
  }
#else
#pragma unroll
  for (int u = 0; u < NMC_NSLOT; ++u) v[u] = pt[u * 64];
#endif
  double a4[4];
#pragma unroll
  for (int u = 0; u < NMC_NSLOT; ++u) a4[u & 3] = u < 4 ? v[u] : a4[u & 3] + v[u];
  return (a4[0] + a4[1]) + (a4[2] + a4[3]);
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
// Row tiles of one group (the likelihood partition): NT = min(NSLOT, ceil(n/tile)) tiles
// (tile = 64 rows unless a diagnostics override sets it) of a multiple of 16 rows, so
// every tile but the last runs whole 16-row blocks of the pipelined loop.  Depends only
// on the group's row count: the tile partials -- and so every log-likelihood sum -- are
// the same whichever wave computes a tile, whatever the chain count, launch mode or GPU
// count.  Tile k covers [start(k), start(k) + len(k)).  (A two-length partition -- the
// first half of the tiles carrying 5/8 of the rows -- measured 9.6 against 8.4 us per
// iteration at cfg 3: the late tiles were not the tail.)
struct nmc_tiling {
  int nt;     // tiles
  int h;      // tiles [0, h) have a rows, [h, nt) b rows (the last one the remainder)
  int a, b;
  int n;
  __device__ __forceinline__ int start(int k) const { return k < h ? k * a : h * a + (k - h) * b; }
  __device__ __forceinline__ int len(int k) const {
    const int s = start(k);
    const int e = s + (k < h ? a : b);
    return (e < n ? e : n) - s;
  }
};
__device__ __forceinline__ nmc_tiling nmc_tiles(int n, int tile) {
  nmc_tiling T;
  T.n = n > 0 ? n : 0;
  if (n <= 0) {
    T.nt = 1; T.h = 1; T.a = T.b = 0;
    return T;
  }
  int t = (n + tile - 1) / tile;
  if (t > NMC_NSLOT) t = NMC_NSLOT;
  int per = (n + t - 1) / t;
  per = (per + 15) & ~15;
  T.a = T.b = per;
  T.nt = (n + per - 1) / per;
  T.h = T.nt;
#if NMC_TILE_TAPER   // (A/B build option) the queue's last tiles smaller: h tiles of 5/4 the
                     // size, then tiles of 3/4, so the last waves to finish wait less
  if (T.nt >= 8) {
    const int a = ((per * 5 / 4) + 15) & ~15, b = ((per * 3 / 4) + 15) & ~15;
    const int h = T.nt / 2;
    const int rest = n - h * a;
    if (b > 0 && rest > 0 && h + (rest + b - 1) / b <= NMC_NSLOT) {
      T.a = a; T.b = b; T.h = h; T.nt = h + (rest + b - 1) / b;
    }
  }
#endif
  return T;
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

// The Gibbs update of parameter p after iteration t for this wave's 64 chains, by ONE
// wave, from the LDS copy hval of the chain block's values of p (hv[i * 64]: group i):
// numpy's pairwise sum (8 interleaved streams r_j = x_j + x_{j+8} + ..., combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), the G % 8 tail added in order; G < 8: a
// sequential sum from 0; G <= 128: one numpy leaf) for mean(x) and sum((x - mu)^2)
// (HyperParameter._updateMean :481-487, _updateVar :489-498).  Run beside the
// likelihood tiles: reads in bursts of 4 elements per stream (32 in flight, one LDS
// round trip per burst under the tiles' broadcast traffic).  hz/hx: this lane's hyper variates of
// (t, p).  Writes the LDS hyp columns of p (and, if write, the global slot of t and the
// sample row of t).
__device__ __forceinline__ void nmc_hyper_compute(const Dev& d, int cb, int t, int p, double* lds,
                                                  const nmc_lds_layout& L, bool write, double hz,
                                                  double hx, int hoff) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G, C = d.C;
  const int c = nmc_lane_chain(d, cb, lane);
  const double* hv = lds + (size_t)(L.hval + hoff) * 64 + lane;   // hv[i * 64]: group i of p
  double* hy = lds + L.hyp * 64 + lane;
  const double sdm = sqrt(hy[(NMC_HY_S2 * P + p) * 64] / G);
  const int m8 = G >= 8 ? G - G % 8 : 0;
  const int cnt = m8 >> 3;   // elements per stream, 0..16
  auto pass = [&](bool sq, double mu) -> double {
    double r[8];
#pragma unroll 1
    for (int e0 = 0; e0 < cnt; e0 += 4) {
      double xv[8][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int uu = e0 + u < cnt ? e0 + u : cnt - 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j][u] = hv[(8 * uu + j) * 64];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        double acc = e0 > 0 ? r[j] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (e0 + u < cnt) {
            double x = xv[j][u];
            if (sq) {
              x = x - mu;
              x = x * x;
            }
            acc = e0 + u == 0 ? x : acc + x;
          }
        }
        r[j] = acc;
      }
    }
    double res = cnt ? ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])) : 0.0;
#pragma unroll 1
    for (int i = m8; i < G; ++i) {   // the G % 8 tail, in order (G < 8: from 0)
      double x = hv[i * 64];
      if (sq) {
        x = x - mu;
        x = x * x;
      }
      res += x;
    }
    return res;
  };
  const double tot = pass(false, 0.0);
  const double mu = tot / G + sdm * hz;                        // mu ~ N(mean(x), sqrt(s2/G))
  const double ss = pass(true, mu);
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
  if (write && nmc_lane_owns(d, c, lane)) {
    const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
    // write-through (sc1): nmc_k_sweep's readers poll for them inside the launch
    __hip_atomic_store(d.mu + ho, mu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.s2 + ho, s2n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.hsd + ho, sdn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.hlsd + ho, lsd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int row = nmc_record_row(d, t);
    if (row >= 0) {
      double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
      out[0] = mu;
      out[C] = s2n;
    }
  }
}

// numpy's pairwise sum (the order of nmc_hyper_compute's pass) over x[0..G) held in
// registers, G <= 64: every index is a compile-time constant, the G-dependent parts
// are wave-uniform branches (cnt blocks of 8, the G % 8 tail picked by m8).
__device__ __forceinline__ double nmc_pairwise_reg(const double (&x)[64], int G, bool sq,
                                                   double mu) {
  const int m8 = G >= 8 ? G - G % 8 : 0;
  const int cnt = m8 >> 3;   // 0..8 blocks of 8
  auto tr = [&](double v) {
    if (sq) {
      v = v - mu;
      v = v * v;
    }
    return v;
  };
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = tr(x[j]);
  if (G == 64) {   // eight full blocks, no tail: no selects (the general path below is
                   // if-converted into a v_cndmask per element and block)
#pragma unroll
    for (int u = 1; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + tr(x[8 * u + j]);
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
#pragma unroll
  for (int u = 1; u < 8; ++u)
    if (u < cnt) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + tr(x[8 * u + j]);
    }
  double res = cnt ? ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])) : 0.0;
  double tv[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) tv[k] = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (8 * u == m8) {
#pragma unroll
      for (int k = 0; k < 7; ++k) tv[k] = x[8 * u + k < 64 ? 8 * u + k : 63];
    }
  const int nt = G - m8;   // the G % 8 tail, in order (G < 8: the whole sum from 0)
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if (k < nt) res += tr(tv[k]);
  return res;
}

__device__ __forceinline__ void nmc_hyper_finish(const Dev& d, int cb, int t, int p, double* lds,
                                                 int hyp, bool write, double mu, double ss,
                                                 double hx);

// The Gibbs update of parameter p after iteration t for this wave's 64 chains from the
// chain block's values x[0..G) of p in registers (G <= 64); otherwise identical to
// nmc_hyper_compute (same sums in the same order, same draws, same outputs).
// hyp: the LDS column of the hyper state ([6][P] columns, NMC_HY_*).
__device__ __forceinline__ void nmc_hyper_compute_reg(const Dev& d, int cb, int t, int p,
                                                      double* lds, int hyp, bool write,
                                                      double hz, double hx,
                                                      const double (&x)[64]) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G;
  double* hy = lds + hyp * 64 + lane;
  const double sdm = sqrt(hy[(NMC_HY_S2 * P + p) * 64] / G);
  const double tot = nmc_pairwise_reg(x, G, false, 0.0);
  const double mu = tot / G + sdm * hz;                        // mu ~ N(mean(x), sqrt(s2/G))
  const double ss = nmc_pairwise_reg(x, G, true, mu);
  nmc_hyper_finish(d, cb, t, p, lds, hyp, write, mu, ss, hx);
}

// mu and sum((x - mu)^2) -> sigma2 draw, LDS hyper state, (write) global slot of t and
// the sample row of t (HyperParameter._updateVar :489-498, setPrior :273-282).
__device__ __forceinline__ void nmc_hyper_finish(const Dev& d, int cb, int t, int p, double* lds,
                                                 int hyp, bool write, double mu, double ss,
                                                 double hx) {
  const int lane = threadIdx.x & 63;
  const int P = d.P, G = d.G, C = d.C;
  const int c = nmc_lane_chain(d, cb, lane);
  double* hy = lds + hyp * 64 + lane;
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
  if (write && nmc_lane_owns(d, c, lane)) {
    const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
    // write-through (sc1): nmc_k_sweep's readers poll for them inside the launch
    __hip_atomic_store(d.mu + ho, mu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.s2 + ho, s2n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.hsd + ho, sdn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.hlsd + ho, lsd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int row = nmc_record_row(d, t);
    if (row >= 0) {
      double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
      out[0] = mu;
      out[C] = s2n;
    }
  }
}

// Poll-free half of the register Gibbs hand-off: the chain block's published values of
// parameter q after iteration tq -> x[0..64) (sc1 loads, all in flight at once: one
// global round trip, no LDS traffic beside the likelihood waves' broadcasts; x[G..64)
// read the buffers' 72-group slack or the next parameter and are never summed), and
// the update's variates {hyper z, gamma}.
__device__ __forceinline__ void nmc_hyper_fetch_reg(const Dev& d, int tq, int q, int cc,
                                                    double (&x)[64], double& hz, double& hx) {
  const int G = d.G, C = d.C;
  const double* src = ((tq & 1) ? d.vb1 : d.vb0) + (size_t)q * G * C + cc;
#pragma unroll
  for (int k = 0; k < 64; ++k) x[k] = nmc_ldv<NMC_SRC_SC1>(src + (size_t)k * C);
  const size_t hvi = (((size_t)(tq - d.vbase) * d.P + q) * C + cc) * 2;
  hz = d.vh[hvi];
  hx = d.vh[hvi + 1];
}

// Row split: member m's partial sums of step k -> xbuf (sc1), counted on the unit's
// counter; once all S members of step k have arrived, every member sums the S partials in
// member order (four interleaved streams m & 3, combined (s0+s1)+(s2+s3)) -- identical in
// every member.  A member is at most one step ahead of the slowest (it cannot pass step
// k+1 before all partials of k+1 exist), so two step-parity slots suffice.  Call with
// the whole (control) wave; bounded spin (d.tmo).
template <int NA>
__device__ __forceinline__ void nmc_split_exchange(const Dev& d, int cb, int g, int m, int k,
                                                   double (&acc)[NA]) {
  const int lane = threadIdx.x & 63;
  const int S = d.S;
  const size_t unit = (size_t)cb * d.G + g;
  double* xb = d.xbuf + (((size_t)((k + d.xbase) & 1) * d.RB * d.G + unit) * S) * NA * 64 + lane;
#pragma unroll
  for (int j = 0; j < NA; ++j)
    __hip_atomic_store(xb + ((size_t)m * NA + j) * 64, acc[j], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  nmc_drain_vm();
  unsigned* ctr = d.xcnt + unit * 32;
  if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned target = (unsigned)S * ((unsigned)k + d.xbase + 1u);
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v >= target) break;
    if ((spins & 255) == 255 &&
        __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
      break;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  // keep the partial loads below the poll (no instruction: wavefront scope)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int m0 = 0; m0 < S; m0 += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = m0 + u < S ? __hip_atomic_load(xb + ((size_t)(m0 + u) * NA + j) * 64,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int mm = m0 + u;
        if (mm < S) s4[mm & 3] = mm < 4 ? v[u] : s4[mm & 3] + v[u];
      }
    }
    acc[j] = S >= 4 ? (s4[0] + s4[1]) + (s4[2] + s4[3])
                    : (S == 1 ? s4[0] : (S == 2 ? s4[0] + s4[1] : (s4[0] + s4[1]) + s4[2]));
  }
}

// numpy's pairwise sum over the chain block's G (64 < G <= 256) values of one parameter,
// streamed from global memory (sc1) in chunks of 64: each numpy leaf (<= 128 values, the
// host plan d.leaf) as 8 interleaved streams carried across chunks plus its tail in
// order, the leaves merged in numpy's recursion order (d.merge) -- the order of
// nmc_hyper_compute and the oracle.  src: the parameter's [G][C] values + this chain.
// CH: values per chunk (loads in flight together, 2 * CH VGPRs).
template <int CH = 64>
__device__ __forceinline__ double nmc_pairwise_stream(const Dev& d, const double* src, bool sq,
                                                      double mu) {
  static_assert(CH % 8 == 0 && CH <= 64, "chunks of whole 8-value blocks");
  const int C = d.C, G = d.G, nl = d.nleaf;
  auto tr = [&](double v) {
    if (sq) {
      v = v - mu;
      v = v * v;
    }
    return v;
  };
  double ls[4] = {0.0, 0.0, 0.0, 0.0};
  for (int lf = 0; lf < nl; ++lf) {
    const int a = nl == 1 ? 0 : d.leaf[lf];
    const int m = nl == 1 ? G : d.leaf[lf + 1] - a;
    const int m8 = m >= 8 ? m - m % 8 : 0;
    double r[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int e0 = 0; e0 < m8; e0 += CH) {
      double x[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k)
        x[k] = e0 + k < m8 ? nmc_ldv<NMC_SRC_SC1>(src + (size_t)(a + e0 + k) * C) : 0.0;
#pragma unroll
      for (int k = 0; k < CH; ++k)
        if (e0 + k < m8) r[k & 7] = e0 + k < 8 ? tr(x[k]) : r[k & 7] + tr(x[k]);
    }
    double res = m8 ? ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])) : 0.0;
    for (int e = m8; e < m; ++e) res += tr(nmc_ldv<NMC_SRC_SC1>(src + (size_t)(a + e) * C));
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == lf) ls[i] = res;
  }
  for (int k = 0; k < d.nmerge; ++k) {   // slot A += slot B
    const int A = d.merge[2 * k], B = d.merge[2 * k + 1];
    double vb = ls[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (i == B) vb = ls[i];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == A) ls[i] = ls[i] + vb;
  }
  return ls[0];
}

// SYNC_OWN: the hyper-parameters of task (tq, q) as its Gibbs workgroup stored them (global
// slot of tq, sc1 loads) -> this workgroup's LDS hyper state (nmc_hyper_finish's values).
__device__ __forceinline__ void nmc_hyper_read(const Dev& d, int tq, int q, int cc, double* lds,
                                               int hyp) {
  const int lane = threadIdx.x & 63;
  const int P = d.P;
  const size_t ho = nmc_hslot(d, tq) + (size_t)q * d.C + cc;
  const double mu = nmc_ldv<NMC_SRC_SC1>(d.mu + ho), s2 = nmc_ldv<NMC_SRC_SC1>(d.s2 + ho);
  const double sd = nmc_ldv<NMC_SRC_SC1>(d.hsd + ho), lsd = nmc_ldv<NMC_SRC_SC1>(d.hlsd + ho);
  double* hy = lds + hyp * 64 + lane;
  hy[(NMC_HY_MU * P + q) * 64] = mu;
  hy[(NMC_HY_SD * P + q) * 64] = sd;
  hy[(NMC_HY_LSD * P + q) * 64] = lsd;
  hy[(NMC_HY_S2 * P + q) * 64] = s2;
  hy[(NMC_HY_ISD * P + q) * 64] = 1.0 / sd;
}

// The register Gibbs update of task (tq, q) for this wave's 64 chains (G <= 64): one
// 64-value fetch (nmc_hyper_fetch_reg), then nmc_hyper_compute_reg.
__device__ __forceinline__ void nmc_hyper_update_reg(const Dev& d, int cb, int tq, int q, int cc,
                                                     double* lds, int hyp, bool write) {
  double xv[64], fz, fx;
  nmc_hyper_fetch_reg(d, tq, q, cc, xv, fz, fx);
  nmc_hyper_compute_reg(d, cb, tq, q, lds, hyp, write, fz, fx, xv);
}

// ---------------------------------------------------------------------------
// K_run: iterations [i0, i1) for every (chain, group); grid = CB*G workgroups of
// 64*W threads (W <= 8); dynamic LDS = nmc_lds(...).total columns.
// Wave roles:
//   wave 0            control: proposal priors, Metropolis decision, tuning, state,
//                     sample/trace stores, variate DMA, publishing, and (persistent
//                     payload-in-LDS mode, P >= 2) the Gibbs payload copy;
//   wave 1 (NAUX = 1) Gibbs update (persistent payload-in-LDS mode): the task the
//                     control wave copied at the previous step (P == 1: poll, copy
//                     and update in the same step);
//   every wave        once its own work is done, takes likelihood row tiles from an
//                     LDS counter until none is left, so a wave that shares its SIMD
//                     with a busy control or Gibbs wave simply takes fewer tiles.
// The control wave adds the tile partials in a fixed order (nmc_tiles): the sums do
// not depend on which wave took which tile.
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
       NMC_MODE_SYNC_LDS = 3,    // persistent, the Gibbs wave works on an LDS copy
       NMC_MODE_SYNC_REG = 4,    // persistent, G <= 64: the Gibbs wave fetches the task's
                                 // values straight into registers and updates in one step
       NMC_MODE_SYNC_OWN = 5,    // nmc_k_sweep (G > 128): Gibbs workgroups update each task
       NMC_MODE_HALF = 6 };      // none/complete pooling, 32 chains per workgroup: lanes l
                                 // and l + 32 hold chain l, on the two row parities
// RL: the groups' rows are staged in LDS for the launch (d.rows_lds) -- a template
// parameter so each instance holds only its own row loop (the LDS-DMA staged loop's
// registers raised the rows-in-LDS kernel's pressure: ~5 % of its time at cfg 3)
// The step kernel's Dev argument (the first kernel argument: offset 0 of the kernarg
// segment) read through a pointer laundered at the top of every step: its fields are
// scalar-loaded (s_load, scalar cache) where a step uses them instead of being hoisted out
// of the persistent loop and held in SGPRs for the whole launch -- some 60 fields, which
// spilled 160-600 SGPRs per instance (MI355X: <= 102 SGPRs per wave).
// The step loops' workgroup barrier (nmc_k_run, nmc_k_sweep): LDS traffic only.  __syncthreads() is a workgroup-scope
// release/acquire, which waits for every outstanding global store of the wave (vmcnt(0)):
// the control wave's write-through publish and sample stores, the Gibbs wave's hyper-state
// stores would then sit on the step's critical path.  The step loop shares nothing through
// global memory inside the workgroup (a wave whose LDS-DMA must have landed drains vmcnt
// itself first), so the barrier waits for LDS operations only; the "memory" clobber keeps
// the compiler from moving memory accesses across it.
__device__ __forceinline__ void nmc_step_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// nmc_k_run's step barriers A and B (NMC_RUN_SYNCTHREADS=1: __syncthreads(), the A/B build)
#ifndef NMC_RUN_SYNCTHREADS
#define NMC_RUN_SYNCTHREADS 0
#endif
__device__ __forceinline__ void nmc_run_barrier() {
#if NMC_RUN_SYNCTHREADS
  __syncthreads();
#else
  nmc_step_barrier();
#endif
}

typedef __attribute__((address_space(4))) const Dev* nmc_kdev_ptr;
__device__ __forceinline__ const Dev* nmc_kdev() {
  nmc_kdev_ptr p = (nmc_kdev_ptr)__builtin_amdgcn_kernarg_segment_ptr();
#if !defined(NMC_STAMPS) && !defined(NMC_NO_LAUNDER)
  // (the stamps build's divergent stamp stores make the backend move the laundered pointer
  //  to VGPRs, an illegal copy: diagnostics keep it plain; NMC_NO_LAUNDER: the A/B build)
  asm volatile("" : "+s"(p));
#endif
  return (const Dev*)p;
}

// RES: the resident launch (Dev.rcmd): iterations [i0, i1) are the first call; later calls
// extend the end (res_gate below).
template <class Fam, int MODE, bool RL = true, bool RES = false>
__global__ void __launch_bounds__(NMC_RUN_THREADS)
nmc_k_run(Dev d_arg, Fam fam, const double* __restrict__ obs, int i0, int i1, int flags) {
  (void)d_arg;   // (read through nmc_kdev(): the same bytes)
  const Dev* dP = nmc_kdev();
#define d (*dP)
  constexpr bool PARTIAL = MODE != NMC_MODE_NOPOOL && MODE != NMC_MODE_HALF;
  // half layout: the grid of 64-chain blocks would leave CUs idle (none/complete pooling,
  // RB * G * 2 <= CUs): 32 chains per workgroup, twice the workgroups, each lane pair
  // (l, l + 32) one chain with the paired row loop's two row parities -- the same rows,
  // accumulators and order as the 64-chain layout, so every sum is bit-identical
  constexpr bool HALF = MODE == NMC_MODE_HALF;
  NMC_RUN_SL(0);
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int P = d.P, G = d.G, C = d.C;
  const int b = blockIdx.x;
  const int S = d.S;
  // the two Dev words the step's restart branches on, held for the launch (read after the
  // per-step argument laundering they cost a scalar round trip each before the first tile)
  const bool paired = d.paired;
  const bool quad = d.quad;
  const bool nstatic = d.nstatic;
  const bool ctlprio = NMC_CTL_TILE_PRIO && !(d.noprio & 1);
  const int mb = b % S;                           // row-split member (S == 1: 0)
  // (chain block, group) of unit u = b / S: chain-block-major, or (Dev.xpc > 0, S == 1) dealt
  // so that a chain block's workgroups share xpc XCDs -- blocks b and b + 8 share an XCD
  // (MI355X_MICROARCH.md, XCD placement) -- and its Gibbs payload is fetched into xpc L2s
  // rather than all 8.  Placement only: every (chain block, group) computes the same.
  const int u = b / S, xpc = d.xpc;
  const int g = xpc ? (u >> 3) * xpc + (u & 7) % xpc : u % G;
  const int cb = (xpc ? (u & 7) / xpc : u / G) + d.cb0;
  const int c = HALF ? cb * 32 + (lane & 31) : nmc_lane_chain(d, cb, lane);
  // member 0 writes the outputs (half layout: lanes 0-31)
  const bool live = nmc_lane_owns(d, c, lane) && mb == 0 && (!HALF || lane < 32);
  const bool g0w = g == 0 && mb == 0;   // writes the chain block's hyper-parameters
  const int cc = c < C ? c : C - 1;
  constexpr bool sync = MODE == NMC_MODE_SYNC || MODE == NMC_MODE_SYNC_LDS ||
                        MODE == NMC_MODE_SYNC_REG;
  static_assert(MODE != NMC_MODE_SYNC_OWN, "SYNC_OWN is nmc_k_sweep's mode");
  // Gibbs-wave modes: payload in LDS (two-stage pipeline) or in registers (one stage)
  constexpr bool hr = MODE == NMC_MODE_SYNC_REG;
  constexpr bool hl = MODE == NMC_MODE_SYNC_LDS || hr;
  // the Gibbs wave's task at global step gs is gs - lag; the register mode updates a
  // task two steps after its publication (P >= 2: the hand-off latency -- store drain,
  // counter add, poll -- is behind a whole step) and the priors that need it come from
  // the Gibbs wave when it lands in the step that uses it (P <= 2)
  const int lag = hr && P >= 2 ? 2 : 1;
  int ie = i1;            // end of the current call (RES: moved by the host's commands)
  int gfirst = i0 * P;    // first global step of the current call: the Gibbs tasks of the
                          // steps before it were closed by the launch before / the last gate
  // register mode: the task this workgroup closes at the end of a call ending at iend (-1:
  // none) -- tasks ge-lag .. ge-1, task ge-lag+j by the workgroup of group j
  auto close_of = [&](int iend) {
    const int ge = iend * P, k0 = ge - lag > gfirst ? ge - lag : gfirst;
    return hr && mb == 0 && k0 + g < ge ? k0 + g : -1;
  };
  // rows in LDS for the launch, or every wave's two staging buffers (nmc_ll_rows_staged)
  const int row_doubles = RL ? d.nmax * Fam::NFIELDS
                             : (Fam::NFIELDS <= 4 ? 0 : nmc_stage_doubles(Fam::NFIELDS, blockDim.x >> 6));
  const nmc_lds_layout L =
      nmc_lds(Fam::NACC, P, PARTIAL, d.nleaf, d.ntail, W, G, hl && !hr ? 1 : 0, row_doubles);
  double* th = lds + L.th * 64 + lane;            // th[p * 64]: this lane's chain, parameter p
  double* st = lds + L.st * 64 + lane;            // st[(k * P + p) * 64]
  double* hy = lds + L.hyp * 64 + lane;           // hy[(k * P + p) * 64]
  // tile counters, one per step parity (two 32-bit words in the flag column)
  unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);
  const int ngrp = (int)(d.off[g + 1] - d.off[g]);   // the group's rows (finish)
  int64_t r0;
  int nrow;                                           // this member's rows
  nmc_chunk(d.off[g], d.off[g + 1], mb, S, &r0, &nrow);
  const nmc_tiling TI = nmc_tiles(nrow, d.tile);
  const int nt = TI.nt;
  const double* grows = obs + r0 * Fam::NFIELDS;
  const double* glim = obs + d.off[g + 1] * Fam::NFIELDS;   // end of the group's rows
  const size_t PGC = (size_t)P * G * C;
  const size_t gc = (size_t)g * C + cc;
  const bool ctl = w == 0;
  const bool gw = hl && w == 1;                   // the Gibbs wave
  // latency-bound roles (control, Gibbs) issue ahead of the waves sharing their SIMD
  if (W > 1 && (ctl || gw) && !(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);

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
  const double gcst = fam.gconst((long)ngrp);   // per-group constant of finish_fast
  // the decision's family constants (finish_fast) and publish targets (this lane's value of
  // parameter 0 in vb0 / vb1), held in registers for the launch: read through the per-step
  // laundered argument pointer they are scalar round trips on the decision's critical path,
  // and barrier B's lgkmcnt(0) waits for them
  Fam fh = fam;   // (used for every family call below)
  fh.hold();
  double* pub0 = d.vb0 + gc;
  double* pub1 = d.vb1 + gc;
  asm volatile("" : "+v"(pub0), "+v"(pub1));
  double* lrows = lds + L.rows * 64;
  if constexpr (RL) {   // this group's rows -> LDS, once for the whole launch
    const int nd = nrow * Fam::NFIELDS;
    if (((r0 * Fam::NFIELDS) & 1) == 0) {
      // LDS-DMA in 16-byte pieces (global_load_lds_dwordx4: 1 KiB per wave-instruction, no
      // VGPRs), every piece in flight at once -- one memory round trip instead of one per
      // strided pass; an odd nd copies one double of slack (the carve has a column spare)
      const int npc = (nd + 1) / 2;
      for (int b0 = w * 64; b0 < npc; b0 += W * 64)
        if (b0 + lane < npc) nmc_dma16(grows + 2 * (b0 + lane), lrows + 2 * b0);
      nmc_drain_vm();   // (this wave's pieces have landed before the barrier below)
    } else {
      for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
    }
  }
  auto zl_src = [&](int tn, int pn) -> const double* {
    return d.vzl + ((size_t)(tn - d.vbase) * PGC + (size_t)pn * G * C + gc) * 2;
  };
  // {z, log u} of step (tn, pn) -> LDS slot: LDS-DMA of the variates nmc_k_fill wrote
  auto put_zl = [&](int tn, int pn, int slot) {
    nmc_dma16(zl_src(tn, pn), lds + (L.zl + 2 * slot) * 64);
  };
  // ... or drawn here (d.zin, build option NMC_ZIN_BUILD=1): the calling wave's 64 lanes,
  // one chain each.  Measured slower: with the Philox / Box-Muller / log code inlined
  // into the tile loop the cfg-3 kernel spills twice the SGPRs (955 against 548) and runs
  // 11.7 against 7.5 us/iter (profiles/r03d_*), more than the fill it saves (0.53 us/iter
  // + 7 us per launch) -- so the shipped build keeps the fill.
  auto gen_zl = [&](int tn, int pn, int slot) {
#if NMC_ZIN_BUILD
    double z, lu;
    nmc_step_variate(d, tn, pn, g, cc, z, lu);
    lds[(L.zl + 2 * slot) * 64 + 2 * lane] = z;
    lds[(L.zl + 2 * slot) * 64 + 2 * lane + 1] = lu;
#else
    (void)tn; (void)pn; (void)slot;
#endif
  };
  double* cwv = lds + L.cw * 64 + lane;    // cwv[k * 64]: control-wave values across barriers
  if (ctl) {     // {z, log u} of the first step -> LDS slot of step i0*P
    if (NMC_ZIN_BUILD && d.zin)
      gen_zl(i0, 0, (i0 * P) & 1);
    else
      put_zl(i0, 0, (i0 * P) & 1);
    for (int j = 0; j < Fam::NACC; ++j)   // x + (-0.0) == x: the fixed slot sum
      for (int k = nt; k < NMC_NSLOT; ++k) lds[(L.part + j * NMC_NSLOT + k) * 64 + lane] = -0.0;
    nmc_drain_vm();
    lds[L.flag * 64 + lane] = 0.0;
    // both tile counters start at the static entries: waves 2 .. W-1 begin on entries
    // 0 .. W-3 by rank, without a take (every wave from 2 on runs lik_tiles in every mode)
    if (lane < 2) tcnt[lane] = (unsigned)(nstatic && W > 2 ? W - 2 : 0);
    if (RES && b == 0 && lane == 0) {   // the launch's own call taken now (its GPU span)
      const unsigned long long clk = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_store(d.rack + 2, (unsigned)clk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(d.rack + 3, (unsigned)(clk >> 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      nmc_drain_vm();
      __hip_atomic_store(d.rack, d.rseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  NMC_RUN_SL(1);

  bool ok = true;
  int pub_p = -1;     // control wave: parameter whose sc1 value store awaits its counter add
  int pend_p = -1, pend_t = 0;   // control wave: decided step whose state update is pending
  // Control-wave values, in registers across the step's barriers (the LDS queue is
  // saturated by the likelihood tiles while they are produced): the proposal, current
  // value, log accept uniform and priors of the step, both outcomes of its counters and
  // scale, the group log-likelihood of the current state, and the decided-but-pending
  // step's accept flag, log prior and log-likelihood.
  // (step-local ones are declared inside the step loop, so they are not live across the
  // Gibbs wave's bursts; the counters' outcomes wait in LDS)
  double c_LL = ctl ? d.ll[gc] : 0.0;
  bool q_acc = false;
  double q_plp = 0, q_pll = 0;
  // the rest of a decided step's state update (:369-383, :608-610): counters, log prior,
  // log-likelihood, sample and trace rows
  // its sample / trace stores wait in registers (w_*) until store_pending, which the control
  // wave issues after the step's publication count: the count's vmcnt drain then waits for
  // the publish store alone, not for stores issued just before it
  int w_q = -1, w_t = 0;
  bool w_acc = false;
  double w_v = 0, w_ll = 0;
  auto apply_pending = [&]() {
    const int q = pend_p, tq = pend_t;
    st[(NMC_ST_LP * P + q) * 64] = q_plp;
    st[(NMC_ST_NA * P + q) * 64] = cwv[(q_acc ? NMC_CW_NAA : NMC_CW_NAR) * 64];
    st[(NMC_ST_NR * P + q) * 64] = cwv[(q_acc ? NMC_CW_NRA : NMC_CW_NRR) * 64];
    st[(NMC_ST_TA * P + q) * 64] = cwv[NMC_CW_TA * 64] + (q_acc ? 1.0 : 0.0);
    if (q_acc) c_LL = q_pll;
    w_q = q;
    w_t = tq;
    w_v = th[q * 64];
    w_acc = q_acc;
    w_ll = q_pll;
    pend_p = -1;
  };
  auto store_pending = [&]() {
    if (w_q < 0) return;
    const int q = w_q, tq = w_t;
    if (live) {
      const int row = nmc_record_row(d, tq);
      if (row >= 0) {
        const int col = q * (G + (PARTIAL ? 2 : 0)) + (PARTIAL ? 2 : 0) + g;
        d.samples[((size_t)row * d.cols + col) * C + c] = w_v;
      }
      if (tq < d.trace_n) {
        const size_t it = (((size_t)tq * P + q) * G + g) * C + c;
        d.tflag[it] = w_acc ? 1 : 0;
        d.tllp[it] = w_ll;
      }
    }
    w_q = -1;
  };
  // ---- the likelihood of step (t, p)'s proposal (:615-635), tile by tile: the wave
  //      takes row tiles from the step's LDS counter until none is left; `between` runs
  //      after its first tile (the control wave's pre-barrier work) ----
  auto lik_tiles = [&](int t, int p, int sp, auto&& between) {
    if (w == 2) NMC_CS((t - i0) * P + p, 12);
    // every LDS read of the restart issued before any is used: one round trip (left alone
    // the scheduler waits for the values before it issues the scale and variate reads)
    const double sv = st[(NMC_ST_S * P + p) * 64], zv = lds[(L.zl + 2 * sp) * 64 + 2 * lane];
    double thp[Fam::MAXP];
#pragma unroll
    for (int q = 0; q < Fam::MAXP; ++q) thp[q] = q < P ? th[q * 64] : 0.0;
    __builtin_amdgcn_sched_barrier(0);
    double vp = 0.0;   // thp[p] (a select per parameter: no dynamically indexed array)
#pragma unroll
    for (int q = 0; q < Fam::MAXP; ++q)
      if (q == p) vp = thp[q];
    const double prop = vp + (1.0 * sv) * zv;
#pragma unroll
    for (int q = 0; q < Fam::MAXP; ++q)
      if (q == p) thp[q] = prop;
    const typename Fam::Reg reg = fh.prepare(thp);
    // quad rows: intercept and slope of the four chains of this lane's quarter position
    double qc[4], qd[4];
    if constexpr (Fam::ASM_ROWS && RL && !HALF) if (quad) {
      nmc_quarters(reg.b0, qc);
      nmc_quarters(reg.b[0], qd);
    }
    // paired rows: the partner lane's (lane ^ 32) proposal parameters
    typename Fam::Reg preg = reg;
    if constexpr (nmc_paired_rows_ok<Fam>() && !HALF) if (paired && !quad) {
      const bool hi = lane >= 32;
#pragma unroll
      for (int q = 0; q < Fam::MAXP; ++q) {
        const nmc_pair2 e = nmc_halves(thp[q]);
        thp[q] = hi ? e.lo : e.hi;
      }
      preg = fh.prepare(thp);
    }
    if (w == 2) NMC_CS((t - i0) * P + p, 13);
    // the next tile is requested before the current one is computed: the atomic's
    // return rides under the tile's own row reads
    auto grab = [&]() -> unsigned {
      unsigned k = 0;
      if (lane == 0)
        k = __hip_atomic_fetch_add(tcnt + sp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return k;
    };
    // d.zin: queue entry 0 is the next step's variate job, entries 1.. the tiles
    const int tn = p + 1 < P ? t : t + 1, pn = p + 1 < P ? p + 1 : 0;
    const int zj = NMC_ZIN_BUILD && d.zin && tn < ie ? 1 : 0;
    // (waves 2.. start on their static entry: one LDS round trip off the step's restart)
    int kq = nstatic && w >= 2 ? (w - 2 < nt + zj ? w - 2 : nt + zj)
                               : (int)__builtin_amdgcn_readlane(grab(), 0);
#ifdef NMC_CSTAMPS
    bool first_tile = true;
#endif
    while (kq < nt + zj) {
      const unsigned kn = grab();
#ifdef NMC_CSTAMPS
      if (first_tile) NMC_CS((t - i0) * P + p, 16 + w);
      first_tile = false;
#endif
      if (kq < zj) {   // the variate job: {z, log u} of the next step -> the other slot
        gen_zl(tn, pn, sp ^ 1);
        kq = (int)__builtin_amdgcn_readlane(kn, 0);
        continue;
      }
      const int k = kq - zj;
      const int ra = TI.start(k);
      const int rn = TI.len(k);
      NMC_TILE_STAMP(k, 0);
      double acc[Fam::NACC];
      if constexpr (RL) {
        bool done = false;
        if constexpr (Fam::ASM_ROWS && !HALF) if (quad) {
          nmc_ll_rows_lds_quad(fh, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc, qc, qd);
          done = true;
        }
        if constexpr (nmc_paired_rows_ok<Fam>()) if (!done && (HALF || paired)) {
          // two chains per lane, row pairs split by lane half (half layout: one chain per
          // lane pair, each lane its row parity)
          nmc_ll_rows_lds<Fam, true, HALF>(fh, reg, lrows + (size_t)ra * Fam::NFIELDS, rn,
                                           acc, &preg);
          done = true;
        }
        if (!done)   // wave-uniform LDS address: broadcast ds_reads, pipelined
          nmc_ll_rows_lds(fh, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc);
      } else if constexpr (Fam::NFIELDS <= 4) {
        // rows beyond LDS, narrow rows: blocks of >= 4 rows per scalar load run ahead in
        // the scalar cache (the staged loop measured 1.7x slower for 2-field rows)
        nmc_ll_rows(fh, reg, grows + (size_t)ra * Fam::NFIELDS, rn, acc);
      } else {          // wide rows beyond LDS: staged per wave by LDS-DMA, two chunks deep
        nmc_ll_rows_staged(fh, reg, grows + (size_t)ra * Fam::NFIELDS, rn, glim,
                           lrows + (size_t)w * 2 * nmc_stage_buf(Fam::NFIELDS), acc);
      }
#pragma unroll
      for (int j = 0; j < Fam::NACC; ++j) lds[(L.part + j * NMC_NSLOT + k) * 64 + lane] = acc[j];
      NMC_TILE_STAMP(k, 1);
      between();
      kq = (int)__builtin_amdgcn_readlane(kn, 0);
    }
  };
  // ---- register mode: the Gibbs wave runs its own loop (gibbs_step below), so its 64-value
  //      payload never shares registers with the control code, and it meets the other
  //      waves at the same two barriers ----
  // the register hand-off's task of step (t, p): task k = gs - lag = (kt, kq) -- poll, fetch,
  // update, and (P <= 2) this step's priors; lane 0 leaves the verdict in the flag word
  auto gibbs_step = [&](int t, int p) {
    const int gs = t * P + p;
    if (gs - lag < gfirst) return;
    // task gs - lag as (kt, kq) without dividing by P (lag <= P)
    const int kq = p >= lag ? p - lag : p - lag + P, kt = p >= lag ? t : t - 1;
    NMC_CS(gs - i0 * P, 24);
    const bool r = nmc_poll_published(d, cb, kq, (unsigned)G * (unsigned)(kt - i0 + 1));
    NMC_CS(gs - i0 * P, 25);
    if (lane == 0)
      __hip_atomic_store(lds + L.flag * 64 + 1, r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (p == 0) NMC_STAMP_AUX(t, 13);
    if (r) {
      // keep the payload loads below the poll (no instruction: wavefront scope)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef NMC_CSTAMPS
      {   // (diagnostics: the fetch and the update stamped apart)
        double xv[64], fz, fx;
        nmc_hyper_fetch_reg(d, kt, kq, cc, xv, fz, fx);
        NMC_CS(gs - i0 * P, 26);
        nmc_hyper_compute_reg(d, cb, kt, kq, lds, L.hyp, g0w, fz, fx, xv);
        NMC_CS(gs - i0 * P, 27);
      }
#else
      nmc_hyper_update_reg(d, cb, kt, kq, cc, lds, L.hyp, g0w);
#endif
      if (p == 0) NMC_STAMP_AUX(t, 15);
      if (P <= 2) {   // the update lands in the step that needs it: this step's priors
        const int sp = gs & 1;
        const double v = th[p * 64];
        const double prop = v + (1.0 * st[(NMC_ST_S * P + p) * 64]) *
                                    lds[(L.zl + 2 * sp) * 64 + 2 * lane];
        const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
        const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
        cwv[NMC_CW_LPC * 64] =
            t > 0 ? nmc_norm_logpdf_r(v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
        cwv[NMC_CW_LPP * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
      }
      NMC_CS(gs - i0 * P, 28);
    }
  };
  // ---- the state after iteration iend - 1 -> HBM (control wave; the launch's epilogue) ----
  auto write_state = [&](int iend) {
    if (!(ctl && live)) return;
    double* vo = ((iend - 1) & 1) ? d.vb1 : d.vb0;
    for (int p = 0; p < P; ++p) {
      const size_t ip = (size_t)p * G * C + gc;
      if (!sync) vo[ip] = th[p * 64];
      d.lp[ip] = st[(NMC_ST_LP * P + p) * 64];
      d.scale[ip] = st[(NMC_ST_S * P + p) * 64];
      d.nacc[ip] = (int)st[(NMC_ST_NA * P + p) * 64];
      d.nrej[ip] = (int)st[(NMC_ST_NR * P + p) * 64];
      d.tacc[ip] = (long long)st[(NMC_ST_TA * P + p) * 64];
    }
    d.ll[gc] = c_LL;
  };
  // ---- resident launch: the end of a call (t == ie), every wave (uniform) ----
  // The call's results are completed as a launch completes them -- the last publication
  // counted, the pending step's state update and sample / trace stores, the call's last Gibbs
  // tasks (register mode: the workgroups of groups 0 .. lag-1, written through and recorded)
  // -- and every wave's stores drained; the workgroup counts itself done (the last one of the
  // grid tells the host: pinned memory) and takes the next command: workgroup 0 polls the
  // host's command word and relays it, the others poll the relay of their XCD.  On a new
  // end: the first step's variates and the hyper-parameters reloaded as a launch's prologue
  // loads them; the Gibbs pipeline restarts as at a launch's start (gfirst), so the next call
  // runs exactly as a new launch of [t, end) would.  The chain state (values, scales,
  // counters, priors, group LLs) stays in LDS and is written to HBM when the launch parks.
  // false: the launch ends (park, or a timeout in d.tmo).
  unsigned rseq = d.rseq, rcall = 0;   // (rcall: calls of this launch done)
  // (s_memrealtime when this workgroup started the current call: reported with its done)
  unsigned long long rt_start = RES ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // (GIBBS: the register-mode Gibbs wave's own loop, which runs the closing update; the
  //  main loop's copy holds no update and no 64-value payload)
  auto res_gate = [&](int t, auto gibbs) -> bool {
    if constexpr (!RES) {
      (void)t;
      (void)gibbs;
      return false;
    } else {
      const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();   // the call's loop done
      if (ctl) {
        if constexpr (sync) if (pub_p >= 0) {
          nmc_drain_vm();
          if (lane == 0)
            __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          pub_p = -1;
        }
        if (pend_p >= 0) apply_pending();
        store_pending();
      }
      // the call's last Gibbs tasks, as a launch closes them: task ge-lag+j by the workgroup
      // of group j, written through and recorded (every workgroup reloads them below)
      if constexpr (hr) {
        const int ck = close_of(ie);
        if (ck >= 0) {
          const bool pub = nmc_wait_published(d, cb, ck % P,
                                              (unsigned)G * (unsigned)(ck / P - i0 + 1), lds, L);
          if constexpr (decltype(gibbs)::value)
            if (pub) nmc_hyper_update_reg(d, cb, ck / P, ck % P, cc, lds, L.hyp, true);
        }
      }
      nmc_drain_vm();
      __syncthreads();
      if (ctl) {
        if (lane == 0) {
          // done: this workgroup's start / loop-end clocks into the launch's maxima, then its
          // arrival on the device counter; the last of the grid tells the host (one write
          // to pinned memory per call, not one per workgroup: PCIe writes are the slow part)
          unsigned long long* mx = (unsigned long long*)(d.rsync + NMC_RSYNC_MAX);
          __hip_atomic_fetch_max(mx, rt_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_max(mx + 1, rt_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          nmc_drain_vm();
          rcall += 1;
          const unsigned n = __hip_atomic_fetch_add(d.rsync + NMC_RSYNC_CNT, 1u,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (n + 1 == rcall * gridDim.x) {
            const unsigned long long ck[3] = {
                __builtin_amdgcn_s_memrealtime(),
                __hip_atomic_load(mx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
            __hip_atomic_store(mx, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(mx + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              __hip_atomic_store(d.rdone + 2 + 2 * k, (unsigned)ck[k], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(d.rdone + 3 + 2 * k, (unsigned)(ck[k] >> 32), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
            }
            nmc_drain_vm();
            __hip_atomic_store(d.rdone, rseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        unsigned end = 0xffffffffu;
        if (blockIdx.x == 0) {
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          unsigned seq = rseq;
          for (unsigned spins = 0;; ++spins) {
            const unsigned long long v =
                __hip_atomic_load(d.rcmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((int)((unsigned)v - rseq) > 0) {
              seq = (unsigned)v;
              end = (unsigned)(v >> 32);
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > d.ridle) break;   // idle: park
            if ((spins & 63) == 63 &&
                __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
              break;
            __builtin_amdgcn_s_sleep(4);
          }
          // (an idle park relays the next seq: the relay only ever moves forward); one copy
          // per XCD's workgroups (b & 7), each on its own 128-B line: 32 pollers a line
          if (lane < 8)
            __hip_atomic_store(
                (unsigned long long*)(d.rsync + NMC_RSYNC_REL + 32 * lane),
                ((unsigned long long)end << 32) | (seq != rseq ? seq : rseq + 1u),
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (lane == 0) {
            if (seq != rseq && end != 0xffffffffu) {   // taken: the clock, then the seq
              const unsigned long long clk = __builtin_amdgcn_s_memrealtime();
              __hip_atomic_store(d.rack + 2, (unsigned)clk, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(d.rack + 3, (unsigned)(clk >> 32), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              nmc_drain_vm();
              __hip_atomic_store(d.rack, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {   // parked (idle, or the host's park command seq)
              __hip_atomic_store(d.rack + 1, 0x80000000u | seq, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
          rseq = seq;
        } else {
          for (unsigned spins = 0;; ++spins) {
            const unsigned long long v =
                __hip_atomic_load((unsigned long long*)(d.rsync + NMC_RSYNC_REL +
                                                        32 * (blockIdx.x & 7)),
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((int)((unsigned)v - rseq) > 0) {
              rseq = (unsigned)v;
              end = (unsigned)(v >> 32);
              break;
            }
            if ((spins & 255) == 255 &&
                __hip_atomic_load(d.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
              break;
            if (spins >= NMC_SPIN_LIMIT) {
              __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
        const bool go = end != 0xffffffffu && (int)end > t;
        if (go) put_zl(t, 0, (t * P) & 1);   // the first step's {z, log u}
        if (lane == 0) lds[L.flag * 64 + 2] = go ? (double)end : -1.0;
      }
      __syncthreads();
      const double e = lds[L.flag * 64 + 2];
      if (e < 0.0) return false;
      if constexpr (hr) {   // the hyper-parameters after iteration t - 1, as a launch's
                            // prologue loads them (parameter p by wave p % W; sc1: the closing
                            // workgroups wrote them through before the call was reported done)
        for (int p = w; p < P; p += W) {
          const size_t ho = nmc_hslot(d, t - 1) + (size_t)p * C + cc;
          const double s2 = nmc_ldv<NMC_SRC_SC1>(d.s2 + ho);
          const double m = nmc_ldv<NMC_SRC_SC1>(d.mu + ho);
          const double sd = nmc_ldv<NMC_SRC_SC1>(d.hsd + ho);
          const double lsd = nmc_ldv<NMC_SRC_SC1>(d.hlsd + ho);
          hy[(NMC_HY_MU * P + p) * 64] = m;
          hy[(NMC_HY_SD * P + p) * 64] = sd;
          hy[(NMC_HY_LSD * P + p) * 64] = lsd;
          hy[(NMC_HY_S2 * P + p) * 64] = s2;
          hy[(NMC_HY_SDM * P + p) * 64] = sqrt(s2 / G);
          hy[(NMC_HY_ISD * P + p) * 64] = 1.0 / sd;
        }
      }
      nmc_drain_vm();   // (the control wave's variate DMA has landed)
      __syncthreads();
      ie = (int)e;
      gfirst = t * P;
      rt_start = __builtin_amdgcn_s_memrealtime();
      return true;
    }
  };
  if constexpr (hr) if (gw) {
    const int gs0 = i0 * P;
    (void)gs0;   // (the control-path stamps build)
    for (int t = i0; ok; ++t) {
      if (t == ie && !res_gate(t, nmc_bool_c<true>{})) break;
      for (int p = 0; p < P; ++p) {
        dP = nmc_kdev();
        const int gs = t * P + p;
        const bool due = gs - lag >= gfirst;
        gibbs_step(t, p);
#if NMC_GIBBS_TILES   // (A/B build option: the Gibbs wave takes likelihood tiles after its task)
        lik_tiles(t, p, gs & 1, [] {});
#endif
        NMC_CS(gs - gs0, w);
        nmc_run_barrier();   // A
        if (due) {
          ok = lds[L.flag * 64 + 1] == 2.0 * ((double)gs + 1);
          if (!ok) break;
        }
        nmc_run_barrier();   // B
      }
    }
    // closing: tasks ge-lag .. ge-1, task ge-lag+j by the workgroup of group j (member 0),
    // which writes and records it -- in parallel, not one after the other; the same
    // barrier as the other waves' nmc_wait_published (RES: closed at the last gate)
    const int close_k = close_of(ie);
    if (!RES && ok && close_k >= 0) {
      if (nmc_wait_published(d, cb, close_k % P, (unsigned)G * (unsigned)(close_k / P - i0 + 1),
                             lds, L))
        nmc_hyper_update_reg(d, cb, close_k / P, close_k % P, cc, lds, L.hyp, true);
    }
    nmc_drain_vm();
    return;
  }

  for (int t = i0; ok; ++t) {
    if (t == ie && !res_gate(t, nmc_bool_c<false>{})) break;
    NMC_STAMP(t, 0);
    for (int p = 0; p < P; ++p) {
      dP = nmc_kdev();
      const int sp = (t * P + p) & 1;
      double c_prop, c_v, c_lu, c_lpc, c_lpp, c_sA, c_sR;   // control wave, this step
      // the proposal's prepared parameters, formed before barrier A (the other values
      // cannot change before the decision), so only the slot sum, finish and the
      // Metropolis test remain between the barriers
      typename Fam::Reg c_reg{};
      // Gibbs update after iteration t-1 in the all-wave modes (persistent SYNC, launch per
      // iteration): every parameter at step 0 of t (NMC_HYPER_ALLP), or parameter p at step
      // (t, p), right before the decision that needs it
      const bool hyper_now = !hl && PARTIAL && (NMC_HYPER_ALLP ? p == 0 : true) && t > 0 &&
                             !(t == i0 && (flags & NMC_RUN_HYPER_LOAD));
      // persistent Gibbs wave: the Gibbs update of parameter q after iteration tq is
      // task k = tq*P + q; every workgroup publishes it right after its decision at
      // global step k, so it is counted at the start of step k+1.  P == 1: the Gibbs
      // wave polls, copies and updates task gs-1 at step gs (needed at once).  P >= 2
      // (two-stage pipeline): the control wave polls task gs-1 at step gs and copies its
      // payload into LDS buffer (gs-1)&1; the Gibbs wave updates task gs-2 from buffer
      // gs&1 at step gs, beside the tiles -- needed first at step gs-2+P.
      const int gs = t * P + p, gs0 = i0 * P;
      const bool pipe = hl && !hr && P >= 2;   // two-stage (payload-in-LDS) hand-off
      const int aq = p > 0 ? p - 1 : P - 1;        // task gs-1 = (atq, aq)
      const int atq = p > 0 ? t : t - 1;
      const bool aux_now = hl && gs - lag >= gfirst;   // the Gibbs wave's task this step
      const bool comp_now = pipe && gs - 2 >= gs0;  // Gibbs task gs-2 = (ctq, cq)
      const int cq = (p + 2 * P - 2) % P;
      const int ctq = p >= 2 ? t : t - 1;
      // this step's priors come from the Gibbs wave when the update they depend on
      // lands during this step (P == 1, or P == 2 with the pipeline full)
      const bool post_prior =
          hr ? P <= 2 && aux_now : (P == 1 ? aux_now : (P == 2 && comp_now));
      // ---- the Gibbs wave, beside this step's likelihood tiles (LDS payload modes) ----
      if constexpr (hl && !hr) if (gw) {
        bool upd = false;
        if (!pipe && aux_now) {   // P == 1: poll task gs-1, copy it, update it
          const size_t hvi = (((size_t)(atq - d.vbase) * P + aq) * C + cc) * 2;
          const double hz = d.vh[hvi], hx = d.vh[hvi + 1];
          const bool r = nmc_poll_published(d, cb, aq, (unsigned)G * (unsigned)(atq - i0 + 1));
          if (lane == 0)
            __hip_atomic_store(lds + L.flag * 64 + 1, r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (p == 0) NMC_STAMP_AUX(t, 13);
          if (r) {
            // keep the payload loads below the poll (no instruction: wavefront scope)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double* src = (atq & 1) ? d.vb1 : d.vb0;
            if ((C & 1) == 0) {
              nmc_hyper_dma(d, src, aq, cb, 0, G, lds, L, 0);
              nmc_drain_vm();
            } else {
              nmc_hyper_load(d, src, aq, cc, 0, G, lds, L, 0);
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            nmc_hyper_compute(d, cb, atq, aq, lds, L, g0w, hz, hx, 0);
            upd = true;
          }
        } else if (comp_now) {   // P >= 2: task gs-2, copied into buffer (gs-2)&1 at step gs-1
          const size_t hvi = (((size_t)(ctq - d.vbase) * P + cq) * C + cc) * 2;
          if (p == 0) NMC_STAMP_CMP(t, 13);
          nmc_hyper_compute(d, cb, ctq, cq, lds, L, g0w, d.vh[hvi], d.vh[hvi + 1],
                            (gs & 1) * (G + 1));
          if (p == 0) NMC_STAMP_CMP(t, 14);
          upd = post_prior;
        }
        if (upd) {   // this step's priors (:293-294) from the update just made
          const double v = th[p * 64];
          const double prop = v + (1.0 * st[(NMC_ST_S * P + p) * 64]) *
                                      lds[(L.zl + 2 * sp) * 64 + 2 * lane];
          const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
          const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
          cwv[NMC_CW_LPC * 64] =
              t > 0 ? nmc_norm_logpdf_r(v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
          cwv[NMC_CW_LPP * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
          if (p == 0) NMC_STAMP_CMP(t, 15);
        }
      }
      // ---- control wave: counter add of the last publish, the poll and payload copy of
      //      task gs-1, the pending state update, both outcomes of the decision --
      //      accept (sA, naA, nrA, ta + 1) / reject (sR, naR, nrR, ta), tuned if due --,
      //      the next step's variates in flight, priors ----
      auto ctl_work = [&]() {
        if constexpr (sync && !hr) {   // the previous step's value is stored; count it published
          if (pub_p >= 0) {
            nmc_drain_vm();
            if (lane == 0)
              __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            pub_p = -1;
          }
        }
        if constexpr (hl) if (pipe && aux_now) {   // verdict word (checked after barrier A), copy
          const bool r = nmc_poll_published(d, cb, aq, (unsigned)G * (unsigned)(atq - i0 + 1));
          if (lane == 0)
            __hip_atomic_store(lds + L.flag * 64 + 1, r ? 2.0 * ((double)gs + 1) : -2.0 * ((double)gs + 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (p == 0) NMC_STAMP(t, 8);
          if (r) {
            // keep the payload loads below the poll (no instruction: wavefront scope)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double* src = (atq & 1) ? d.vb1 : d.vb0;
            if ((C & 1) == 0)
              nmc_hyper_dma(d, src, aq, cb, 0, G, lds, L, ((gs - 1) & 1) * (G + 1));
            else
              nmc_hyper_load(d, src, aq, cc, 0, G, lds, L, ((gs - 1) & 1) * (G + 1));
          }
        }
        if (pend_p >= 0) apply_pending();
        c_v = th[p * 64];
        const double s = st[(NMC_ST_S * P + p) * 64];
        c_prop = c_v + (1.0 * s) * lds[(L.zl + 2 * sp) * 64 + 2 * lane];   // propose (:304-306)
        c_lu = lds[(L.zl + 2 * sp) * 64 + 2 * lane + 1];
        {
          double thp[Fam::MAXP];
#pragma unroll
          for (int q = 0; q < Fam::MAXP; ++q)
            thp[q] = q < P ? (q == p ? c_prop : th[q * 64]) : 0.0;
          c_reg = fh.prepare(thp);
        }
        {
          const double na = st[(NMC_ST_NA * P + p) * 64], nr = st[(NMC_ST_NR * P + p) * 64];
          double naA = na + 1.0, nrA = nr, naR = na, nrR = nr + 1.0;
          c_sA = s;
          c_sR = s;
          // (tuning is the control wave's alone: evaluated here, the burn-in and interval
          //  loads and the division stay off the other waves' restart)
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
        }
        if (!hl && hyper_now) nmc_hyper_variates(d, cb, t - 1, lds, L, 0, 1);
        if (PARTIAL && !hl && p == (P > 1 ? 1 : 0)) nmc_hyper_sdm(d, lds, L, lane);
        if (!hyper_now && !(hl && post_prior)) {   // priors (:293-294)
          if (PARTIAL) {
            const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
            const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
            c_lpc = t > 0 ? nmc_norm_logpdf_r(c_v, m, sd, isd, lsd) : st[(NMC_ST_LP * P + p) * 64];
            c_lpp = nmc_norm_logpdf_r(c_prop, m, sd, isd, lsd);
          } else {
            c_lpc = st[(NMC_ST_LP * P + p) * 64];
            c_lpp = nmc_prior_logpdf(d.pfam[p], d.ppar + 8 * p, c_prop);
          }
        }
      };
      // ---- the control wave's memory work, last before its tiles: the count of the previous
      //      step's publication (register Gibbs mode: after the pre-work above, so the publish
      //      store has drained), then the pending sample / trace stores (issued after the count,
      //      whose vmcnt wait then covers the publish store alone) and the next step's variate
      //      DMA.  (Deferring this work until after the control wave's first tile measured
      //      slower: 15.4-15.6 against 14.7-15.0 ms per 2 000 iterations, profiles/r06.)
      auto ctl_post = [&]() {
        if constexpr (hr) {   // count the previous step's value published (the Gibbs waves
                              // poll it two steps on)
          if (pub_p >= 0) {
            nmc_drain_vm();
            if (lane == 0)
              __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            pub_p = -1;
          }
        }
        store_pending();
        const int tn = p + 1 < P ? t : t + 1;
        const int pn = p + 1 < P ? p + 1 : 0;
        if (tn < ie && !(NMC_ZIN_BUILD && d.zin)) put_zl(tn, pn, sp ^ 1);   // (zin: the job)
      };
      if (ctl) {
        ctl_work();
        ctl_post();
      }
      // the control wave's tiles at the issue priority of the tile waves (its SIMD partner is
      // one of them); the decision after barrier A runs at priority 3 again
      if (ctl && ctlprio) __builtin_amdgcn_s_setprio(0);
      // ---- likelihood of the proposal (:615-635), tile by tile, every wave ----
      lik_tiles(t, p, sp, [] {});
      if (ctl && ctlprio) __builtin_amdgcn_s_setprio(3);
      NMC_STAMP(t, 1 + 3 * (p & 1));
      if (ctl || (hl && !pipe && gw)) nmc_drain_vm();   // this wave's LDS-DMA has landed
      NMC_CS(gs - gs0, w);
      nmc_run_barrier();   // A
      NMC_STAMP(t, 2 + 3 * (p & 1));
      if (ctl) NMC_CS(gs - gs0, 8);

      // ---- Gibbs update after iteration t-1 (needed by this iteration's priors) ----
      // (Gibbs-wave modes: the poller's verdict is read in the same LDS batch as the
      // decision's operands and checked after the decision; an aborted step's decision is
      // never used -- the launch reports the timeout)
      double verdict = 0.0;
      if constexpr (hl) if (aux_now) verdict = lds[L.flag * 64 + 1];
      if constexpr (PARTIAL && !hl) if (hyper_now) {
        // (NMC_HYPER_ALLP: every parameter at step 0, once P-1's count is full)
        const int hp = NMC_HYPER_ALLP ? -1 : p, wp = NMC_HYPER_ALLP ? P - 1 : p;
        if constexpr (sync) {   // parameter p of t-1 is published once its count is full
          ok = nmc_wait_published(d, cb, wp, (unsigned)G * (unsigned)(t - i0), lds, L);
          if (!ok) break;
          nmc_hyper<NMC_SRC_SC1>(d, ((t - 1) & 1) ? d.vb1 : d.vb0, cb, t - 1, lds, L, g0w, hp);
        } else {
          nmc_hyper<NMC_SRC_GLOBAL>(d, ((t - 1) & 1) ? d.vb1 : d.vb0, cb, t - 1, lds, L, g0w, hp);
        }
        if (ctl) {
          const double m = hy[(NMC_HY_MU * P + p) * 64], sd = hy[(NMC_HY_SD * P + p) * 64];
          const double lsd = hy[(NMC_HY_LSD * P + p) * 64], isd = hy[(NMC_HY_ISD * P + p) * 64];
          c_lpc = nmc_norm_logpdf_r(c_v, m, sd, isd, lsd);   // t > 0 (setPrior :281)
          c_lpp = nmc_norm_logpdf_r(c_prop, m, sd, isd, lsd);
        }
        NMC_STAMP(t, 9);
      }

      // ---- control wave: group log-likelihood of the proposal (tiles in order) and
      //      the Metropolis decision, one chain per lane (:334-383) ----
      if (ctl) {
        // this step's tiles are all taken; reused at step +2 (from the static entries on)
        if (lane == 0) tcnt[sp] = (unsigned)(nstatic && W > 2 ? W - 2 : 0);
        if (hl && post_prior) {   // the Gibbs wave evaluated this step's priors (read in the
                                  // slot sums' LDS round trip)
          c_lpc = cwv[NMC_CW_LPC * 64];
          c_lpp = cwv[NMC_CW_LPP * 64];
        }
        double acc[Fam::NACC];
#pragma unroll
        for (int j = 0; j < Fam::NACC; ++j) {
          acc[j] = nmc_sum_slots(lds + (L.part + j * NMC_NSLOT) * 64 + lane);
        }
        if (S > 1)   // row split: every member's partials, in member order
          nmc_split_exchange(d, cb, g, mb, t * P + p - i0 * P, acc);
        if (p == 0) NMC_STAMP(t, 10);
        NMC_CS(gs - gs0, 14);
        const double llp = fh.finish_fast(c_reg, acc, (long)ngrp, gcst);
        if (p == 0) NMC_STAMP(t, 11);
        NMC_CS(gs - gs0, 15);
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
        if constexpr (sync) {   // publish write-through; counted at the next step's start
          if (live) nmc_store_wt(((t & 1) ? pub1 : pub0) + (size_t)p * G * C, vn);
          if (mb == 0) pub_p = p;   // (row split: member 0 publishes and counts)
        }
        st[(NMC_ST_S * P + p) * 64] = accept ? c_sA : c_sR;
        q_acc = accept;
        q_plp = accept ? c_lpp : c_lpc;
        q_pll = llp;
        pend_p = p;
        pend_t = t;
        // the rest of the update waits for the next step's pre-barrier slack
        if (p == 0) NMC_STAMP(t, 12);
      }
      if constexpr (hl) if (aux_now) {
        ok = verdict == 2.0 * ((double)gs + 1);
        if (!ok) break;
      }
      if (p == 0) NMC_STAMP(t, 3);
      if (ctl) NMC_CS(gs - gs0, 9);
      nmc_run_barrier();   // B: the new value is visible to every wave
      if (ctl) NMC_CS(gs - gs0, 10);
      if (w == 2) NMC_CS(gs - gs0, 11);
    }
    NMC_STAMP(t, 6);
    if (!ok) break;
    NMC_STAMP(t, 7);
  }

  NMC_RUN_SL(2);
  if constexpr (RES) {   // (the last call was closed at its gate): the state to HBM
    if (ok) write_state(ie);
    nmc_drain_vm();
    return;
  }
  if constexpr (sync) if (ctl && pub_p >= 0) {   // the last parameter's count
    nmc_drain_vm();
    if (lane == 0)
      __hip_atomic_fetch_add(nmc_counter(d, cb, pub_p, g & 7), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }

  if (ctl && pend_p >= 0) apply_pending();
  if (ctl) store_pending();
  // ---- epilogue: state back to HBM (control wave) ----
  if (ok) write_state(i1);
  // ---- closing Gibbs updates after i1-1 (group-0 workgroups write and record them; the
  //      register mode: the workgroups of groups 0 .. lag-1) ----
  const int close_k = close_of(i1);
  if constexpr (hl) if (ok && (hr ? close_k >= 0 : g0w)) {
    const int ge = i1 * P;   // tasks ge-2 (copied at the last step; P >= 2) and ge-1 are left
    if (!hr && P >= 2 && gw) {
      const size_t hvi = (((size_t)(i1 - 1 - d.vbase) * P + (P - 2)) * C + cc) * 2;
      nmc_hyper_compute(d, cb, i1 - 1, P - 2, lds, L, true, d.vh[hvi], d.vh[hvi + 1],
                        ((ge - 2) & 1) * (G + 1));
    }
    // (register mode: the Gibbs wave closes in its own loop; this is the matching barrier)
    const int wk = hr ? close_k : ge - 1;   // the task whose publication is awaited
    const bool pub = nmc_wait_published(d, cb, wk % P, (unsigned)G * (unsigned)(wk / P - i0 + 1),
                                        lds, L);
    if (!hr && pub && gw) {
      const double* src = ((i1 - 1) & 1) ? d.vb1 : d.vb0;
      const int ho = ((ge - 1) & 1) * (G + 1);
      if ((C & 1) == 0) {
        nmc_hyper_dma(d, src, P - 1, cb, 0, G, lds, L, ho);
        nmc_drain_vm();
      } else {
        nmc_hyper_load(d, src, P - 1, cc, 0, G, lds, L, ho);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      const size_t hvi = (((size_t)(i1 - 1 - d.vbase) * P + (P - 1)) * C + cc) * 2;
      nmc_hyper_compute(d, cb, i1 - 1, P - 1, lds, L, true, d.vh[hvi], d.vh[hvi + 1], ho);
    }
  }
  if constexpr (sync && !hl) if (ok && g0w) {
    nmc_hyper_sdm(d, lds, L, lane);
    nmc_hyper_variates(d, cb, i1 - 1, lds, L, 0, W);
    nmc_drain_vm();
    if (nmc_wait_published(d, cb, P - 1, (unsigned)G * (unsigned)(i1 - i0), lds, L))
      nmc_hyper<NMC_SRC_SC1>(d, ((i1 - 1) & 1) ? d.vb1 : d.vb0, cb, i1 - 1, lds, L, true);
  }
  NMC_RUN_SL(3);
#undef d
}

// Group log-likelihoods for arbitrary theta [P][G][C] (the batched start-point search and
// partial init of nestmc/init.py), summed EXACTLY as the step kernels sum a proposal's
// likelihood: the same row-split members, tile partition (nmc_tiles), row loop (rows
// staged in LDS or read from global memory, as the step kernel of this context does),
// 16-slot combine, member order and finish_fast -- so a chain's stored group LL never
// depends on which kernel produced it, on the wave count or on the chain sharding.
// Part 1: grid CB * G * S workgroups (member m of group g of chain block cb), W waves take
// tiles k = w, w + W, ...; out part[m][j][g][C] (NACC accumulators).
template <class Fam, bool RL>
__global__ void __launch_bounds__(512)
nmc_k_group_part(Dev d, Fam fam, const double* __restrict__ obs, const double* theta,
                 double* part) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // [NACC][NSLOT] slots, rows
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int S = d.S;
  const int mb = blockIdx.x % S;
  const int g = (blockIdx.x / S) % d.G, cb = (blockIdx.x / S) / d.G;
  const int c = cb * 64 + lane;
  const int cc = c < d.C ? c : d.C - 1;
  double th[Fam::MAXP];
  nmc_load_theta(d, theta, g, cc, th);
  const typename Fam::Reg reg = fam.prepare(th);
  int64_t r0;
  int nrow;
  nmc_chunk(d.off[g], d.off[g + 1], mb, S, &r0, &nrow);
  const nmc_tiling TI = nmc_tiles(nrow, d.tile);
  const double* grows = obs + r0 * Fam::NFIELDS;
  double* lrows = lds + Fam::NACC * NMC_NSLOT * 64;
  if constexpr (RL) {
    const int nd = nrow * Fam::NFIELDS;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
  }
  for (int j = 0; j < Fam::NACC; ++j)
    for (int k = TI.nt + w; k < NMC_NSLOT; k += W) lds[(j * NMC_NSLOT + k) * 64 + lane] = -0.0;
  __syncthreads();
  for (int k = w; k < TI.nt; k += W) {
    const int ra = TI.start(k), rn = TI.len(k);
    double acc[Fam::NACC];
    if constexpr (RL)
      nmc_ll_rows_lds(fam, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc);
    else
      nmc_ll_rows(fam, reg, grows + (size_t)ra * Fam::NFIELDS, rn, acc);
#pragma unroll
    for (int j = 0; j < Fam::NACC; ++j) lds[(j * NMC_NSLOT + k) * 64 + lane] = acc[j];
  }
  __syncthreads();
  if (w != 0 || c >= d.C) return;
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j)
    part[(((size_t)mb * Fam::NACC + j) * d.G + g) * d.C + c] = nmc_sum_slots(lds + j * NMC_NSLOT * 64 + lane);
}

// Part 2: the members' partials in member order (nmc_split_exchange's four streams),
// finish_fast -> out [G][C].  One thread per (group, chain).
template <class Fam>
__global__ void __launch_bounds__(256)
nmc_k_group_fin(Dev d, Fam fam, const double* theta, const double* part, double* out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)d.G * d.C) return;
  const int c = (int)(i % d.C), g = (int)(i / d.C);
  const int S = d.S;
  double th[Fam::MAXP];
  nmc_load_theta(d, theta, g, c, th);
  const typename Fam::Reg reg = fam.prepare(th);
  double acc[Fam::NACC];
#pragma unroll
  for (int j = 0; j < Fam::NACC; ++j) {
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int m = 0; m < S; ++m) {
      const double v = part[(((size_t)m * Fam::NACC + j) * d.G + g) * d.C + c];
      s4[m & 3] = m < 4 ? v : s4[m & 3] + v;
    }
    acc[j] = S >= 4 ? (s4[0] + s4[1]) + (s4[2] + s4[3])
                    : (S == 1 ? s4[0] : (S == 2 ? s4[0] + s4[1] : (s4[0] + s4[1]) + s4[2]));
  }
  const long n = (long)(d.off[g + 1] - d.off[g]);
  out[i] = fam.finish_fast(reg, acc, n, fam.gconst(n));
}

// StepMethod.logLikelihood (:656-659) at recorded rows of the device sample store:
// out[c - c0][r][i] = observation i's log-likelihood at the values of row row0 + r (the state
// Sampler._printLogLikelihood evaluated at that recorded iteration, :890-891).  One
// thread per (observation, chain, row), writes coalesced along the observations.
// pc: 2 if the sample columns carry the hyper-parameters (partial pooling), else 0.
template <class Fam>
__global__ void __launch_bounds__(256)
nmc_k_obs_ll_rows(Dev d, Fam fam, const int* __restrict__ gidx, int64_t n_obs, int pc, int row0,
                  int nrows, int c0, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = c0 + (int)blockIdx.y, r = blockIdx.z;   // (chains [c0, c0 + gridDim.y))
  if (i >= n_obs) return;
  const int g = gidx[i];
  const double* row = d.samples + (size_t)(row0 + r) * d.cols * d.C + c;
  double th[Fam::MAXP];
#pragma unroll
  for (int q = 0; q < Fam::MAXP; ++q)
    th[q] = q < d.P ? row[((size_t)q * (d.G + pc) + pc + g) * d.C] : 0.0;
  const typename Fam::Reg reg = fam.prepare(th);
  out[((size_t)blockIdx.y * nrows + r) * n_obs + i] = fam.obs_ll(reg, d.obs + i * Fam::NFIELDS);
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

