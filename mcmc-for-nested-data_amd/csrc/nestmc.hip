// nestmc.hip -- libnestmc.so: the C-ABI (include/nestmc.h) over the gfx950 kernels.
//
// One context = one (process, GPU) shard of chains.  All device state is resident
// in HBM for the whole run; nmc_run enqueues P step launches per iteration on the
// context's stream (partial pooling folds each Gibbs update into the next launch)
// and never synchronises, so a whole chunk of iterations is queued back to back.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "ctx.h"
#include "kernels_misc.h"

#define NMC_VERSION "nestmc 0.2.0 (gfx950)"

static thread_local std::string g_err;

int nmc_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
static int fail(int code, const std::string& msg) { return nmc_fail(code, msg); }

template <class T>
static int dalloc(nmc_ctx* x, T** p, size_t n) {
  void* q = nullptr;
  if (n == 0) n = 1;
  HIPCHK(hipMalloc(&q, n * sizeof(T)));
  x->owned.push_back(q);
  *p = (T*)q;
  return 0;
}

static void dfree(nmc_ctx* x, void* p) {
  if (!p) return;
  for (auto& q : x->owned)
    if (q == p) { hipFree(q); q = nullptr; }
}

// Waves per workgroup: one per 64 rows of the largest group plus the control wave
// (and the Gibbs wave under partial pooling), at most 8 (one 512-thread workgroup per
// CU, 256 VGPRs per lane): the row loop is LDS-broadcast bound at ~5 cycles per row
// from 5 waves on (tools/llbench4.hip, profiles/llbench4_r02.json), so more waves only
// cost registers.  Every wave takes likelihood tiles once its own role is done; the
// tile partition depends on the group's rows alone (nmc_tiles), so W, NAUX and the
// launch mode never change a sum.
static void choose_geometry(nmc_ctx* x) {
  Dev& d = x->d;
  int64_t w = 1 + (d.nmax + 63) / 64;
  if (x->pooling == NMC_POOL_PARTIAL && w >= 2) w += 1;
  if (w > 8) w = 8;   // (a 768-thread build runs 12 only when asked: NMC_WAVES)
  if (w < 1) w = 1;
  d.CL = 64;   // one chain per lane, every kernel
  // the wave count from the rows alone: the none/complete-pooling tile balance below sizes
  // the tiles from it, so the NMC_WAVES override never changes a sum
  const int64_t w_rows = w;
  if (const char* e = getenv("NMC_WAVES")) {
    const int v = atoi(e);
    if (v >= 1 && v <= NMC_RUN_THREADS / 64) w = v;
  }
  d.RB = (d.C + d.CL - 1) / d.CL;
  d.W = (int)w;
  d.tile = 64;   // rows per likelihood tile (a multiple of 16)
#ifdef NMC_DEBUG_KNOBS   // (diagnostic builds only: changes the summation order)
  if (const char* e = getenv("NMC_TILE_ROWS")) {
    const int v = atoi(e);
    if (v >= 16 && v % 16 == 0) d.tile = v;
  }
#endif
  // partial pooling, persistent payload-in-LDS mode: wave 1 is the Gibbs wave
  d.naux = x->pooling == NMC_POOL_PARTIAL && d.W >= 3 && d.nleaf <= 4 ? 1 : 0;
  // rows in LDS when they fit beside the rest of the carve (64 KiB for the rows)
  d.rows_lds = (size_t)d.nmax * x->nf * 8 <= (size_t)64 * 1024 &&
               lds_bytes_for(x, 0, 1) <= (size_t)96 * 1024;
#ifdef NMC_DEBUG_KNOBS   // (diagnostic builds only: the scalar-load row loop's blocks differ)
  if (getenv("NMC_NO_LDS_ROWS") && atoi(getenv("NMC_NO_LDS_ROWS"))) d.rows_lds = 0;
#endif

  // the persistent Gibbs update by the auxiliary waves needs G <= 128 (one numpy
  // leaf) and one parameter's chain-block values in LDS
  d.noprio = getenv("NMC_NOPRIO") ? atoi(getenv("NMC_NOPRIO")) : 0;   // diagnostics bits
  d.ctiles = getenv("NMC_CTL_TILES") ? atoi(getenv("NMC_CTL_TILES")) : 1;   // (Dev.ctiles)
  d.gtiles = getenv("NMC_GIBBS_TILES") ? atoi(getenv("NMC_GIBBS_TILES")) : 1;   // (Dev.gtiles)
  d.pubearly = 0;   // (Dev.pubearly: set with the geometry, NMC_PUB_EARLY overrides)
  d.gwaves = 4;   // (waves of nmc_k_sweep_gibbs)
  d.nstatic = getenv("NMC_STATIC_TILES") ? atoi(getenv("NMC_STATIC_TILES")) != 0 : 1;
  d.hlds = d.naux > 0 && d.G <= 128 && lds_bytes_for(x, 1, d.rows_lds) <= (size_t)160 * 1024 &&
           !(getenv("NMC_NO_HLDS") && atoi(getenv("NMC_NO_HLDS")));
  // G <= 64: the Gibbs wave fetches a task's values into registers (one sc1 round trip)
  // and updates in the step after publication (no LDS payload, no two-stage pipeline).
  // (An owner hand-off for 64 < G -- one workgroup's Gibbs wave updating each task once
  //  for its chain block, the others reading its results -- measured slower, 62 against
  //  53 us/iter at the cfg-4 shard, and was removed in round 5; G > 128 runs nmc_k_sweep's
  //  Gibbs workgroups, which do the same with whole workgroups.)
  d.hreg = d.naux > 0 && d.G <= 64 && d.hlds &&
           !(getenv("NMC_NO_HREG") && atoi(getenv("NMC_NO_HREG")));
  // Partial pooling whose grid is more than one 8-wave workgroup per CU but fits two
  // 4-wave ones (cfg-4 shards: 2 chain blocks x 256 groups): four waves, so the whole
  // grid is resident and runs persistent (both chain blocks' workgroups share each CU
  // and interleave their serial phases) -- measured 48.5 against 67.6 us/iter in
  // launch-per-iteration mode at 128 x 256 x 2000.
  if (x->pooling == NMC_POOL_PARTIAL && d.W > 4 && !getenv("NMC_WAVES")) {
    const int64_t wgs = (int64_t)d.RB * d.G * d.S;
    if (wgs > x->ncu && wgs <= 2 * (int64_t)x->ncu) {
      const int w8 = d.W;
      d.W = 4;
      if (lds_bytes_for(x, d.hlds, d.rows_lds) > (size_t)80 * 1024) d.W = w8;
    }
  }
  // likelihood rows in LDS for a family whose row blocks pair up (<= 4 fields): each lane
  // evaluates its rows for two chains (kernels.h nmc_ll_rows_lds<Fam, true>), half the LDS
  // reads; NMC_ROWS=bcast keeps the one-chain broadcast loop (same sums bit for bit)
  d.paired = d.rows_lds && x->nf <= 4;
  if (const char* e = getenv("NMC_ROWS")) d.paired = d.paired && strcmp(e, "bcast") != 0;
  // {x, y} rows (linear regression with one covariate): four chains per lane instead
  // (kernels.h nmc_ll_rows_lds_quad, nmc_k_run only), the same sums bit for bit;
  // NMC_ROWS=pair keeps the paired loop
  d.quad = d.paired && x->family == NMC_LL_LINREG && x->nf == 2;
  if (const char* e = getenv("NMC_ROWS")) d.quad = d.quad && strcmp(e, "pair") != 0;

  // none/complete pooling whose 64-chain grid fills at most half the CUs (cfg 2: 4 chain
  // blocks x 32 groups on 256 CUs): 32 chains per workgroup, each lane pair one chain on
  // the paired loop's two row parities (NMC_MODE_HALF) -- twice the workgroups, the same
  // sums bit for bit.  NMC_HALF=0 keeps 64 chains per workgroup (tests compare them).
  if (x->pooling != NMC_POOL_PARTIAL && d.S == 1 && d.paired &&
      (int64_t)d.RB * d.G * 2 <= x->ncu && !(getenv("NMC_HALF") && !atoi(getenv("NMC_HALF")))) {
    d.CL = 32;
    d.RB = (d.C + d.CL - 1) / d.CL;
  }
  // none/complete pooling: a step's likelihood tiles go to the W - 1 waves other than the
  // control wave (which first prepares the step).  When the 64-row tiles are a few more
  // than those waves, one wave runs two and the step waits for it (cfg 2: 8 tiles of its
  // 500 rows on 7 waves; the last wave reaches barrier A 2.3k cycles after the others,
  // profiles/r05/r05s_cstamps_cfg3_cfg2.jsonl), so the tiles are sized ceil(n / (W - 1))
  // rows instead, one per wave.  (A different tile partition: the sums' last bits.)  The
  // partition depends on the rows only (w_rows, not the launched W, which NMC_WAVES may
  // override), so every sum stays independent of the wave count.  The A/B knob
  // NMC_TILE_BALANCE=0 (64-row tiles) changes sums and exists in diagnostic builds only.
  bool balance = true;
#ifdef NMC_DEBUG_KNOBS
  if (getenv("NMC_TILE_BALANCE") && !atoi(getenv("NMC_TILE_BALANCE"))) balance = false;
#endif
  if (x->pooling != NMC_POOL_PARTIAL && d.S == 1 && w_rows >= 3 && balance) {
    const int64_t wt = w_rows - 1, n = d.nmax, t64 = (n + 63) / 64;
    if (t64 > wt && t64 < 2 * wt) {
      const int64_t tile = (((n + wt - 1) / wt) + 15) & ~15;
      if (tile <= 128) d.tile = (int)tile;
    }
  }

  // nmc_k_sweep (sweep.h) for partial pooling over more than one numpy leaf (G > 128, at
  // most 4 leaves; cfg 4) with the groups' rows in LDS, no row split and a built-in family:
  // RB * P Gibbs workgroups compute each Gibbs task once per chain block (SYNC_OWN), off the
  // likelihood workgroups' critical path -- 31 against nmc_k_run's 52 us/iter at the cfg-4
  // shard (profiles/r04q_cfg4_gsep.jsonl, profiles/r05).  Up to 12 waves per workgroup
  // (three per SIMD, <= 168 VGPRs), 4 when the grid needs two or three workgroups per CU.
  // NMC_SWEEP=0 keeps nmc_k_run.  (The sweep's other modes -- none/complete pooling and
  // G <= 128 -- measured slower than nmc_k_run, profiles/r04m_sweep_vs_run.jsonl, and were
  // removed in round 5.)
  x->sweep = false;
  d.gsep = 0;
  const bool sweep_want = x->pooling == NMC_POOL_PARTIAL && d.G > 128 && d.nleaf <= 4 &&
                          x->family < NMC_LL_USER_BASE &&
                          !(getenv("NMC_SWEEP") && !atoi(getenv("NMC_SWEEP")));
  if (d.rows_lds && d.S == 1 && !x->no_sweep && sweep_want) {
    // (a multiple of four waves: a workgroup's waves spread evenly over the four SIMDs, so
    // two or three 4-wave workgroups per CU are resident whenever the occupancy API says so)
    const int64_t wgs = (int64_t)d.RB * d.G + (int64_t)d.RB * d.P;
    int sw = wgs <= x->ncu ? NMC_SWEEP_THREADS / 64 : 4;
    if (const char* e = getenv("NMC_SWEEP_WAVES")) {
      const int v = atoi(e);
      if (v >= 3 && v <= NMC_SWEEP_THREADS / 64) sw = v;
    }
    // a control, a Gibbs and at least one likelihood wave, all resident (in resident batches
    // of chain blocks if need be, with the Gibbs workgroups as their own kernel: nmc_create)
    x->sweep = true;
    d.W = sw;
    // the count of a publication is the start of the Gibbs workgroups' update, which every
    // step two later waits for -- count it before the control's first tile (cfg-4 shard
    // 30.8 vs 32.4 us/iter, profiles/r04u_ab.txt)
    d.pubearly = 1;
    if (const char* e = getenv("NMC_PUB_EARLY")) d.pubearly = atoi(e) != 0;
    // (the Gibbs workgroups go into their own kernel, Dev.gsep, only when the one grid
    // cannot be resident: nmc_create; NMC_GSEP=1 forces it)
    if (getenv("NMC_GSEP")) d.gsep = atoi(getenv("NMC_GSEP")) != 0;
  }
}

// numpy's pairwise-sum recursion over G groups (numpy/_core/src/umath/loops_utils.h):
// leaves of <= 128 elements in order, and the post-order merges of their sums.
static int pairwise_plan(int s, int n, std::vector<int>& starts, std::vector<int>& merges) {
  if (n <= 128) {
    starts.push_back(s);
    return (int)starts.size() - 1;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  const int a = pairwise_plan(s, n2, starts, merges);
  const int b = pairwise_plan(s + n2, n - n2, starts, merges);
  merges.push_back(a);
  merges.push_back(b);
  return a;
}

// Gibbs update after iteration t alone (closes a chunk in launch-per-iteration mode).
static int launch_hyper(nmc_ctx* x, int t) {
  std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
  if (x->ktiming) {
    if (int rc = pop_event_pair(x, x->hev, x->hev_used, &ev)) return rc;
    HIPCHK(hipEventRecord(ev->first, x->stream));
  }
  const Dev& d = x->d;
  const size_t lds = (size_t)nmc_lds(0, d.P, 1, d.nleaf, d.ntail, 0, d.G, 0).total * 512;
  hipLaunchKernelGGL(nmc_k_hyper, dim3(d.RB), dim3(64 * d.W), lds, x->stream, x->d,
                     (const double*)vslot(x, t & 1), t);
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev->second, x->stream));
  return 0;
}

// publish counters [RB <= ceil(C / 32)][P][8 shards][32]
static size_t cnt_bytes(const nmc_ctx* x) {
  return (size_t)32 * 8 * ((x->C + 31) / 32) * x->P * sizeof(unsigned);
}

// The timeout word lives in coherent pinned host memory mapped into the device: the
// kernels' (rare) system-scope store lands in host memory, so the host reads it with a
// plain load after a synchronize -- no device-to-host copy on every synchronize.
// nmc_k_sweep's hyper-ready counters [RB <= ceil(C / 32)][P][32]
static size_t hrd_words(const nmc_ctx* x) { return (size_t)32 * ((x->C + 31) / 32) * x->P; }
// Dev.gsep role words [RB <= ceil(C / 32)][16] (u64, one 128-B line per chain block)
static size_t grole_words(const nmc_ctx* x) { return (size_t)16 * ((x->C + 31) / 32); }

static int check_timeout(nmc_ctx* x) {
  if (*x->tmo_host)
    return fail(-5, "persistent kernel: a chain-block wait timed out (workgroups not resident?)");
  return 0;
}

// ---------------------------------------------------------------------------
// Variate fill.  nmc_run draws a chunk's variates (nmc_k_fill) before its step launch; the
// two variate buffers let the fill of the NEXT chunk -- the rest of the call, or the same
// length after it, the next call of a sampling loop -- run on pstream beside the step
// launch that reads the other buffer (a prefill).  A chunk starting where the pending
// prefill starts takes its iterations and fills only what is missing; any other chunk waits
// for the prefill's writes and fills its own.  The variates are a function of (seed,
// chain, iteration, ...) alone, so where they are drawn never changes a bit.
// ---------------------------------------------------------------------------
// iterations per step launch: launch_iters, at most a buffer's capacity
static int fill_chunk(const nmc_ctx* x) {
  return x->launch_iters > 0 && x->launch_iters < x->d.vcap ? x->launch_iters : x->d.vcap;
}
// fill elements of T iterations (nmc_k_sweep with Dev.zin draws every variate itself; the
// step kernels with Dev.zin draw the step variates)
static size_t fill_elements(const nmc_ctx* x, int T) {
  if (x->sweep && x->d.zin) return 0;
  const bool partial = x->pooling == NMC_POOL_PARTIAL;
  return (size_t)T * x->P * x->C * ((x->d.zin ? 0 : x->G) + (partial ? 1 : 0));
}
// nmc_k_fill of iterations [a, b) into buffer buf, whose first iteration is vb (beside: the
// instance whose waves fit beside a resident step launch's, kernels_misc.h NMC_FILL_RES_MINB)
static int launch_fill(nmc_ctx* x, int buf, int vb, int a, int b, hipStream_t s, int bpc,
                       bool beside = false) {
  const size_t n = fill_elements(x, b - a);
  if (!n) return 0;
  Dev df = x->d;
  df.vzl = x->vzlb[buf] + (size_t)(a - vb) * 2 * x->P * x->G * x->C;
  df.vh = x->vhb[buf] + (size_t)(a - vb) * 2 * x->P * x->C;
  df.vbase = a;
  // a resident grid walking the elements (kernels_misc.h): bpc blocks per CU
  const int64_t cap = (int64_t)bpc * x->ncu;
  const int blocks = (int)std::min<int64_t>((int64_t)((n + 255) / 256), cap);
  if (x->rng == NMC_RNG_REPLAY)
    hipLaunchKernelGGL(nmc_k_fill<true>, dim3(blocks), dim3(256), 0, s, df, a, b - a);
  else if (beside && x->res.fill_minb == 4)
    hipLaunchKernelGGL((nmc_k_fill<false, 4>), dim3(blocks), dim3(256), 0, s, df, a, b - a);
  else if (beside && x->res.fill_minb == 5)
    hipLaunchKernelGGL((nmc_k_fill<false, 5>), dim3(blocks), dim3(256), 0, s, df, a, b - a);
  else if (beside && x->res.fill_minb == 6)
    hipLaunchKernelGGL((nmc_k_fill<false, 6>), dim3(blocks), dim3(256), 0, s, df, a, b - a);
  else if (beside && x->res.fill_minb == 8)
    hipLaunchKernelGGL((nmc_k_fill<false, 8>), dim3(blocks), dim3(256), 0, s, df, a, b - a);
  else
    hipLaunchKernelGGL(nmc_k_fill<false>, dim3(blocks), dim3(256), 0, s, df, a, b - a);
  HIPCHK(hipGetLastError());
  return 0;
}
// prefill of iterations [a, b) (at most a buffer) into the buffer the latest chunk does not
// read, once the last step launch reading it is done; replaces a pending prefill
static int enqueue_prefill(nmc_ctx* x, int a, int b) {
  b = std::min(b, a + x->d.vcap);
  const int buf = x->vbuf ^ 1;
  HIPCHK(hipStreamWaitEvent(x->pstream, x->rd_ev[buf], 0));
  if (int rc = launch_fill(x, buf, a, a, b, x->pstream, x->prefill_bpc)) return rc;
  HIPCHK(hipEventRecord(x->pf_ev, x->pstream));
  x->pf.valid = true;
  x->pf.i0 = a;
  x->pf.i1 = b;
  x->pf.buf = buf;
  x->pf.vb = a;
  x->pf_issued += b - a;
  return 0;
}

// Diagnostics (NMC_TRACE_CALLS=1): host time of nmc_run's / nmc_synchronize's phases, one
// line per call on stderr (microseconds since the call's entry).
static const bool g_trace_calls = [] {
  const char* e = getenv("NMC_TRACE_CALLS");
  return e && atoi(e) != 0;
}();
struct nmc_call_trace {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  char buf[256];
  int n = 0;
  explicit nmc_call_trace(const char* nm) : name(nm) { buf[0] = 0; }
  void mark(const char* what) {
    if (!g_trace_calls) return;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    n += snprintf(buf + n, sizeof(buf) - n > 0 ? sizeof(buf) - n : 0, " %s %.2f", what, us);
  }
  ~nmc_call_trace() {
    if (g_trace_calls) fprintf(stderr, "[nmc trace] %s:%s\n", name, buf);
  }
};

// ---------------------------------------------------------------------------
// Resident launch (nmc_set_resident).  A call of a sampling loop that continues where the
// resident launch's last call ended, fits its variate buffer and finds its variates
// prefilled there is handed to the running launch as a command (pinned host memory) instead
// of a new launch: no dispatch, no prologue (rows and chain state stay in LDS), no closing
// beyond the call's own.  Each call is still closed completely at its end (kernels.h
// res_gate): when nmc_synchronize returns, its sample rows, hyper-parameters and state are
// in HBM exactly as after a launch of that call.  Every other entry point parks the launch
// first; workgroup 0 parks it by itself after NMC_RESIDENT_IDLE_US (20 ms) without a call.
// ---------------------------------------------------------------------------
static bool res_kernel_gone(nmc_ctx* x) { return hipStreamQuery(x->stream) == hipSuccess; }

// wait until every workgroup reported the latest seq done; record the call's GPU span
static int res_wait_done(nmc_ctx* x) {
  auto& r = x->res;
  if (!r.active || r.done == r.seq) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned long spins = 0;; ++spins) {
    if (r.done_w[0] == r.seq) break;
    if ((spins & 1023) == 1023) {
      if (*x->tmo_host) {
        r.active = false;
        hipStreamSynchronize(x->stream);
        return check_timeout(x);
      }
      if (res_kernel_gone(x)) {
        r.active = false;
        return fail(-5, "resident launch ended before its call completed");
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100))
        std::this_thread::yield();
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  // GPU span: workgroup 0 taking the command -> the last workgroup done (s_memrealtime)
  if (r.ack[0] == r.seq) {
    auto clk = [&](int j) {
      return ((unsigned long long)r.done_w[3 + 2 * j] << 32) | r.done_w[2 + 2 * j];
    };
    const unsigned long long a = ((unsigned long long)r.ack[3] << 32) | r.ack[2];
    const unsigned long long e = clk(0), le = clk(1), st = clk(2);
    r.spans.emplace_back(r.seq, e >= a ? (double)(e - a) / 1e5 : -1.0);
    if (g_trace_calls)   // (the critical path: the last workgroup to start, to end its loop)
      fprintf(stderr, "[nmc trace] resident call %u: relay %.2f loop %.2f close %.2f us; host "
              "post -> done seen %.2f us\n",
              r.seq, ((double)st - (double)a) / 100.0, ((double)le - (double)st) / 100.0,
              ((double)e - (double)le) / 100.0,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() -
                                                        r.t_post).count());
    if (r.spans.size() > 64) r.spans.erase(r.spans.begin(), r.spans.begin() + 32);
  }
  r.done = r.seq;
  return 0;
}

// end the resident launch (park command) and wait for it (its pending prefill stays: a
// launch starting there reads it at its offset, Dev.vbase = pf.vb)
static int res_park(nmc_ctx* x) {
  auto& r = x->res;
  if (!r.active) return 0;
  hipSetDevice(x->device);
  const unsigned seq = r.seq + 1;
  *r.cmd = (0xffffffffull << 32) | seq;
  r.seq = seq;
  r.done = seq;
  r.active = false;
  HIPCHK(hipStreamSynchronize(x->stream));
  return check_timeout(x);
}
#define RES_PARK(x)                          \
  do {                                       \
    if (int rc_ = res_park(x)) return rc_;   \
  } while (0)

// prefill of iterations [a, b) into the resident launch's buffer, at their offset from its
// first iteration (the launch reads other iterations of the same buffer: no wait)
static int res_prefill(nmc_ctx* x, int a, int b) {
  auto& r = x->res;
  b = std::min(b, r.vbase + x->d.vcap);
  if (b <= a) return 0;
  if (int rc = launch_fill(x, r.buf, r.vbase, a, b, x->pstream, x->prefill_bpc, true)) return rc;
  HIPCHK(hipEventRecord(x->pf_ev, x->pstream));
  x->pf.valid = true;
  x->pf.i0 = a;
  x->pf.i1 = b;
  x->pf.buf = r.buf;
  x->pf.vb = r.vbase;
  x->pf_issued += b - a;
  return 0;
}

// nmc_run's iterations [i0, i1) as the resident launch's next call: 1 taken, 0 not
// possible (the launch is parked: the caller launches), < 0 error
static int res_continue(nmc_ctx* x, int i0, int i1) {
  auto& r = x->res;
  // why a call is not continued (nmc_resident_stats): 1 another start, 2 kernel timing,
  // 3 longer than a chunk, 4 past the launch's variate buffer, 5 its variates not prefilled
  // there, 6 the counters would wrap, 7 the launch had parked itself (idle)
  const int why = i0 != r.end ? 1 : x->ktiming ? 2 : i1 - i0 > fill_chunk(x) ? 3
                : i1 - r.vbase > x->d.vcap ? 4
                : !(x->pf.valid && x->pf.buf == r.buf && x->pf.i0 == i0 && x->pf.i1 >= i1) ? 5
                : ((uint64_t)x->G * (x->d.pbase + (uint64_t)(i1 - i0)) >= (1ull << 31) ||
                   (uint64_t)x->d.S * (x->d.xbase + (uint64_t)(i1 - i0) * x->P) >= (1ull << 31))
                    ? 6 : 0;
  if (why) {
    r.why = why;
    RES_PARK(x);
    return 0;
  }
  const auto t_in = std::chrono::steady_clock::now();
  if (int rc = res_wait_done(x)) return rc;
  const auto t_wd = std::chrono::steady_clock::now();
  // the call's variates have landed (the prefill runs beside the launch, which it fits:
  // nmc_set_resident); a prefill not done within 2 ms parks the launch rather than wait
  // for its idle limit -- whatever held the fill back, it cannot start beside the launch
  {
    const auto tq = std::chrono::steady_clock::now();
    while (hipEventQuery(x->pf_ev) != hipSuccess) {
      if (std::chrono::steady_clock::now() - tq > std::chrono::milliseconds(2)) {
        // (kernels serialized -- a profiler's counter pass does it -- or no room beside the
        //  launch: later calls launch as they would without nmc_set_resident)
        r.why = 8;
        r.on = false;
        RES_PARK(x);
        return 0;
      }
      std::this_thread::yield();
    }
  }
  const unsigned seq = r.seq + 1;
  const auto t_post = std::chrono::steady_clock::now();
  *r.cmd = ((unsigned long long)(unsigned)i1 << 32) | seq;
  std::atomic_thread_fence(std::memory_order_seq_cst);   // (out of the store buffer now)
  r.seq = seq;
  r.t_post = t_post;
  // taken, or workgroup 0 parked (idle) before it saw the command
  for (unsigned long spins = 0;; ++spins) {
    if (r.ack[0] == seq) {
      if (g_trace_calls) {
        auto us = [&](std::chrono::steady_clock::time_point t) {
          return std::chrono::duration<double, std::micro>(t - t_in).count();
        };
        fprintf(stderr, "[nmc trace] resident call %u: host done-wait %.2f prefill-query %.2f "
                "ack seen %.2f us\n", seq, us(t_wd), us(t_post),
                us(std::chrono::steady_clock::now()));
      }
      break;
    }
    if (r.ack[1] == (0x80000000u | (seq - 1))) {
      r.why = 7;
      r.done = seq;
      r.active = false;
      HIPCHK(hipStreamSynchronize(x->stream));
      if (int rc = check_timeout(x)) return rc;
      return 0;
    }
    if ((spins & 1023) == 1023) {
      if (*x->tmo_host) return check_timeout(x);
      if (res_kernel_gone(x) && r.ack[0] != seq &&
          r.ack[1] != (0x80000000u | (seq - 1))) {
        r.active = false;
        return fail(-5, "resident launch ended without taking or refusing a call");
      }
    }
  }
  x->pf_used += i1 - i0;
  x->pf.valid = false;
  r.end = i1;
  r.calls += 1;
  x->d.pbase += (unsigned)(i1 - i0);
  x->d.xbase += (unsigned)((i1 - i0) * x->P);
  x->cur_slot = (i1 - 1) & 1;
  // the next call's variates beside this one (the same length, while the schedule and the
  // buffer last; NMC_RES_PREFILL=0, diagnostics: none -- the next call then launches anew)
  static const bool res_prefill_on = !(getenv("NMC_RES_PREFILL") && !atoi(getenv("NMC_RES_PREFILL")));
  if (x->prefill_on && res_prefill_on) {
    const int n1 = std::min({i1 + (i1 - i0), x->n_iter, r.vbase + x->d.vcap});
    if (n1 > i1)
      if (int rc = res_prefill(x, i1, n1)) return rc;
  }
  return 1;
}

// ---------------------------------------------------------------------------
extern "C" {

const char* nmc_last_error(void) { return g_err.c_str(); }
const char* nmc_version(void) { return NMC_VERSION; }

int nmc_device_count(int* n) {
  int k = 0;
  hipError_t e = hipGetDeviceCount(&k);
  if (e != hipSuccess) k = 0;
  *n = k;
  return 0;
}

int nmc_create(nmc_ctx** out, int device, int n_chains, int chain_base, int n_groups,
               int n_params, int pooling, int ll_family, const double* ll_consts,
               int n_ll_consts, const int64_t* group_offsets, const double* obs,
               int64_t n_obs, int n_fields, const int* prior_family,
               const double* prior_params, uint32_t seed, int rng_mode) {
  *out = nullptr;
  if (n_chains < 1 || n_groups < 1 || n_params < 1 || n_params > NMC_MAXP)
    return fail(-1, "need n_chains >= 1, n_groups >= 1, 1 <= n_params <= 16");
  if (pooling < 0 || pooling > 2) return fail(-1, "invalid pooling");
  if (pooling == NMC_POOL_PARTIAL && n_groups < 2)
    return fail(-1, "partial pooling needs at least 2 groups (invgamma shape (G-1)/2 > 0)");
  if (n_fields < 1 || n_fields > 9) return fail(-1, "n_fields must be 1..9");
  if (group_offsets[0] != 0 || group_offsets[n_groups] != n_obs)
    return fail(-1, "group_offsets must start at 0 and end at n_obs");
  for (int g = 0; g < n_groups; ++g)
    if (group_offsets[g + 1] < group_offsets[g]) return fail(-1, "group_offsets not monotone");
  if (pooling != NMC_POOL_PARTIAL && (!prior_family || !prior_params))
    return fail(-1, "none/complete pooling needs priors");
  if (ll_family == NMC_LL_GAUSS_MEAN && n_fields != n_params)
    return fail(-1, "gauss_mean: n_fields must equal n_params");
  if (ll_family == NMC_LL_GAUSS_MEAN && n_ll_consts < 2 * n_fields)
    return fail(-1, "gauss_mean consts = {sd[P], log sd[P]}");
  if ((ll_family == NMC_LL_LINREG || ll_family == NMC_LL_LOGISTIC) && n_ll_consts < 3)
    return fail(-1, "linreg/logistic consts = {k, intercept, sigma, log sigma}");
  if (ll_family == NMC_LL_LINREG) {
    const int need = (n_fields - 1) + (int)ll_consts[1] + (ll_consts[2] > 0 ? 0 : 1);
    if (need != n_params) return fail(-1, "linreg: n_params != k + intercept + (sigma sampled)");
  }
  if (ll_family == NMC_LL_LOGISTIC && (n_fields - 1) + (int)ll_consts[1] != n_params)
    return fail(-1, "logistic: n_params != k + intercept");
  if (ll_family >= NMC_LL_USER_BASE) {
    int unf = 0, unp = 0;
    if (int rc0 = nmc_user_family_shape(ll_family, &unf, &unp)) return rc0;
    if (unf != n_fields || unp != n_params)
      return fail(-1, "user family compiled for other n_fields / n_params");
  } else if (ll_family < 0 || ll_family > NMC_LL_LOGISTIC) {
    return fail(-1, "unknown likelihood family");
  }

  nmc_ctx* x = new nmc_ctx();
  x->device = device;
  x->C = n_chains; x->chain_base = chain_base; x->G = n_groups; x->P = n_params;
  x->pooling = pooling; x->family = ll_family; x->nf = n_fields; x->seed = seed;
  x->rng = rng_mode; x->n_obs = n_obs;
  x->llc.assign(ll_consts, ll_consts + n_ll_consts);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete x; return fail(-2, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
  e = hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking);
  if (e != hipSuccess) { nmc_destroy(x); return fail(-2, std::string("hipStreamCreate: ") + hipGetErrorString(e)); }
  for (auto& ev : x->ev) hipEventCreate(&ev);
  e = hipStreamCreateWithFlags(&x->gstream, hipStreamNonBlocking);
  if (e != hipSuccess) { nmc_destroy(x); return fail(-2, std::string("hipStreamCreate: ") + hipGetErrorString(e)); }
  for (auto& ev : x->gev) hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  e = hipStreamCreateWithFlags(&x->pstream, hipStreamNonBlocking);
  if (e != hipSuccess) { nmc_destroy(x); return fail(-2, std::string("hipStreamCreate: ") + hipGetErrorString(e)); }
  hipEventCreateWithFlags(&x->pf_ev, hipEventDisableTiming);
  for (auto& ev : x->rd_ev) {   // (recorded on the empty stream: complete)
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipEventRecord(ev, x->stream);
  }

  Dev& d = x->d;
  const size_t PGC = (size_t)n_params * n_groups * n_chains, GC = (size_t)n_groups * n_chains,
               PC = (size_t)n_params * n_chains;
  int rc = 0;
  int64_t* off = nullptr;
  double* dobs = nullptr;
  int* pf = nullptr;
  double* pp = nullptr;
  rc |= dalloc(x, &off, n_groups + 1);
  rc |= dalloc(x, &dobs, (size_t)n_obs * n_fields + 4);   // (+32 B: staged-row DMA slack)
  rc |= dalloc(x, &pf, n_params);
  rc |= dalloc(x, &pp, (size_t)8 * n_params);
  // (+72 C + 128 slack: the Gibbs wave reads 72 groups' values unconditionally, and the
  // payload copies read whole 64-chain rows of the last group)
  rc |= dalloc(x, &d.vb0, PGC + (size_t)72 * n_chains + 128);
  rc |= dalloc(x, &d.vb1, PGC + (size_t)72 * n_chains + 128);
  rc |= dalloc(x, &d.lp, PGC);
  rc |= dalloc(x, &d.ll, GC);
  rc |= dalloc(x, &d.scale, PGC);
  rc |= dalloc(x, &d.nacc, PGC);
  rc |= dalloc(x, &d.nrej, PGC);
  rc |= dalloc(x, &d.tacc, PGC);
  // hyper-parameters after iteration t live in slot t & 1 ([2][P][C]), like the values
  rc |= dalloc(x, &d.mu, 2 * PC);
  rc |= dalloc(x, &d.s2, 2 * PC);
  rc |= dalloc(x, &d.hsd, 2 * PC);
  rc |= dalloc(x, &d.hlsd, 2 * PC);
  if (rc) { nmc_destroy(x); return rc; }
  d.off = off; d.obs = dobs; d.pfam = pf; d.ppar = pp;
  d.C = n_chains; d.G = n_groups; d.P = n_params; d.pooling = pooling; d.nf = n_fields;
  d.chain_base = chain_base; d.rng_mode = rng_mode; d.seed = seed;
  d.CB = (n_chains + 63) / 64;
  d.ha = (n_groups - 1) / 2.0;
  d.hlga = lgamma(d.ha > 0 ? d.ha : 1.0);
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      x->ncu = prop.multiProcessorCount;
  }
  x->nacc = ll_family == NMC_LL_GAUSS_MEAN ? n_fields : 1;
  if (ll_family >= NMC_LL_USER_BASE) {   // runtime-compiled family: module + constants
    if (int rc0 = nmc_user_attach(x, ll_family)) { nmc_destroy(x); return rc0; }
    if (n_ll_consts > 0) {
      if (int rc0 = dalloc(x, &x->user_k, (size_t)n_ll_consts)) { nmc_destroy(x); return rc0; }
      HIPCHK(hipMemcpy(x->user_k, ll_consts, (size_t)n_ll_consts * 8, hipMemcpyHostToDevice));
    }
  }
  // numpy pairwise-sum plan of the hyper update (partial pooling)
  std::vector<int> starts, merges;
  pairwise_plan(0, n_groups, starts, merges);
  int ntail = 0;
  for (size_t k = 0; k < starts.size(); ++k) {
    const int m = (k + 1 < starts.size() ? starts[k + 1] : n_groups) - starts[k];
    const int m8 = m >= 8 ? m - m % 8 : 0;
    ntail = std::max(ntail, m - m8);
  }
  starts.push_back(n_groups);
  d.nleaf = (int)starts.size() - 1;
  d.nmerge = (int)merges.size() / 2;
  d.ntail = ntail;
  int* dleaf = nullptr;
  int* dmerge = nullptr;
  rc |= dalloc(x, &dleaf, starts.size());
  rc |= dalloc(x, &dmerge, merges.size());
  // [RB][P][8 shards][32], RB <= ceil(C / 32)
  rc |= dalloc(x, &d.cnt, cnt_bytes(x) / sizeof(unsigned));
  rc |= dalloc(x, &d.hrd, hrd_words(x));
  // Dev.gsep role words [RB <= ceil(C / 32)][16] and the fallback count
  rc |= dalloc(x, &d.grole, grole_words(x));
  rc |= dalloc(x, &d.gfb, 32);
  if (rc) { nmc_destroy(x); return rc; }
  {
    void* h = nullptr;
    void* dp = nullptr;
    e = hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) x->tmo_host = (volatile unsigned*)h;
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, h, 0);
    if (e != hipSuccess) {
      nmc_destroy(x);
      return fail(-2, std::string("timeout word (pinned host memory): ") + hipGetErrorString(e));
    }
    memset(h, 0, 64);
    d.tmo = (unsigned*)dp;
  }
  HIPCHK(hipMemset(d.cnt, 0, cnt_bytes(x)));
  HIPCHK(hipMemset(d.hrd, 0, hrd_words(x) * sizeof(unsigned)));
  HIPCHK(hipMemset(d.grole, 0, grole_words(x) * sizeof(unsigned long long)));
  HIPCHK(hipMemset(d.gfb, 0, 32 * sizeof(unsigned)));
  d.pbase = d.xbase = 0;
  // Dev.gsep: how long the two kernels may take to meet before the likelihood workgroups take
  // a launch's Gibbs tasks over (NMC_GSEP_PATIENCE_US, default 20 ms: 2 ms was sometimes too
  // short for the Gibbs kernel to be dispatched beside a running step kernel and the variate
  // fill, and a launch fell back while both kernels ran -- the same results, slower);
  // NMC_GSEP_SERIAL (tests) serializes them on one stream
  d.gep = 0;
  d.gpat = 2000000u;
  if (const char* e = getenv("NMC_GSEP_PATIENCE_US")) d.gpat = (unsigned)(atol(e) * 100);
  x->gserial = getenv("NMC_GSEP_SERIAL") ? atoi(getenv("NMC_GSEP_SERIAL")) : 0;
  // nmc_k_fill's grid: 3 blocks of 256 per CU (its Philox instance's 140 VGPRs: three waves
  // per SIMD); NMC_FILL_BPC overrides (A/B)
  x->fill_bpc = getenv("NMC_FILL_BPC") ? std::max(1, atoi(getenv("NMC_FILL_BPC"))) : 3;
  // the pipelined fill beside a step kernel: one block per CU (one wave per SIMD next to the
  // step kernel's), NMC_PREFILL_BPC overrides; NMC_PREFILL=0 turns the pipelining off (A/B)
  x->prefill_bpc = getenv("NMC_PREFILL_BPC") ? std::max(1, atoi(getenv("NMC_PREFILL_BPC"))) : 1;
  x->prefill_on = !(getenv("NMC_PREFILL") && atoi(getenv("NMC_PREFILL")) == 0);
  d.leaf = dleaf;
  d.merge = dmerge;
  HIPCHK(hipMemcpy(dleaf, starts.data(), starts.size() * sizeof(int), hipMemcpyHostToDevice));
  if (!merges.empty())
    HIPCHK(hipMemcpy(dmerge, merges.data(), merges.size() * sizeof(int), hipMemcpyHostToDevice));
  int64_t nmax = 0;
  for (int g = 0; g < n_groups; ++g)
    nmax = std::max<int64_t>(nmax, group_offsets[g + 1] - group_offsets[g]);
  x->nmax_group = nmax;
  // Row split: groups far larger than one workgroup's 64 KiB LDS row area are shared by S
  // workgroups, at most 64 and at most one per CU of a full MI355X (256 CUs) per group.
  // S depends on (rows, fields, groups) only -- never on the chain count or on the
  // device's CU count -- so the partial-sum order, and every result, is the same whatever
  // the sharding, the launch batching or the GPU partition (a partition too small to
  // hold the S members of one group at once refuses the run: nmc_create below).
  d.S = 1;
  d.cb0 = 0;
  {
    const int64_t target = std::max<int64_t>(256, (64 * 1024) / (n_fields * 8));
    if (nmax > 2 * target)
      d.S = (int)std::min<int64_t>({64, (nmax + target - 1) / target,
                                    std::max<int64_t>(1, NMC_SPLIT_CU_BASIS / n_groups)});
#ifdef NMC_DEBUG_KNOBS   // (diagnostic builds only: changes the summation order)
    if (const char* e = getenv("NMC_SPLIT")) {
      const int v = atoi(e);
      if (v >= 1 && v <= 256) d.S = v;
    }
#endif
  }
  d.nmax = (int)((nmax + d.S - 1) / d.S);   // rows of the largest member
  choose_geometry(x);
  if (run_lds_bytes(x) > (size_t)160 * 1024) {
    nmc_destroy(x);
    return fail(-1, "workgroup state exceeds the 160 KiB LDS of a CU (too many parameters, "
                    "groups or rows per group)");
  }
  if (pooling == NMC_POOL_PARTIAL) {
    NmcCall c;
    c.op = NMC_OP_CAN_PERSIST;
    if (int rc2 = nmc_call_family(x, c)) { nmc_destroy(x); return rc2; }
    if (x->sweep && c.result != 1 && run_mode(x) == NMC_MODE_SYNC_OWN && !d.gsep &&
        x->family < NMC_LL_USER_BASE && !getenv("NMC_GSEP")) {
      // the likelihood and Gibbs workgroups in one grid do not fit: two kernels, one per
      // stream (nmc_k_sweep + nmc_k_sweep_gibbs), each workgroup with its own LDS size
      d.gsep = 1;
      if (int rc2 = nmc_call_family(x, c)) { nmc_destroy(x); return rc2; }
    }
    if (x->sweep && c.result != 1) {   // the sweep grid cannot be resident: nmc_k_run
      x->no_sweep = true;
      choose_geometry(x);
      if (int rc2 = nmc_call_family(x, c)) { nmc_destroy(x); return rc2; }
    }
    // row split: always persistent (the members exchange every step), in resident batches
    // of chain blocks when the whole grid is not (chain blocks are independent)
    x->persistent = c.result == 1 || d.S > 1;
  }
  // XCD-aware placement of nmc_k_run's persistent partial-pooling grid (Dev.xpc, NMC_XMAP=1):
  // the RB chain blocks on 8 / RB XCDs each, when RB divides 8 and the groups split evenly.
  // Measured 1.5-2.5 % slower at cfg 3 than chain-block-major (profiles/r06/r06n_*): off
  d.xpc = 0;
  if (pooling == NMC_POOL_PARTIAL && x->persistent && !x->sweep && d.S == 1 && d.RB <= 8 &&
      8 % d.RB == 0 && n_groups % (8 / d.RB) == 0 && getenv("NMC_XMAP") &&
      atoi(getenv("NMC_XMAP")) == 1)
    d.xpc = 8 / d.RB;
  if (d.S > 1) {   // row split: resident batches of chain blocks, exchange buffers
    NmcCall c;
    c.op = NMC_OP_CAPACITY;
    if (int rc2 = nmc_call_family(x, c)) { nmc_destroy(x); return rc2; }
    const int64_t per_cb = (int64_t)d.G * d.S;
    if (c.result < per_cb) {
      nmc_destroy(x);
      return fail(-1, "row split: the S workgroups of one group are not co-resident");
    }
    x->split_batch = (int)std::min<int64_t>(d.RB, c.result / per_cb);
    if (const char* e = getenv("NMC_SPLIT_BATCH")) {
      const int v = atoi(e);
      if (v >= 1 && v < x->split_batch) x->split_batch = v;
    }
    rc |= dalloc(x, &d.xbuf, (size_t)2 * d.RB * d.G * d.S * x->nacc * 64);
    rc |= dalloc(x, &d.xcnt, (size_t)d.RB * d.G * 32);
    if (rc) { nmc_destroy(x); return rc; }
    HIPCHK(hipMemset(d.xcnt, 0, (size_t)d.RB * d.G * 32 * sizeof(unsigned)));
  }
  // build option NMC_ZIN_BUILD=1: the step kernel draws its {z, log u} itself (a job in
  // each step's tile queue) unless the opt-in one-barrier kernel runs (it DMAs them from
  // the fill's ring); NMC_ZIN=0 keeps the fill (bit-identical; tests compare them)
  d.zin = NMC_ZIN_BUILD &&
          !(getenv("NMC_ZIN") && !atoi(getenv("NMC_ZIN")));
  // nmc_k_sweep: every variate drawn in the kernel (NMC_ZIN=1) or from the fill's ring
  if (x->sweep) d.zin = getenv("NMC_ZIN") ? (atoi(getenv("NMC_ZIN")) != 0) : 0;
  d.thin = 1; d.tune_interval = 100;
  HIPCHK(hipMemcpy(off, group_offsets, (n_groups + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (n_obs > 0)
    HIPCHK(hipMemcpy(dobs, obs, (size_t)n_obs * n_fields * sizeof(double), hipMemcpyHostToDevice));
  if (prior_family) HIPCHK(hipMemcpy(pf, prior_family, n_params * sizeof(int), hipMemcpyHostToDevice));
  if (prior_params) HIPCHK(hipMemcpy(pp, prior_params, 8 * n_params * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(d.nacc, 0, PGC * sizeof(int)));
  HIPCHK(hipMemset(d.nrej, 0, PGC * sizeof(int)));
  HIPCHK(hipMemset(d.tacc, 0, PGC * sizeof(long long)));
  std::vector<double> ones(PGC, 1.0);
  HIPCHK(hipMemcpy(d.scale, ones.data(), PGC * sizeof(double), hipMemcpyHostToDevice));
  *out = x;
  return 0;
}

int nmc_destroy(nmc_ctx* x) {
  if (!x) return 0;
  hipSetDevice(x->device);
  res_park(x);
  if (x->stream) hipStreamSynchronize(x->stream);
  if (x->gstream) hipStreamSynchronize(x->gstream);
  if (x->pstream) hipStreamSynchronize(x->pstream);
  for (void* p : x->owned) if (p) hipFree(p);
  for (auto& ev : x->ev) if (ev) hipEventDestroy(ev);
  for (auto& pr : x->kev) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  for (auto& pr : x->hev) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  for (auto& ev : x->gev) if (ev) hipEventDestroy(ev);
  if (x->pf_ev) hipEventDestroy(x->pf_ev);
  for (auto& ev : x->rd_ev) if (ev) hipEventDestroy(ev);
  if (x->pstream) hipStreamDestroy(x->pstream);
  if (x->gstream) hipStreamDestroy(x->gstream);
  if (x->stream) hipStreamDestroy(x->stream);
  if (x->tmo_host) hipHostFree((void*)x->tmo_host);
  if (x->res.host) hipHostFree(x->res.host);
  delete x;
  return 0;
}

int nmc_set_state(nmc_ctx* x, const double* value, const double* log_prior, const double* ll,
                  const double* hyper_mu, const double* hyper_sigma2, const double* scale) {
  RES_PARK(x);
  hipSetDevice(x->device);
  Dev& d = x->d;
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C, PC = (size_t)x->P * x->C;
  HIPCHK(hipMemcpy(d.vb1, value, PGC * 8, hipMemcpyHostToDevice));
  x->cur_slot = 1;
  HIPCHK(hipMemcpy(d.lp, log_prior, PGC * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d.ll, ll, GC * 8, hipMemcpyHostToDevice));
  if (x->pooling == NMC_POOL_PARTIAL) {
    if (!hyper_mu || !hyper_sigma2) return fail(-1, "partial pooling needs hyper_mu/hyper_sigma2");
    std::vector<double> sd(PC), lsd(PC);
    for (size_t i = 0; i < PC; ++i) { sd[i] = sqrt(hyper_sigma2[i]); lsd[i] = log(sd[i]); }
    // the state "after iteration -1" lives in slot 1 (values: vb1)
    HIPCHK(hipMemcpy(d.mu + PC, hyper_mu, PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.s2 + PC, hyper_sigma2, PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.hsd + PC, sd.data(), PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.hlsd + PC, lsd.data(), PC * 8, hipMemcpyHostToDevice));
  }
  if (scale) {
    HIPCHK(hipMemcpy(d.scale, scale, PGC * 8, hipMemcpyHostToDevice));
  } else {
    std::vector<double> ones(PGC, 1.0);
    HIPCHK(hipMemcpy(d.scale, ones.data(), PGC * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(d.nacc, 0, PGC * sizeof(int)));
  HIPCHK(hipMemset(d.nrej, 0, PGC * sizeof(int)));
  HIPCHK(hipMemset(d.tacc, 0, PGC * sizeof(long long)));
  return 0;
}

int nmc_get_state(nmc_ctx* x, double* value, double* log_prior, double* ll, double* hyper_mu,
                  double* hyper_sigma2, double* scale) {
  RES_PARK(x);
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  Dev& d = x->d;
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C, PC = (size_t)x->P * x->C;
  if (value) HIPCHK(hipMemcpy(value, vslot(x, x->cur_slot), PGC * 8, hipMemcpyDeviceToHost));
  if (log_prior) HIPCHK(hipMemcpy(log_prior, d.lp, PGC * 8, hipMemcpyDeviceToHost));
  if (ll) HIPCHK(hipMemcpy(ll, d.ll, GC * 8, hipMemcpyDeviceToHost));
  const size_t ho = (size_t)x->cur_slot * PC;
  if (hyper_mu) HIPCHK(hipMemcpy(hyper_mu, d.mu + ho, PC * 8, hipMemcpyDeviceToHost));
  if (hyper_sigma2) HIPCHK(hipMemcpy(hyper_sigma2, d.s2 + ho, PC * 8, hipMemcpyDeviceToHost));
  if (scale) HIPCHK(hipMemcpy(scale, d.scale, PGC * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_set_replay(nmc_ctx* x, const double* z, const double* u, const double* hz,
                   const double* hu, int n_iter) {
  RES_PARK(x);
  hipSetDevice(x->device);
  Dev& d = x->d;
  const size_t n = (size_t)n_iter * x->P * x->G * x->C, nh = (size_t)n_iter * x->P * x->C;
  double *rz, *ru, *rhz, *rhu;
  // (a pending prefill reads the replay arrays about to be freed; its variates are stale)
  HIPCHK(hipStreamSynchronize(x->pstream));
  x->pf.valid = false;
  dfree(x, (void*)d.rz); dfree(x, (void*)d.ru); dfree(x, (void*)d.rhz); dfree(x, (void*)d.rhu);
  int rc = dalloc(x, &rz, n) | dalloc(x, &ru, n) | dalloc(x, &rhz, nh) | dalloc(x, &rhu, nh);
  if (rc) return rc;
  HIPCHK(hipMemcpy(rz, z, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ru, u, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(rhz, hz, nh * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(rhu, hu, nh * 8, hipMemcpyHostToDevice));
  d.rz = rz; d.ru = ru; d.rhz = rhz; d.rhu = rhu; d.replay_n = n_iter;
  return 0;
}

static int alloc_trace(nmc_ctx* x) {
  Dev& d = x->d;
  dfree(x, d.tflag); dfree(x, d.tllp);
  d.tflag = nullptr; d.tllp = nullptr; d.trace_n = 0;
  if (!x->trace || !x->scheduled) return 0;
  const size_t n = (size_t)x->n_iter * x->P * x->G * x->C;
  int rc = dalloc(x, &d.tflag, n) | dalloc(x, &d.tllp, n);
  if (rc) return rc;
  HIPCHK(hipMemset(d.tflag, 0xff, n));
  d.trace_n = x->n_iter;
  return 0;
}

int nmc_set_schedule(nmc_ctx* x, int n_iter, int burn, int thin, int tune_interval) {
  RES_PARK(x);
  hipSetDevice(x->device);
  if (n_iter < 0 || burn < 0 || burn > n_iter || thin < 1 || tune_interval < 1)
    return fail(-1, "invalid schedule");
  Dev& d = x->d;
  int rows = 0;
  for (int i = burn; i < n_iter; ++i)
    if (i % thin == 0) ++rows;
  d.burn = burn; d.thin = thin; d.tune_interval = tune_interval; d.n_rows = rows;
  d.cols = x->P * (x->G + (x->pooling == NMC_POOL_PARTIAL ? 2 : 0));
  dfree(x, d.samples);
  int rc = dalloc(x, &d.samples, (size_t)rows * d.cols * x->C);
  if (rc) return rc;
  // variate buffers: two chunks of iterations' worth of pre-drawn variates (<= ~1 GiB
  // each): a chunk's step launch reads one while the next chunk's fill writes the other
  const size_t per_iter = ((size_t)2 * x->P * x->G * x->C + (size_t)2 * x->P * x->C) * 8;
  size_t budget = (size_t)1 << 30;
  if (const char* e = getenv("NMC_VARIATE_BYTES")) budget = (size_t)atoll(e);
  int vcap = (int)(budget / per_iter);
  if (vcap < 1) vcap = 1;
  if (vcap > n_iter) vcap = n_iter > 0 ? n_iter : 1;
  // (a pending prefill writes the buffers about to be freed)
  HIPCHK(hipStreamSynchronize(x->pstream));
  x->pf.valid = false;
  const size_t PGC = (size_t)x->P * x->G * x->C, PC = (size_t)x->P * x->C;
  for (int b = 0; b < 2; ++b) {
    dfree(x, x->vzlb[b]); dfree(x, x->vhb[b]);
    rc = dalloc(x, &x->vzlb[b], 2 * vcap * PGC) | dalloc(x, &x->vhb[b], 2 * vcap * PC);
    if (rc) return rc;
  }
  d.vzl = x->vzlb[0];
  d.vh = x->vhb[0];
  x->vbuf = 1;
  d.vcap = vcap;
  d.vbase = 0;
  x->n_iter = n_iter;
  x->scheduled = true;
  return alloc_trace(x);
}

int nmc_n_rows(nmc_ctx* x, int* rows, int* cols) {
  *rows = x->d.n_rows;
  *cols = x->P * (x->G + (x->pooling == NMC_POOL_PARTIAL ? 2 : 0));
  return 0;
}

int nmc_set_trace(nmc_ctx* x, int enable) {
  RES_PARK(x);
  hipSetDevice(x->device);
  x->trace = enable != 0;
  return alloc_trace(x);
}

int nmc_get_trace(nmc_ctx* x, uint8_t* accept, double* ll_prop) {
  RES_PARK(x);
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  if (!x->d.trace_n) return fail(-1, "trace not enabled");
  const size_t n = (size_t)x->d.trace_n * x->P * x->G * x->C;
  if (accept) HIPCHK(hipMemcpy(accept, x->d.tflag, n, hipMemcpyDeviceToHost));
  if (ll_prop) HIPCHK(hipMemcpy(ll_prop, x->d.tllp, n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_run(nmc_ctx* x, int iter_begin, int iter_end) {
  nmc_call_trace tr("nmc_run");
  hipSetDevice(x->device);
  tr.mark("setdev");
  if (!x->scheduled) return fail(-1, "nmc_set_schedule first");
  if (iter_begin < 0 || iter_end < iter_begin) return fail(-1, "invalid iteration range");
  if (iter_begin == iter_end) return 0;
  if (x->rng == NMC_RNG_REPLAY && (!x->d.rz || iter_end > x->d.replay_n))
    return fail(-1, "replay variates do not cover the iteration range");
  // a persistent launch that already timed out: stop before queueing more work
  if (int rc0 = check_timeout(x)) return rc0;
  tr.mark("tmo");
  if (x->res.active) {   // the next call of the resident launch, or park it
    const int rc = res_continue(x, iter_begin, iter_end);
    tr.mark("resident");
    if (rc < 0) return rc;
    if (rc == 1) return 0;
  }
  const bool partial = x->pooling == NMC_POOL_PARTIAL;
  const int P = x->P;
  // the kernels read the values after iteration iter_begin-1 from vb[(iter_begin-1)&1]
  const int need = (iter_begin - 1) & 1;
  if (x->cur_slot != need) {
    HIPCHK(hipMemcpyAsync(vslot(x, need), vslot(x, x->cur_slot),
                          (size_t)x->P * x->G * x->C * 8, hipMemcpyDeviceToDevice, x->stream));
    if (partial) {
      const size_t PC = (size_t)x->P * x->C;
      for (double* h : {x->d.mu, x->d.s2, x->d.hsd, x->d.hlsd})
        HIPCHK(hipMemcpyAsync(h + need * PC, h + x->cur_slot * PC, PC * 8,
                              hipMemcpyDeviceToDevice, x->stream));
    }
    x->cur_slot = need;
  }
  auto launch_run = [&](int i0, int i1, int flags, bool res = false) -> int {
    NmcCall c;
    c.op = NMC_OP_RUN;
    c.i0 = i0;
    c.i1 = i1;
    c.flags = flags;
    c.res = res ? 1 : 0;
    return nmc_call_family(x, c);
  };
  int rc = [&]() -> int {
    const int chunk = fill_chunk(x);
    const bool fills = fill_elements(x, 1) > 0;
    for (int c0 = iter_begin; c0 < iter_end; c0 += chunk) {
      const int c1 = c0 + chunk < iter_end ? c0 + chunk : iter_end;
      // every variate of iterations [c0, c1) before the chunk's step launch: the hyper
      // variates (partial pooling) and the step variates (unless the step kernel draws them),
      // from the pending prefill where it starts at c0, the rest in one fully parallel launch
      int buf = x->vbuf ^ 1, have = c0, vb = c0;
      if (x->pf.valid) {
        // (whatever it holds, the prefill's writes end before this stream goes on; no
        // barrier packet when it is already done)
        if (hipEventQuery(x->pf_ev) != hipSuccess)
          HIPCHK(hipStreamWaitEvent(x->stream, x->pf_ev, 0));
        tr.mark("pfq");
        // (a prefill into a resident launch's buffer sits at its offset from that launch's
        // first iteration pf.vb: usable while the chunk fits the buffer from there)
        if (x->pf.i0 == c0 && c1 - x->pf.vb <= x->d.vcap) {
          buf = x->pf.buf;
          vb = x->pf.vb;
          have = std::min(c1, x->pf.i1);
          x->pf_used += have - c0;
        }
        x->pf.valid = false;
      }
      x->vbuf = buf;
      x->d.vzl = x->vzlb[buf];
      x->d.vh = x->vhb[buf];
      x->d.vbase = vb;
      if (fills && have < c1)
        if (int rc = launch_fill(x, buf, vb, have, c1, x->stream, x->fill_bpc)) return rc;
      // the next chunk's variates beside this chunk's step launch (enqueued after it): the
      // rest of this call, or the same length again after it (the next call of a sampling
      // loop) while the schedule lasts
      int n0 = c1, n1 = c1 < iter_end ? std::min(c1 + chunk, iter_end)
                                      : std::min({c1 + (iter_end - iter_begin), c1 + chunk,
                                                  x->n_iter});
      // (replayed variates: within the call only -- the replay arrays may change between calls)
      if (!fills || !x->prefill_on || (x->rng == NMC_RNG_REPLAY && c1 == iter_end)) n1 = n0;
      // counters continue from the earlier launches (Dev.pbase / xbase): reset only
      // before they could wrap
      const uint64_t steps = (uint64_t)(c1 - c0) * P;
      if ((uint64_t)x->G * (x->d.pbase + (uint64_t)(c1 - c0)) >= (1ull << 31) ||
          (uint64_t)x->d.S * (x->d.xbase + steps) >= (1ull << 31)) {
        HIPCHK(hipMemsetAsync(x->d.cnt, 0, cnt_bytes(x), x->stream));
        HIPCHK(hipMemsetAsync(x->d.hrd, 0, hrd_words(x) * sizeof(unsigned), x->stream));
        if (x->d.xcnt)
          HIPCHK(hipMemsetAsync(x->d.xcnt, 0, (size_t)x->d.RB * x->d.G * 32 * sizeof(unsigned),
                                x->stream));
        x->d.pbase = x->d.xbase = 0;
      }
      // a one-chunk call of a resident context: the resident instance, which then takes the
      // following calls (res_continue)
      const bool resl = x->res.on && !x->ktiming && c0 == iter_begin && c1 == iter_end &&
                        (!partial || x->persistent);
      if (resl) {
        auto& r = x->res;
        HIPCHK(hipMemsetAsync(r.rsync, 0, NMC_RSYNC_WORDS * sizeof(unsigned), x->stream));
        r.ack[1] = 0;
        r.seq += 1;
        r.done = r.seq - 1;
        x->d.rseq = r.seq;
        if (int rc = launch_run(c0, c1, partial ? NMC_RUN_HYPER_LOAD : 0, true)) return rc;
        tr.mark("launch");
        r.active = true;
        r.end = c1;
        r.buf = buf;
        r.vbase = vb;
        r.nwg = x->d.RB * x->G * x->d.S;
        r.launches += 1;
        x->d.pbase += (unsigned)(c1 - c0);
        x->d.xbase += (unsigned)steps;
      } else if (!partial) {
        if (int rc = launch_run(c0, c1, 0)) return rc;
        x->d.xbase += (unsigned)steps;
      } else if (x->persistent) {
        if (int rc = launch_run(c0, c1, NMC_RUN_HYPER_LOAD)) return rc;
        tr.mark("launch");
        x->d.pbase += (unsigned)(c1 - c0);
        x->d.xbase += (unsigned)steps;
      } else {
        for (int it = c0; it < c1; ++it)
          if (int rc = launch_run(it, it + 1, it == c0 ? NMC_RUN_HYPER_LOAD : 0)) return rc;
        if (int rc = launch_hyper(x, c1 - 1)) return rc;   // closes the chunk
      }
      HIPCHK(hipEventRecord(x->rd_ev[buf], x->stream));
      tr.mark("rdev");
      if (n1 > n0) {
        if (resl) {   // into the resident launch's buffer, after this call's iterations
          if (int rc = res_prefill(x, n0, n1)) return rc;
        } else if (int rc = enqueue_prefill(x, n0, n1)) {
          return rc;
        }
      }
      tr.mark("prefill");
    }
    return 0;
  }();
  x->cur_slot = (iter_end - 1) & 1;
  return rc;
}

int nmc_prefill(nmc_ctx* x, int iter_begin, int iter_end) {
  hipSetDevice(x->device);
  if (!x->scheduled) return fail(-1, "nmc_set_schedule first");
  if (iter_begin < 0 || iter_end < iter_begin || iter_end > x->n_iter)
    return fail(-1, "invalid iteration range");
  if (x->rng == NMC_RNG_REPLAY && (!x->d.rz || iter_end > x->d.replay_n))
    return fail(-1, "replay variates do not cover the iteration range");
  if (iter_begin == iter_end || !x->prefill_on || fill_elements(x, 1) == 0) return 0;
  if (x->res.active) {   // the resident launch's next call: into its buffer
    if (iter_begin == x->res.end && iter_end - x->res.vbase <= x->d.vcap)
      return res_prefill(x, iter_begin, iter_end);
    RES_PARK(x);
  }
  return enqueue_prefill(x, iter_begin, iter_end);
}

int nmc_prefill_stats(nmc_ctx* x, int64_t* issued, int64_t* used) {
  if (issued) *issued = x->pf_issued;
  if (used) *used = x->pf_used;
  return 0;
}

// Wait for the context's stream by polling it (hipStreamQuery), then blocking: the
// blocking wait's wake-up costs ~10 us per call (profiles/r03_launchcost: wall minus event
// time), a tenth of a 20-iteration run.  The first 100 us spin; up to 50 ms the poll yields
// the core between queries (one rank per GPU must not hold a host core each while the CSV
// writers and init threads need them); after that the blocking wait.  NMC_SYNC_POLL_US sets
// the polling window (0: block at once).
int nmc_synchronize(nmc_ctx* x) {
  nmc_call_trace tr("nmc_synchronize");
  hipSetDevice(x->device);
  int nq = 0;
  static const long poll_us = [] {
    const char* e = getenv("NMC_SYNC_POLL_US");
    return e ? atol(e) : 50000L;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  // a resident launch: every workgroup reports the latest call done (the launch itself stays)
  if (x->res.active) {
    if (int rc = res_wait_done(x)) return rc;
    tr.mark("resident");
  }
  // the step stream, then the prefill stream (a prefill is part of the work a call enqueued)
  for (hipStream_t s : {x->stream, x->pstream}) {
    if (s == x->stream && x->res.active) continue;
    const auto ts = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = poll_us > 0 ? hipStreamQuery(s) : hipErrorNotReady;
      ++nq;
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) return fail(-2, std::string("hipStreamQuery: ") + hipGetErrorString(e));
      // a prefill that has not finished 2 ms after the resident call did: it cannot run beside
      // the launch (kernels serialized, e.g. a profiler's counter pass) -- park the launch so
      // that it runs, and launch from now on (nmc_resident_stats reason 8)
      if (x->res.active &&
          std::chrono::steady_clock::now() - ts > std::chrono::milliseconds(2)) {
        x->res.why = 8;
        x->res.on = false;
        RES_PARK(x);
      }
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt >= std::chrono::microseconds(poll_us)) {
        HIPCHK(hipStreamSynchronize(s));
        break;
      }
      if (dt > std::chrono::microseconds(100)) std::this_thread::yield();
    }
    tr.mark(s == x->stream ? "stream" : "pstream");
  }
  if (g_trace_calls) {
    char q[32];
    snprintf(q, sizeof(q), "queries=%d", nq);
    tr.mark(q);
  }
  return check_timeout(x);
}

int nmc_get_samples(nmc_ctx* x, int row_begin, int n_rows, double* out) {
  RES_PARK(x);
  hipSetDevice(x->device);
  const Dev& d = x->d;
  if (row_begin < 0 || n_rows < 0 || row_begin + n_rows > d.n_rows)
    return fail(-1, "row range out of bounds");
  HIPCHK(hipStreamSynchronize(x->stream));
  if (int rc = check_timeout(x)) return rc;
  const size_t per = (size_t)d.cols * x->C;
  if (n_rows)
    HIPCHK(hipMemcpy(out, d.samples + (size_t)row_begin * per, (size_t)n_rows * per * 8,
                     hipMemcpyDeviceToHost));
  return 0;
}

int nmc_get_accept_counts(nmc_ctx* x, int64_t* out) {
  RES_PARK(x);
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  HIPCHK(hipMemcpy(out, x->d.tacc, (size_t)x->P * x->G * x->C * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_eval_group_ll(nmc_ctx* x, const double* theta, double* out) {
  RES_PARK(x);
  hipSetDevice(x->device);
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C;
  double *th = nullptr, *o = nullptr, *part = nullptr;
  HIPCHK(hipMalloc(&th, PGC * 8));
  HIPCHK(hipMalloc(&o, GC * 8));
  HIPCHK(hipMalloc(&part, (size_t)x->d.S * x->nacc * GC * 8));
  HIPCHK(hipMemcpyAsync(th, theta, PGC * 8, hipMemcpyHostToDevice, x->stream));
  NmcCall c;
  c.op = NMC_OP_GROUP_LL;
  c.in = th;
  c.out = o;
  c.aux = part;
  int rc = nmc_call_family(x, c);
  if (!rc) {
    hipError_t e = hipMemcpyAsync(out, o, GC * 8, hipMemcpyDeviceToHost, x->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
    if (e != hipSuccess) rc = fail(-2, std::string("eval_group_ll: ") + hipGetErrorString(e));
  }
  hipStreamSynchronize(x->stream);
  hipFree(th);
  hipFree(o);
  hipFree(part);
  return rc;
}

int nmc_eval_obs_ll(nmc_ctx* x, double* out) {
  RES_PARK(x);
  hipSetDevice(x->device);
  const size_t n = (size_t)x->C * x->n_obs;
  double* o = nullptr;
  HIPCHK(hipMalloc(&o, (n ? n : 1) * 8));
  NmcCall c;
  c.op = NMC_OP_OBS_LL;
  c.in = vslot(x, x->cur_slot);
  c.out = o;
  int rc = nmc_call_family(x, c);
  if (!rc && n) {
    hipError_t e = hipMemcpyAsync(out, o, n * 8, hipMemcpyDeviceToHost, x->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
    if (e != hipSuccess) rc = fail(-2, std::string("eval_obs_ll: ") + hipGetErrorString(e));
  }
  if (!rc) rc = check_timeout(x);   // rows from a timed-out persistent launch are not valid
  hipFree(o);
  return rc;
}

// With a resident launch on the stream an event would complete only when the launch ends:
// the slot marks the latest call issued instead, and the elapsed time up to such a mark is
// the sum of the GPU spans (s_memrealtime: workgroup 0 taking the call, or starting the
// launch for its first call -> the last workgroup done) of the calls issued since slot a.
int nmc_event_record(nmc_ctx* x, int slot) {
  if (slot < 0 || slot >= 16) return fail(-1, "event slot 0..15");
  hipSetDevice(x->device);
  x->res.ev_res[slot] = x->res.active;
  x->res.ev_seq[slot] = x->res.seq;
  if (!x->res.active) HIPCHK(hipEventRecord(x->ev[slot], x->stream));
  return 0;
}

int nmc_event_elapsed(nmc_ctx* x, int a, int b, float* ms) {
  if (a < 0 || a >= 16 || b < 0 || b >= 16) return fail(-1, "event slot 0..15");
  hipSetDevice(x->device);
  auto& r = x->res;
  if (r.ev_res[b]) {   // (a: a marker, or an event recorded before the launch started)
    if ((int)(r.ev_seq[b] - r.done) > 0)
      if (int rc = res_wait_done(x)) return rc;
    double sum = 0;
    for (unsigned q = r.ev_seq[a] + 1; (int)(r.ev_seq[b] - q) >= 0; ++q) {
      auto it = std::find_if(r.spans.begin(), r.spans.end(),
                             [&](const std::pair<unsigned, double>& e) { return e.first == q; });
      if (it == r.spans.end() || it->second < 0)
        return fail(-1, "no GPU span for a call between the event slots (a call of a launch "
                        "that has parked since)");
      sum += it->second;
    }
    *ms = (float)sum;
    return 0;
  }
  if (r.ev_res[a]) return fail(-1, "event slot a marks a resident call, b does not");
  HIPCHK(hipEventSynchronize(x->ev[b]));
  HIPCHK(hipEventElapsedTime(ms, x->ev[a], x->ev[b]));
  return 0;
}

int nmc_set_resident(nmc_ctx* x, int enable) {
  hipSetDevice(x->device);
  auto& r = x->res;
  if (!enable) {
    RES_PARK(x);
    r.on = false;
    return 0;
  }
  if (r.on) return 0;
  // possible: a built-in family on nmc_k_run with the rows in LDS, one member per group,
  // drawn (not replayed) variates from the fill, and a resident instance of the run mode
  // whose whole grid is co-resident
  if (x->family >= NMC_LL_USER_BASE || x->sweep || x->rng == NMC_RNG_REPLAY || x->d.zin ||
      !x->d.rows_lds || x->d.S != 1 ||
      (x->pooling == NMC_POOL_PARTIAL && !x->persistent))
    return 0;
  NmcCall c;
  c.op = NMC_OP_RES_OK;
  if (int rc = nmc_call_family(x, c)) return rc;
  if (c.result != 1) return 0;
  if (g_trace_calls)
    fprintf(stderr, "[nmc trace] resident instance: %d VGPRs\n", c.result2);
  // the prefill's fill beside the launch: the largest instance that fits the VGPRs the
  // launch's waves leave per SIMD lane (512; allocation granule 8), else none fits
  {
    const int wps = (x->d.W + 3) / 4;   // the launch's waves per SIMD
    const int left = 512 - wps * ((c.result2 + 7) / 8) * 8;
    r.fill_minb = left >= 144 ? 1 : left >= 128 ? 4 : left >= 96 ? 5 : left >= 80 ? 6
                : left >= 64 ? 8 : 0;
    if (!r.fill_minb) return 0;
    // (diagnostics, A/B: a smaller fill instance than the one that fits)
    if (const char* e = getenv("NMC_RES_FILL_MINB")) {
      const int v = atoi(e);
      if ((v == 4 || v == 5 || v == 6 || v == 8) && v > r.fill_minb) r.fill_minb = v;
    }
  }
  if (!r.host) {
    const size_t bytes = 512;
    void* h = nullptr;
    void* dp = nullptr;
    HIPCHK(hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    memset(h, 0, bytes);
    r.host = h;
    if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess)
      return fail(-2, "resident launch: pinned command block not mapped");
    r.cmd = (volatile unsigned long long*)h;
    r.ack = (volatile unsigned*)((char*)h + 128);
    r.done_w = (volatile unsigned*)((char*)h + 256);
    x->d.rcmd = (unsigned long long*)dp;
    x->d.rack = (unsigned*)((char*)dp + 128);
    x->d.rdone = (unsigned*)((char*)dp + 256);
    if (int rc = dalloc(x, &r.rsync, NMC_RSYNC_WORDS)) return rc;
    x->d.rsync = r.rsync;
  }
  // workgroup 0 parks the launch after this long without a call (NMC_RESIDENT_IDLE_US)
  const char* e = getenv("NMC_RESIDENT_IDLE_US");
  x->d.ridle = (unsigned)std::min(4.0e9, 100.0 * (e ? atof(e) : 20000.0));
  r.on = true;
  return 0;
}

int nmc_resident_stats(nmc_ctx* x, int* enabled, int* active, int64_t* launches, int64_t* calls,
                       int* last_refusal) {
  if (last_refusal) *last_refusal = x->res.why;
  if (enabled) *enabled = x->res.on ? 1 : 0;
  if (active) *active = x->res.active ? 1 : 0;
  if (launches) *launches = x->res.launches;
  if (calls) *calls = x->res.calls;
  return 0;
}


int nmc_set_launch_iters(nmc_ctx* x, int max_iters) {
  RES_PARK(x);
  if (max_iters < 0) return fail(-1, "max_iters < 0");
  x->launch_iters = max_iters;
  return 0;
}

int nmc_set_kernel_timing(nmc_ctx* x, int enable) {
  if (enable) RES_PARK(x);   // (per-launch events: the timed launches are not resident)
  x->ktiming = enable != 0;
  x->kev_used = x->hev_used = 0;
  x->step_ms = x->hyper_ms = 0;
  x->step_n = x->hyper_n = 0;
  x->step_iters = 0;
  return 0;
}

int nmc_get_kernel_timing(nmc_ctx* x, double* step_ms, int64_t* step_n, int64_t* step_iters,
                          double* hyper_ms, int64_t* hyper_n) {
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  for (size_t i = 0; i < x->kev_used; ++i) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, x->kev[i].first, x->kev[i].second));
    x->step_ms += ms;
    x->step_n += 1;
    x->step_iters += x->kev_iters[i];
  }
  for (size_t i = 0; i < x->hev_used; ++i) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, x->hev[i].first, x->hev[i].second));
    x->hyper_ms += ms;
    x->hyper_n += 1;
  }
  x->kev_used = x->hev_used = 0;
  if (step_ms) *step_ms = x->step_ms;
  if (step_n) *step_n = x->step_n;
  if (step_iters) *step_iters = x->step_iters;
  if (hyper_ms) *hyper_ms = x->hyper_ms;
  if (hyper_n) *hyper_n = x->hyper_n;
  return 0;
}

int nmc_split_config(nmc_ctx* x, int* members, int* chain_blocks_per_launch) {
  *members = x->d.S;
  *chain_blocks_per_launch = x->d.S > 1 ? x->split_batch
                             : x->sweep && x->d.gsep && x->sweep_batch > 0 ? x->sweep_batch
                                                                           : x->d.RB;
  return 0;
}

int nmc_kernel_name(nmc_ctx* x, char* out, int cap) {
  static const char* const modes[] = {"NMC_MODE_NOPOOL", "NMC_MODE_LAUNCH", "NMC_MODE_SYNC",
                                      "NMC_MODE_SYNC_LDS", "NMC_MODE_SYNC_REG", "NMC_MODE_SYNC_OWN",
                                      "NMC_MODE_HALF"};
  const int mode = run_mode(x);
  std::string fam;
  switch (x->family) {
    case NMC_LL_LINREG: fam = "FamLinreg<" + std::to_string(x->nf) + ">"; break;
    case NMC_LL_GAUSS_MEAN: fam = "FamGaussMean<" + std::to_string(x->nf) + ">"; break;
    case NMC_LL_LOGISTIC: fam = "FamLogistic<" + std::to_string(x->nf) + ">"; break;
    default: fam = "FamUser"; break;
  }
  if (x->sweep) {
    snprintf(out, (size_t)(cap > 0 ? cap : 1), "%s",
             ("nmc_k_sweep<" + fam + ", " + modes[mode] + ">").c_str());
    return cap < 1 ? fail(-1, "kernel name: cap < 1") : 0;
  }
  const std::string k = "nmc_k_run<" + fam + ", " + modes[mode] + ", " +
                        (x->d.rows_lds ? "true" : "false") + ">";
  if (cap < 1) return fail(-1, "kernel name: cap < 1");
  snprintf(out, (size_t)cap, "%s", k.c_str());
  return 0;
}

int nmc_gibbs_fallbacks(nmc_ctx* x, int64_t* out) {
  RES_PARK(x);
  if (!out) return fail(-1, "gibbs fallbacks: null output");
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  unsigned n = 0;
  HIPCHK(hipMemcpy(&n, x->d.gfb, sizeof(unsigned), hipMemcpyDeviceToHost));
  *out = (int64_t)n;
  return 0;
}

int nmc_variate_source(nmc_ctx* x, int* in_kernel) {
  if (!in_kernel) return fail(-1, "variate source: null output");
  *in_kernel = x->d.zin ? 1 : 0;
  return 0;
}

int nmc_launch_config(nmc_ctx* x, int* waves_per_group, int* chain_blocks, int* persistent,
                      int* chains_per_block, int* mode) {
  *waves_per_group = x->d.W;
  *chain_blocks = x->d.RB;
  if (persistent) *persistent = x->persistent || x->pooling != NMC_POOL_PARTIAL ? 1 : 0;
  if (chains_per_block) *chains_per_block = x->d.CL;
  if (mode) *mode = run_mode(x);
  return 0;
}

// ---------------------------------------------------------------------------
// CSV output with the reference's formatting (Python "%f" == C "%f" except the
// spelling of NaN, which Python always prints as "nan").
// ---------------------------------------------------------------------------
// std::to_chars(fixed, 6) is the exact decimal "%f" produces (both correctly rounded),
// at several times snprintf's speed; 512 bytes hold any finite double's fixed form.
static inline void put_f(std::string& s, double v) {
  char buf[512];
  if (isnan(v)) { s += "nan"; return; }
  if (isinf(v)) { s += v > 0 ? "inf" : "-inf"; return; }
  const std::to_chars_result r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::fixed, 6);
  if (r.ec == std::errc()) {
    s.append(buf, r.ptr - buf);
  } else {
    const int n = snprintf(buf, sizeof(buf), "%f", v);
    s.append(buf, n < (int)sizeof(buf) ? n : (int)sizeof(buf) - 1);
  }
}

int nmc_write_sample_csv(const char* path, int append, const char* header, const double* samples,
                         int n_chains, int c, int cols, const int32_t* row_index, int n_rows,
                         int chain_id) {
  FILE* f = fopen(path, append ? "a" : "w");
  if (!f) return fail(-3, std::string("cannot open ") + path);
  std::string s;
  s.reserve((size_t)(n_rows + 1) * (cols * 12 + 16));
  if (header) { s += header; s += '\n'; }
  char pre[64];
  for (int r = 0; r < n_rows; ++r) {
    int n = snprintf(pre, sizeof(pre), "%d,%d,", row_index[r], chain_id);
    s.append(pre, n);
    for (int k = 0; k < cols; ++k) {
      if (k) s += ',';
      put_f(s, samples[((size_t)r * cols + k) * n_chains + c]);
    }
    s += '\n';
  }
  size_t w = fwrite(s.data(), 1, s.size(), f);
  fclose(f);
  if (w != s.size()) return fail(-3, std::string("short write to ") + path);
  return 0;
}

// the group of every observation (CSR order), built once per context
static int ensure_gidx(nmc_ctx* x) {
  if (x->gidx || x->n_obs == 0) return 0;
  std::vector<int64_t> off(x->G + 1);
  HIPCHK(hipMemcpy(off.data(), x->d.off, (x->G + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<int> gi(x->n_obs);
  for (int g = 0; g < x->G; ++g)
    for (int64_t i = off[g]; i < off[g + 1]; ++i) gi[i] = g;
  if (int rc = dalloc(x, &x->gidx, (size_t)x->n_obs)) return rc;
  HIPCHK(hipMemcpy(x->gidx, gi.data(), x->n_obs * sizeof(int), hipMemcpyHostToDevice));
  return 0;
}

int nmc_obs_ll_rows(nmc_ctx* x, int row_begin, int n_rows, double* out) {
  RES_PARK(x);
  hipSetDevice(x->device);
  if (row_begin < 0 || n_rows < 0 || row_begin + n_rows > x->d.n_rows || n_rows > 65535)
    return fail(-1, "row range out of bounds (at most 65535 rows per call)");
  HIPCHK(hipStreamSynchronize(x->stream));
  if (int rc = check_timeout(x)) return rc;
  if (int rc = ensure_gidx(x)) return rc;
  const size_t n = (size_t)x->C * n_rows * x->n_obs;
  if (n == 0) return 0;
  double* o = nullptr;
  HIPCHK(hipMalloc(&o, n * 8));
  NmcCall c;
  c.op = NMC_OP_OBS_LL_ROWS;
  c.i0 = row_begin;
  c.i1 = row_begin + n_rows;
  c.out = o;
  int rc = nmc_call_family(x, c);
  if (!rc) {
    hipError_t e = hipMemcpyAsync(out, o, n * 8, hipMemcpyDeviceToHost, x->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
    if (e != hipSuccess) rc = fail(-2, std::string("obs_ll_rows: ") + hipGetErrorString(e));
  }
  hipFree(o);
  return rc;
}

// saveLogLikelihood (Sampler._printLogLikelihood :907-909 at every recorded row, the LL
// of :656-659 evaluated at the recorded values): batches are evaluated on the device into
// one of two buffers and copied to pinned host memory while the host formats and appends
// the previous batch, one thread per group of chain files.  A batch is several rows of
// every chain within a 256 MiB budget, or -- when one row of every chain exceeds it
// (many chains x many observations) -- one row of a sub-range of the chains.
int nmc_write_ll_csvs(nmc_ctx* x, const char* dir, const int32_t* chain_ids, int threads) {
  RES_PARK(x);
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  if (int rc = check_timeout(x)) return rc;
  const int rows = x->d.n_rows;
  const int C = x->C;
  const int64_t n_obs = x->n_obs;
  if (rows == 0 || n_obs == 0) return 0;
  if (int rc = ensure_gidx(x)) return rc;
  // (NMC_LL_BATCH_BYTES: a smaller budget, so the tests can reach the chain-batched branch)
  size_t budget = (size_t)256 << 20;
  if (const char* e = getenv("NMC_LL_BATCH_BYTES"))
    if (atoll(e) > 0) budget = (size_t)atoll(e);
  const size_t per_chain_row = (size_t)n_obs * 8;
  const size_t per_row = (size_t)C * per_chain_row;
  int nb, ncb;   // rows per batch, chains per batch
  if (per_row <= budget) {
    nb = (int)std::min<size_t>({budget / per_row, (size_t)rows, (size_t)65535});
    ncb = C;
  } else {
    nb = 1;
    ncb = (int)std::max<size_t>(1, std::min<size_t>(budget / per_chain_row, 65535));
  }
  const int nrb = (rows + nb - 1) / nb, ncbk = (C + ncb - 1) / ncb;
  const int nbatch = nrb * ncbk;   // batch b: rows of block b / ncbk, chains of block b % ncbk
  const size_t buf_bytes = (size_t)nb * ncb * per_chain_row;
  double* dbuf[2] = {nullptr, nullptr};
  double* hbuf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  int rc = 0;
  auto cleanup = [&]() {
    for (int i = 0; i < 2; ++i) {
      if (dbuf[i]) hipFree(dbuf[i]);
      if (hbuf[i]) hipHostFree(hbuf[i]);
      if (ev[i]) hipEventDestroy(ev[i]);
    }
  };
  for (int i = 0; i < 2 && !rc; ++i) {
    if (hipMalloc(&dbuf[i], buf_bytes) != hipSuccess ||
        hipHostMalloc(&hbuf[i], buf_bytes, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
      rc = fail(-2, "write_ll_csvs: out of device or pinned host memory");
  }
  struct Batch { int r0, n, c0, nc; };
  auto batch = [&](int b) {
    Batch q;
    q.r0 = (b / ncbk) * nb;
    q.n = std::min(nb, rows - q.r0);
    q.c0 = (b % ncbk) * ncb;
    q.nc = std::min(ncb, C - q.c0);
    return q;
  };
  auto launch = [&](int b) -> int {
    const Batch q = batch(b);
    NmcCall c;
    c.op = NMC_OP_OBS_LL_ROWS;
    c.i0 = q.r0;
    c.i1 = q.r0 + q.n;
    c.c0 = q.c0;
    c.nc = q.nc;
    c.out = dbuf[b & 1];
    if (int e = nmc_call_family(x, c)) return e;
    HIPCHK(hipMemcpyAsync(hbuf[b & 1], dbuf[b & 1], (size_t)q.n * q.nc * per_chain_row,
                          hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipEventRecord(ev[b & 1], x->stream));
    return 0;
  };
  if (!rc) rc = launch(0);
  for (int b = 0; b < nbatch && !rc; ++b) {
    if (b + 1 < nbatch && (rc = launch(b + 1))) break;
    if (hipEventSynchronize(ev[b & 1]) != hipSuccess) { rc = fail(-2, "write_ll_csvs: device"); break; }
    const Batch q = batch(b);
    const double* hb = hbuf[b & 1];
    const int T = std::max(1, std::min(threads, q.nc));
    std::vector<std::string> errs(T);
    auto work = [&](int tid) {
      std::string s;
      for (int k = tid; k < q.nc; k += T) {
        const int c = q.c0 + k;
        if (chain_ids[c] < 0) continue;   // (no file: a rank's padding chain)
        char path[4096];
        snprintf(path, sizeof(path), "%slogLikelihood.%d.csv", dir, chain_ids[c]);
        FILE* f = fopen(path, q.r0 == 0 ? "w" : "a");
        if (!f) { errs[tid] = std::string("cannot open ") + path; return; }
        s.clear();
        for (int r = 0; r < q.n; ++r) {
          const double* v = hb + ((size_t)k * q.n + r) * n_obs;
          for (int64_t i = 0; i < n_obs; ++i) {
            if (i) s += ',';
            put_f(s, v[i]);
          }
          s += '\n';
          if (s.size() > (1u << 22)) { fwrite(s.data(), 1, s.size(), f); s.clear(); }
        }
        const size_t w = fwrite(s.data(), 1, s.size(), f);
        if (fclose(f) != 0 || w != s.size()) { errs[tid] = std::string("short write to ") + path; return; }
      }
    };
    std::vector<std::thread> pool;
    for (int tid = 1; tid < T; ++tid) pool.emplace_back(work, tid);
    work(0);
    for (auto& th : pool) th.join();
    for (auto& e : errs)
      if (!e.empty()) { rc = fail(-3, e); break; }
  }
  if (rc) hipStreamSynchronize(x->stream);
  cleanup();
  return rc;
}

int nmc_write_ll_csv(const char* path, int append, const double* ll, int64_t n, int n_rows) {
  FILE* f = fopen(path, append ? "a" : "w");
  if (!f) return fail(-3, std::string("cannot open ") + path);
  std::string s;
  for (int r = 0; r < n_rows; ++r) {
    for (int64_t k = 0; k < n; ++k) {
      if (k) s += ',';
      put_f(s, ll[(size_t)r * n + k]);
    }
    s += '\n';
    if (s.size() > (1u << 24)) { fwrite(s.data(), 1, s.size(), f); s.clear(); }
  }
  fwrite(s.data(), 1, s.size(), f);
  fclose(f);
  return 0;
}

// ---------------------------------------------------------------------------
// RCCL: one gather of every rank's sample store to the root over xGMI
// ---------------------------------------------------------------------------
int nmc_comm_unique_id(unsigned char* out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(-4, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int nmc_comm_init(void** comm, const unsigned char* idb, int nranks, int rank, int device) {
  HIPCHK(hipSetDevice(device));
  ncclUniqueId id;
  memcpy(id.internal, idb, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess) return fail(-4, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  *comm = (void*)c;
  return 0;
}

int nmc_comm_destroy(void* comm) {
  if (comm) ncclCommDestroy((ncclComm_t)comm);
  return 0;
}

int nmc_comm_size(void* comm, int* nranks, int* rank) {
  ncclComm_t c = (ncclComm_t)comm;
  ncclResult_t r = ncclCommCount(c, nranks);
  if (r == ncclSuccess) r = ncclCommUserRank(c, rank);
  if (r != ncclSuccess) return fail(-4, std::string("ncclCommCount: ") + ncclGetErrorString(r));
  return 0;
}

int nmc_gather_samples(nmc_ctx* x, void* comm, int root, double* host_out,
                       int64_t host_capacity) {
  RES_PARK(x);
  hipSetDevice(x->device);
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0, rank = 0;
  if (int rc = nmc_comm_size(comm, &nranks, &rank)) return rc;
  const size_t count = (size_t)x->d.n_rows * x->d.cols * x->C;
  if (rank == root && (!host_out || host_capacity < (int64_t)(count * nranks)))
    return fail(-1, "gather: the root's host buffer holds fewer than nranks * rows * cols * C "
                    "doubles");
  double* recv = nullptr;
  if (rank == root) HIPCHK(hipMalloc(&recv, (count ? count : 1) * nranks * 8));
  ncclResult_t r = ncclGather(x->d.samples, recv, count, ncclDouble, root, c, x->stream);
  if (r != ncclSuccess) {
    if (recv) hipFree(recv);
    return fail(-4, std::string("ncclGather: ") + ncclGetErrorString(r));
  }
  HIPCHK(hipStreamSynchronize(x->stream));
  if (rank == root) {
    HIPCHK(hipMemcpy(host_out, recv, count * nranks * 8, hipMemcpyDeviceToHost));
    hipFree(recv);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// verification hooks: device numerics on caller-supplied inputs
// ---------------------------------------------------------------------------
int nmc_debug_prior_logpdf(int fam, const double* prm8, const double* xs, int n, double* out) {
  double *dp, *dx, *dout;
  HIPCHK(hipMalloc(&dp, 64));
  HIPCHK(hipMalloc(&dx, (n ? n : 1) * 8));
  HIPCHK(hipMalloc(&dout, (n ? n : 1) * 8));
  HIPCHK(hipMemcpy(dp, prm8, 64, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx, xs, n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(nmc_k_debug_prior, dim3((n + 63) / 64), dim3(64), 0, 0, fam, dp, dx, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
  hipFree(dp); hipFree(dx); hipFree(dout);
  return 0;
}

// Diagnostic build only: (re)allocate and zero the stamp buffer (n > 0) and/or copy
// it back (out != NULL): NMC_STAMP_WORDS uint64 (kernels.h NMC_STAMP / NMC_CS layouts).
int nmc_debug_stamps(nmc_ctx* x, int n, uint64_t* out) {
  RES_PARK(x);
#if defined(NMC_STAMPS) || defined(NMC_CSTAMPS)
  hipSetDevice(x->device);
  if (n > 0) {
    if (!x->d.stamps)
      if (int rc = dalloc(x, &x->d.stamps, NMC_STAMP_WORDS)) return rc;
    HIPCHK(hipMemset(x->d.stamps, 0, NMC_STAMP_WORDS * 8));
  }
  if (out) {   // layouts: kernels.h NMC_STAMP / NMC_CS (nmc_k_run), sweep.h NMC_RS_STAMP
    HIPCHK(hipStreamSynchronize(x->stream));
    HIPCHK(hipMemcpy(out, x->d.stamps, NMC_STAMP_WORDS * 8, hipMemcpyDeviceToHost));
  }
  return 0;
#else
  (void)x; (void)n; (void)out;
  return fail(-1, "not a stamps build (make stamps)");
#endif
}

int nmc_debug_igamci(const double* a, const double* q, const double* lga, int n, double* out) {
  double *da, *dq, *dl, *dout;
  const size_t b = (n ? n : 1) * 8;
  HIPCHK(hipMalloc(&da, b)); HIPCHK(hipMalloc(&dq, b)); HIPCHK(hipMalloc(&dl, b));
  HIPCHK(hipMalloc(&dout, b));
  HIPCHK(hipMemcpy(da, a, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dq, q, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dl, lga, n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(nmc_k_debug_igamci, dim3((n + 63) / 64), dim3(64), 0, 0, da, dq, dl, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
  hipFree(da); hipFree(dq); hipFree(dl); hipFree(dout);
  return 0;
}

int nmc_debug_rng(const uint32_t* ctr5, int n, uint32_t seed, double gamma_shape, double* out4) {
  uint32_t* dc;
  double* dout;
  HIPCHK(hipMalloc(&dc, (size_t)(n ? n : 1) * 5 * 4));
  HIPCHK(hipMalloc(&dout, (size_t)(n ? n : 1) * 4 * 8));
  HIPCHK(hipMemcpy(dc, ctr5, (size_t)n * 5 * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(nmc_k_debug_rng, dim3((n + 63) / 64), dim3(64), 0, 0, dc, n, seed,
                     gamma_shape, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out4, dout, (size_t)n * 4 * 8, hipMemcpyDeviceToHost));
  hipFree(dc); hipFree(dout);
  return 0;
}

int nmc_debug_softplus(const double* x, int n, double* out, int on_device) {
  if (n < 0) return fail(-1, "n < 0");
  if (!on_device) {
    for (int i = 0; i < n; ++i) out[i] = nmc_softplus(x[i]);
    return 0;
  }
  double *dx, *dout;
  HIPCHK(hipMalloc(&dx, (size_t)(n ? n : 1) * 8));
  HIPCHK(hipMalloc(&dout, (size_t)(n ? n : 1) * 8));
  HIPCHK(hipMemcpy(dx, x, (size_t)n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(nmc_k_debug_softplus, dim3((n + 255) / 256 > 0 ? (n + 255) / 256 : 1),
                     dim3(256), 0, 0, (const double*)dx, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost));
  hipFree(dx);
  hipFree(dout);
  return 0;
}

}  // extern "C"
