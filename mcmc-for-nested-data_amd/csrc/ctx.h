// ctx.h -- libnestmc internals shared by the C-ABI (nestmc.hip) and the per-family
// translation units (fam_*.hip): the context, error plumbing, the LDS/geometry helpers
// and the family dispatch table.
//
// The kernels are templates over the likelihood family (families.h); instantiating all
// of them for every family and row width in one translation unit took ~90 s, so each
// family lives in its own TU (built in parallel) and is reached through nmc_call_*().
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <utility>
#include <vector>

#include "../../include/nestmc.h"
#include "kernels.h"
#include "sweep.h"

// error message of the calling thread (nestmc.hip); returns code
int nmc_fail(int code, const std::string& msg);

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return nmc_fail(-2, std::string(#x) + ": " + hipGetErrorString(e_));            \
  } while (0)

struct nmc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t gstream = nullptr;          // nmc_k_sweep_gibbs beside the sweep (Dev.gsep)
  hipEvent_t gev[2] = {nullptr, nullptr}; // fork / join of the two streams
  // Pipelined variate fill (nmc_run, nmc_prefill): two variate buffers; the fill of the next
  // chunk's (or the next call's) iterations runs on pstream into the buffer the running
  // chunk does not read.  pf: the pending prefill -- iterations [i0, i1) into buffer buf,
  // done at pf_ev; rd_ev[b]: the last step launch that reads buffer b.
  hipStream_t pstream = nullptr;
  hipEvent_t pf_ev = nullptr, rd_ev[2] = {nullptr, nullptr};
  double* vzlb[2] = {nullptr, nullptr};
  double* vhb[2] = {nullptr, nullptr};
  int vbuf = 1;                           // buffer of the most recent chunk
  // (vb: the iteration at the start of buffer buf -- pf.i0, or a resident launch's first)
  struct { bool valid; int i0, i1, buf, vb; } pf = {false, 0, 0, 0, 0};
  int prefill_bpc = 1;                    // prefill grid: blocks per CU (beside a step kernel)
  bool prefill_on = true;                 // pipelined fill (NMC_PREFILL=0: off, the A/B)
  long long pf_issued = 0, pf_used = 0;   // iterations prefilled / consumed from a prefill
  int C = 0, chain_base = 0, G = 0, P = 0, pooling = 0, family = 0, nf = 0, rng = 0;
  uint32_t seed = 0;
  int64_t n_obs = 0;
  std::vector<double> llc;
  Dev d{};
  std::vector<void*> owned;
  int n_iter = 0;
  bool scheduled = false;
  bool trace = false;
  hipEvent_t ev[16] = {};
  bool ktiming = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kev;   // step launches
  std::vector<std::pair<hipEvent_t, hipEvent_t>> hev;   // hyper-only launches
  size_t kev_used = 0, hev_used = 0;
  double step_ms = 0, hyper_ms = 0;
  long long step_n = 0, hyper_n = 0;
  long long step_iters = 0;
  int launch_iters = 0;                    // cap on iterations per launch (0: vcap)
  std::vector<int> kev_iters;             // iterations covered by each timed step launch
  int cur_slot = 1;                       // state after the last iteration: slot cur_slot
  int nacc = 1;                           // likelihood accumulators of the family
  bool persistent = false;                // partial pooling: one resident launch per chunk
  int ncu = 256;
  int* gidx = nullptr;                    // [n_obs] group of each observation (obs-LL rows)
  int64_t nmax_group = 0;                 // rows of the largest group
  int split_batch = 0;                    // row split: chain blocks per (resident) launch
  int sweep_batch = 0;                    // nmc_k_sweep with Dev.gsep: chain blocks per launch
  unsigned gepoch = 0;                    // Dev.gsep launches so far (Dev.gep)
  int fill_bpc = 3;                       // nmc_k_fill blocks per CU (nmc_run)
  int gserial = 0;                        // tests (NMC_GSEP_SERIAL): the gsep kernels serialized
                                          // on one stream, 1 Gibbs kernel first, 2 second
  volatile unsigned* tmo_host = nullptr;  // host view of d.tmo (coherent pinned memory)
  void* user = nullptr;                   // user family: its per-device kernel table (user.hip)
  double* user_k = nullptr;               // user family: device copy of the model constants
  bool sweep = false;                     // nmc_k_sweep runs the loop (choose_geometry)
  bool no_sweep = false;                  // (its grid could not be resident: nmc_k_run)
  // Resident launch (nmc_set_resident; kernels.h Dev.rcmd): one step launch serves the
  // consecutive nmc_run calls of a sampling loop; any other entry point parks it first.
  struct Resident {
    bool on = false;                      // requested and possible for this context
    bool active = false;                  // a resident launch is on the stream
    unsigned seq = 0;                     // the latest command seq issued
    unsigned done = 0;                    // the latest seq every workgroup reported done
    int end = 0;                          // end of the latest call
    int buf = 0, vbase = 0;               // the variate buffer it reads, its first iteration
    int nwg = 0;                          // workgroups of the launch
    void* host = nullptr;                 // pinned block: cmd | ack | done
    volatile unsigned long long* cmd = nullptr;
    volatile unsigned* ack = nullptr;
    volatile unsigned* done_w = nullptr;
    unsigned* rsync = nullptr;            // device: relay, done count, clocks (Dev.rsync)
    long long launches = 0, calls = 0;    // resident launches / calls continued in one
    int why = 0;                          // why the latest call was not continued (0: it was)
    int fill_minb = 1;                    // nmc_k_fill instance that fits beside the launch
    std::chrono::steady_clock::time_point t_post;   // (NMC_TRACE_CALLS: the latest post)
    std::vector<std::pair<unsigned, double>> spans;   // (seq, GPU ms) of continued calls
    bool ev_res[16] = {};                 // event slot recorded as a resident marker
    unsigned ev_seq[16] = {};
  } res;
};

static inline double* vslot(nmc_ctx* x, int slot) { return slot ? x->d.vb1 : x->d.vb0; }

static inline size_t lds_bytes_for(const nmc_ctx* x, int hlds, int rows_lds) {
  const Dev& d = x->d;
  // (register hand-off: no LDS payload buffers)
  return (size_t)nmc_lds(x->nacc, d.P, x->pooling == NMC_POOL_PARTIAL, d.nleaf, d.ntail, d.W,
                         d.G, hlds && !d.hreg,
                         rows_lds ? d.nmax * x->nf
                                  : (x->nf <= 4 ? 0 : nmc_stage_doubles(x->nf, d.W)))
             .total * 512;
}
static inline int run_mode(const nmc_ctx* x) {
  if (x->pooling != NMC_POOL_PARTIAL) return x->d.CL == 32 ? NMC_MODE_HALF : NMC_MODE_NOPOOL;
  if (x->sweep)
    return x->d.G <= 64 ? NMC_MODE_SYNC_REG : x->d.G <= 128 ? NMC_MODE_SYNC_LDS : NMC_MODE_SYNC_OWN;
  if (!x->persistent) return NMC_MODE_LAUNCH;
  if (x->d.hreg) return NMC_MODE_SYNC_REG;
  return x->d.hlds ? NMC_MODE_SYNC_LDS : NMC_MODE_SYNC;
}

// LDS of nmc_k_sweep (sweep.h); partial pooling over G > 128 groups also runs the Gibbs
// workgroups (SYNC_OWN) in the same launch: their hyper carve (nmc_lds, no rows) must fit
static inline size_t sweep_lds_bytes(const nmc_ctx* x) {
  const Dev& d = x->d;
  const bool partial = x->pooling == NMC_POOL_PARTIAL;
  size_t b = (size_t)nmc_sweep_lds(x->nacc, d.P, partial, d.G > 64 && d.G <= 128 ? 1 : 0, d.G,
                                   d.nmax * x->nf).total * 512;
  if (partial && d.G > 128 && !d.gsep)
    b = std::max(b, (size_t)nmc_lds(0, d.P, 1, d.nleaf, d.ntail, d.W, d.G, 0, 0).total * 512);
  return b;
}
// dynamic LDS of nmc_k_sweep_gibbs (four waves)
static inline size_t sweep_gibbs_lds_bytes(const nmc_ctx* x) {
  const Dev& d = x->d;
  return (size_t)nmc_lds(0, d.P, 1, d.nleaf, d.ntail, 4, d.G, 0, 0).total * 512;
}
// workgroups of the sweep grid: RB * G likelihood workgroups (+ RB * P Gibbs workgroups)
static inline int64_t sweep_grid(const nmc_ctx* x) {
  const Dev& d = x->d;
  return (int64_t)d.RB * d.G +
         (x->pooling == NMC_POOL_PARTIAL && d.G > 128 && !d.gsep ? (int64_t)d.RB * d.P : 0);
}

static inline size_t run_lds_bytes(const nmc_ctx* x) {
  if (x->sweep) return sweep_lds_bytes(x);
  return lds_bytes_for(x, x->persistent && x->d.hlds ? 1 : 0, x->d.rows_lds);
}

// Resident blocks per CU to rely on, from the occupancy API's answer nb.  The API can
// answer one block per CU too many where SGPRs bind (MI355X_MICROARCH.md, residency:
// min(API, floor(800 / (ceil(sgpr / 16) * 16 + 16))) waves per SIMD); the step kernels use
// <= 112 SGPRs -> 6 waves per SIMD, i.e. 24 / W blocks of W = 4k waves.  Other block
// sizes keep one block of margin.
static inline int nmc_safe_blocks(const nmc_ctx* x, int nb) {
  const int W = x->d.W;
  return W % 4 == 0 ? std::min(nb, 24 / W) : (nb > 1 ? nb - 1 : nb);
}
// mode of the persistent partial-pooling kernel (its occupancy query)
static inline int nmc_persist_mode(const nmc_ctx* x) {
  if (x->sweep) return run_mode(x);
  return x->d.hreg ? NMC_MODE_SYNC_REG : x->d.hlds ? NMC_MODE_SYNC_LDS : NMC_MODE_SYNC;
}
// LDS of the persistent partial-pooling kernel (its occupancy query)
static inline size_t nmc_persist_lds(const nmc_ctx* x) {
  if (x->sweep) return sweep_lds_bytes(x);
  return lds_bytes_for(x, x->d.hlds && !x->d.hreg, x->d.rows_lds);
}

// dynamic LDS of nmc_k_group_part: the tile slots and (rows in LDS) the member's rows
static inline size_t nmc_group_ll_lds(const nmc_ctx* x) {
  const Dev& d = x->d;
  return ((size_t)x->nacc * NMC_NSLOT + (d.rows_lds ? (d.nmax * x->nf + 63) / 64 + 1 : 0)) * 512;
}

static inline int pop_event_pair(nmc_ctx* x, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v,
                                 size_t& used, std::pair<hipEvent_t, hipEvent_t>** out) {
  if (used == v.size()) {
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    v.emplace_back(a, b);
  }
  *out = &v[used++];
  return 0;
}

// The step-kernel launches of iterations [i0, i1): launch(mode, dev, grid, block, lds)
// issues one kernel (built-in families: hipLaunchKernelGGL of the template instance;
// user families: hipModuleLaunchKernel of the JIT module).  Row split: one launch per
// resident batch of chain blocks.  Kernel timing events bracket the whole call.
template <class Launch>
static int nmc_run_launches(nmc_ctx* x, int i0, int i1, Launch&& launch) {
  const Dev& d = x->d;
  const size_t lds = run_lds_bytes(x);
  std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
  if (x->ktiming) {
    if (int rc = pop_event_pair(x, x->kev, x->kev_used, &ev)) return rc;
    if (x->kev_iters.size() < x->kev_used) x->kev_iters.resize(x->kev_used);
    x->kev_iters[x->kev_used - 1] = i1 - i0;
    HIPCHK(hipEventRecord(ev->first, x->stream));
  }
  const dim3 block(64 * d.W);
  const int mode = run_mode(x);
  const bool batched = d.S > 1 || (x->sweep && d.gsep && x->sweep_batch > 0 &&
                                   x->sweep_batch < d.RB);
  const int batch = d.S > 1 ? x->split_batch : x->sweep_batch;
  if (batched) {
    // resident batches of chain blocks (chain blocks are independent): the row split, and
    // the sweep with its Gibbs kernel when the whole grid is not co-resident
    for (int cb0 = 0; cb0 < d.RB; cb0 += batch) {
      Dev db = d;
      db.cb0 = cb0;
      const int nb = std::min(batch, d.RB - cb0);
      launch(mode, db, dim3(nb * d.G * d.S), block, lds);
    }
  } else {
    launch(mode, d, dim3(d.RB * d.G * d.S), block, lds);
  }
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev->second, x->stream));
  return 0;
}

// ---------------------------------------------------------------------------
// family dispatch: one entry per family TU; op selects what to launch
// ---------------------------------------------------------------------------
enum {
  NMC_OP_RUN = 0,          // step kernel over iterations [i0, i1) with flags
  NMC_OP_CAN_PERSIST = 1,  // result = 1 if the persistent grid is co-resident
  NMC_OP_GROUP_LL = 2,     // in = theta [P][G][C] (device), out = [G][C] (device)
  NMC_OP_OBS_LL = 3,       // in = values [P][G][C] (device), out = [C][n_obs] (device)
  NMC_OP_OBS_LL_ROWS = 4,  // sample rows [i0, i1), chains [c0, c0 + nc) -> out = [nc][i1 - i0][n_obs]
  NMC_OP_CAPACITY = 5,     // result = resident step-kernel workgroups on the device
  NMC_OP_RES_OK = 6        // result = 1: the run mode has a resident instance, grid co-resident
};
struct NmcCall {
  int op = 0;
  int i0 = 0, i1 = 0, flags = 0;
  int res = 0;             // NMC_OP_RUN: the resident instance (Dev.rcmd set)
  int c0 = 0, nc = 0;      // NMC_OP_OBS_LL_ROWS: chains [c0, c0 + nc) (nc = 0: every chain)
  const double* in = nullptr;
  double* out = nullptr;
  double* aux = nullptr;   // op-specific device scratch
  int result = 0;
  int result2 = 0;         // NMC_OP_RES_OK: the resident instance's VGPRs per lane
};
int nmc_call_linreg(nmc_ctx* x, NmcCall& c);
int nmc_call_gauss_mean(nmc_ctx* x, NmcCall& c);
int nmc_call_logistic(nmc_ctx* x, NmcCall& c);

// user families (user.hip): runtime-compiled FamUser modules, ids >= NMC_LL_USER_BASE
int nmc_call_user(nmc_ctx* x, NmcCall& c);
int nmc_user_attach(nmc_ctx* x, int family);   // load the module on x's device, check shapes

// the sweep kernel's launches and occupancy queries (sweep_*.hip)
int nmc_sweep_linreg(nmc_ctx* x, NmcCall& c);
int nmc_sweep_gauss_mean(nmc_ctx* x, NmcCall& c);
int nmc_sweep_logistic(nmc_ctx* x, NmcCall& c);

static inline int nmc_call_family(nmc_ctx* x, NmcCall& c) {
  if (x->sweep && x->family < NMC_LL_USER_BASE &&
      (c.op == NMC_OP_RUN || c.op == NMC_OP_CAN_PERSIST || c.op == NMC_OP_CAPACITY)) {
    switch (x->family) {
      case NMC_LL_LINREG: return nmc_sweep_linreg(x, c);
      case NMC_LL_GAUSS_MEAN: return nmc_sweep_gauss_mean(x, c);
      case NMC_LL_LOGISTIC: return nmc_sweep_logistic(x, c);
    }
  }
  switch (x->family) {
    case NMC_LL_LINREG: return nmc_call_linreg(x, c);
    case NMC_LL_GAUSS_MEAN: return nmc_call_gauss_mean(x, c);
    case NMC_LL_LOGISTIC: return nmc_call_logistic(x, c);
  }
  if (x->family >= NMC_LL_USER_BASE) return nmc_call_user(x, c);
  return nmc_fail(-1, "unknown likelihood family");
}
