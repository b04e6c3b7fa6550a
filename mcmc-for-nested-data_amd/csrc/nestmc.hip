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

#include <string>
#include <utility>
#include <vector>
#include <algorithm>

#include "../../include/nestmc.h"
#include "kernels.h"

#define NMC_VERSION "nestmc 0.1.0 (gfx950)"

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      return fail(-2, std::string(#x) + ": " + hipGetErrorString(e_));                \
  } while (0)

struct nmc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
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
  int stamp_blocks = 0;
  double* vbuf[2] = {nullptr, nullptr};   // value ping-pong ([P][G][C] each)
  int vcur = 0;
};

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

// ---------------------------------------------------------------------------
// family dispatch: (family, n_fields) -> concrete functor type
// ---------------------------------------------------------------------------
template <int NF>
static FamLinreg<NF> make_linreg(const std::vector<double>& c) {
  FamLinreg<NF> f{};
  f.intercept = (int)c[1];
  f.sigma_known = c[2];
  f.log_sigma_known = c.size() > 3 ? c[3] : 0.0;
  return f;
}
template <int NF>
static FamGaussMean<NF> make_gauss(const std::vector<double>& c) {
  FamGaussMean<NF> f{};
  for (int j = 0; j < NF; ++j) { f.sd[j] = c[j]; f.lsd[j] = c[NF + j]; }
  return f;
}
template <int NF>
static FamLogistic<NF> make_logistic(const std::vector<double>& c) {
  FamLogistic<NF> f{};
  f.intercept = (int)c[1];
  return f;
}

template <int NF, class Fn>
static int with_nf(nmc_ctx* x, Fn&& fn) {
  switch (x->family) {
    case NMC_LL_LINREG: return fn(make_linreg<NF>(x->llc));
    case NMC_LL_GAUSS_MEAN: return fn(make_gauss<NF>(x->llc));
    case NMC_LL_LOGISTIC: return fn(make_logistic<NF>(x->llc));
  }
  return fail(-1, "unknown likelihood family");
}

template <class Fn>
static int with_family(nmc_ctx* x, Fn&& fn) {
  switch (x->nf) {
    case 1: return with_nf<1>(x, fn);
    case 2: return with_nf<2>(x, fn);
    case 3: return with_nf<3>(x, fn);
    case 4: return with_nf<4>(x, fn);
    case 5: return with_nf<5>(x, fn);
    case 6: return with_nf<6>(x, fn);
    case 7: return with_nf<7>(x, fn);
    case 8: return with_nf<8>(x, fn);
    case 9: return with_nf<9>(x, fn);
  }
  return fail(-1, "n_fields must be 1..9");
}

static int choose_waves(int CB, int G, int64_t n_obs) {
  if (const char* e = getenv("NMC_WAVES")) {
    int w = atoi(e);
    if (w >= 1 && w <= 8) return w;
  }
  const int64_t wgs = (int64_t)CB * G;
  int64_t w = (2048 + wgs - 1) / wgs;                 // ~8 waves per CU on 256 CUs
  const int64_t navg = G > 0 ? n_obs / G : 0;
  const int64_t wmax_rows = navg / 32 > 1 ? navg / 32 : 1;   // >= 32 rows per wave
  if (w > wmax_rows) w = wmax_rows;
  if (w > 8) w = 8;                 // nmc_k_iter launch bound: 512 threads
  if (w < 1) w = 1;
  return (int)w;
}

static int pop_event_pair(nmc_ctx* x, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v,
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

static int nacc_of(const nmc_ctx* x) { return x->family == NMC_LL_GAUSS_MEAN ? x->nf : 1; }

// One launch per iteration: reads the current value buffer, writes the other one.
template <class Fam>
static int launch_iter(nmc_ctx* x, const Fam& fam, int iter) {
  Dev& d = x->d;
  const nmc_lds_layout L = nmc_lds(d.stage_rows, Fam::NFIELDS, d.W, Fam::NACC, d.P);
  const size_t lds = (size_t)L.total * sizeof(double);
  double* src = x->vbuf[x->vcur];
  double* dst = x->vbuf[x->vcur ^ 1];
  d.value = src;
  std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
  if (x->ktiming) {
    if (int rc = pop_event_pair(x, x->kev, x->kev_used, &ev)) return rc;
    HIPCHK(hipEventRecord(ev->first, x->stream));
  }
  if (d.stage_rows)
    hipLaunchKernelGGL((nmc_k_iter<Fam, true>), dim3(d.CB * d.G), dim3(64 * d.W), lds,
                       x->stream, d, fam, d.obs, (const double*)src, dst, iter);
  else
    hipLaunchKernelGGL((nmc_k_iter<Fam, false>), dim3(d.CB * d.G), dim3(64 * d.W), lds,
                       x->stream, d, fam, d.obs, (const double*)src, dst, iter);
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev->second, x->stream));
  x->vcur ^= 1;
  d.value = dst;
  return 0;
}

// Gibbs update of every parameter at iteration hiter (closes a chunk of iterations).
static int launch_hyper(nmc_ctx* x, int hiter) {
  std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
  if (x->ktiming) {
    if (int rc = pop_event_pair(x, x->hev, x->hev_used, &ev)) return rc;
    HIPCHK(hipEventRecord(ev->first, x->stream));
  }
  x->d.value = x->vbuf[x->vcur];
  const size_t lds = (size_t)12 * x->P * 64 * sizeof(double);
  hipLaunchKernelGGL(nmc_k_hyper, dim3(x->d.CB), dim3(64 * x->d.W), lds, x->stream, x->d,
                     hiter);
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev->second, x->stream));
  return 0;
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

  nmc_ctx* x = new nmc_ctx();
  x->device = device;
  x->C = n_chains; x->chain_base = chain_base; x->G = n_groups; x->P = n_params;
  x->pooling = pooling; x->family = ll_family; x->nf = n_fields; x->seed = seed;
  x->rng = rng_mode; x->n_obs = n_obs;
  x->llc.assign(ll_consts, ll_consts + n_ll_consts);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete x; return fail(-2, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
  e = hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking);
  if (e != hipSuccess) { delete x; return fail(-2, std::string("hipStreamCreate: ") + hipGetErrorString(e)); }
  for (auto& ev : x->ev) hipEventCreate(&ev);

  Dev& d = x->d;
  const size_t PGC = (size_t)n_params * n_groups * n_chains, GC = (size_t)n_groups * n_chains,
               PC = (size_t)n_params * n_chains;
  int rc = 0;
  int64_t* off = nullptr;
  double* dobs = nullptr;
  int* pf = nullptr;
  double* pp = nullptr;
  rc |= dalloc(x, &off, n_groups + 1);
  rc |= dalloc(x, &dobs, (size_t)n_obs * n_fields);
  rc |= dalloc(x, &pf, n_params);
  rc |= dalloc(x, &pp, (size_t)8 * n_params);
  rc |= dalloc(x, &x->vbuf[0], PGC);
  rc |= dalloc(x, &x->vbuf[1], PGC);
  d.value = x->vbuf[0];
  rc |= dalloc(x, &d.lp, PGC);
  rc |= dalloc(x, &d.ll, GC);
  rc |= dalloc(x, &d.scale, PGC);
  rc |= dalloc(x, &d.nacc, PGC);
  rc |= dalloc(x, &d.nrej, PGC);
  rc |= dalloc(x, &d.tacc, PGC);
  rc |= dalloc(x, &d.mu, PC);
  rc |= dalloc(x, &d.s2, PC);
  rc |= dalloc(x, &d.hsd, PC);
  rc |= dalloc(x, &d.hlsd, PC);
  if (rc) { nmc_destroy(x); return rc; }
  d.off = off; d.obs = dobs; d.pfam = pf; d.ppar = pp;
  d.C = n_chains; d.G = n_groups; d.P = n_params; d.pooling = pooling; d.nf = n_fields;
  d.chain_base = chain_base; d.rng_mode = rng_mode; d.seed = seed;
  d.CB = (n_chains + 63) / 64;
  d.W = choose_waves(d.CB, n_groups, n_obs);
  d.ha = (n_groups - 1) / 2.0;
  d.hlga = lgamma(d.ha > 0 ? d.ha : 1.0);
  {
    // stage each group's rows in LDS when the whole workgroup carve fits 96 KiB
    int64_t nmax = 0;
    for (int g = 0; g < n_groups; ++g)
      nmax = std::max<int64_t>(nmax, group_offsets[g + 1] - group_offsets[g]);
    const int nacc = ll_family == NMC_LL_GAUSS_MEAN ? n_fields : 1;
    const nmc_lds_layout L = nmc_lds((int)std::min<int64_t>(nmax, 1 << 20), n_fields, d.W,
                                     nacc, n_params);
    d.stage_rows = ((size_t)L.total * 8 <= (size_t)96 * 1024 && !getenv("NMC_NO_STAGE"))
                       ? (int)nmax : 0;
  }
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
  if (x->stream) hipStreamSynchronize(x->stream);
  for (void* p : x->owned) if (p) hipFree(p);
  for (auto& ev : x->ev) if (ev) hipEventDestroy(ev);
  for (auto& pr : x->kev) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  for (auto& pr : x->hev) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  if (x->stream) hipStreamDestroy(x->stream);
  delete x;
  return 0;
}

int nmc_set_state(nmc_ctx* x, const double* value, const double* log_prior, const double* ll,
                  const double* hyper_mu, const double* hyper_sigma2, const double* scale) {
  hipSetDevice(x->device);
  Dev& d = x->d;
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C, PC = (size_t)x->P * x->C;
  HIPCHK(hipMemcpy(d.value, value, PGC * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d.lp, log_prior, PGC * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d.ll, ll, GC * 8, hipMemcpyHostToDevice));
  if (x->pooling == NMC_POOL_PARTIAL) {
    if (!hyper_mu || !hyper_sigma2) return fail(-1, "partial pooling needs hyper_mu/hyper_sigma2");
    std::vector<double> sd(PC), lsd(PC);
    for (size_t i = 0; i < PC; ++i) { sd[i] = sqrt(hyper_sigma2[i]); lsd[i] = log(sd[i]); }
    HIPCHK(hipMemcpy(d.mu, hyper_mu, PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.s2, hyper_sigma2, PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.hsd, sd.data(), PC * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.hlsd, lsd.data(), PC * 8, hipMemcpyHostToDevice));
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
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  Dev& d = x->d;
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C, PC = (size_t)x->P * x->C;
  if (value) HIPCHK(hipMemcpy(value, d.value, PGC * 8, hipMemcpyDeviceToHost));
  if (log_prior) HIPCHK(hipMemcpy(log_prior, d.lp, PGC * 8, hipMemcpyDeviceToHost));
  if (ll) HIPCHK(hipMemcpy(ll, d.ll, GC * 8, hipMemcpyDeviceToHost));
  if (hyper_mu) HIPCHK(hipMemcpy(hyper_mu, d.mu, PC * 8, hipMemcpyDeviceToHost));
  if (hyper_sigma2) HIPCHK(hipMemcpy(hyper_sigma2, d.s2, PC * 8, hipMemcpyDeviceToHost));
  if (scale) HIPCHK(hipMemcpy(scale, d.scale, PGC * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_set_replay(nmc_ctx* x, const double* z, const double* u, const double* hz,
                   const double* hu, int n_iter) {
  hipSetDevice(x->device);
  Dev& d = x->d;
  const size_t n = (size_t)n_iter * x->P * x->G * x->C, nh = (size_t)n_iter * x->P * x->C;
  double *rz, *ru, *rhz, *rhu;
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
  // variate ring: a chunk of iterations' worth of pre-drawn variates (<= ~1 GiB)
  const size_t per_iter = ((size_t)2 * x->P * x->G * x->C + (size_t)2 * x->P * x->C) * 8;
  size_t budget = (size_t)1 << 30;
  if (const char* e = getenv("NMC_VARIATE_BYTES")) budget = (size_t)atoll(e);
  int vcap = (int)(budget / per_iter);
  if (vcap < 1) vcap = 1;
  if (vcap > n_iter) vcap = n_iter > 0 ? n_iter : 1;
  dfree(x, d.vz); dfree(x, d.vlu); dfree(x, d.vhz); dfree(x, d.vhx);
  const size_t PGC = (size_t)x->P * x->G * x->C, PC = (size_t)x->P * x->C;
  rc = dalloc(x, &d.vz, vcap * PGC) | dalloc(x, &d.vlu, vcap * PGC) |
       dalloc(x, &d.vhz, vcap * PC) | dalloc(x, &d.vhx, vcap * PC);
  if (rc) return rc;
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
  hipSetDevice(x->device);
  x->trace = enable != 0;
  return alloc_trace(x);
}

int nmc_get_trace(nmc_ctx* x, uint8_t* accept, double* ll_prop) {
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  if (!x->d.trace_n) return fail(-1, "trace not enabled");
  const size_t n = (size_t)x->d.trace_n * x->P * x->G * x->C;
  if (accept) HIPCHK(hipMemcpy(accept, x->d.tflag, n, hipMemcpyDeviceToHost));
  if (ll_prop) HIPCHK(hipMemcpy(ll_prop, x->d.tllp, n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_run(nmc_ctx* x, int iter_begin, int iter_end) {
  hipSetDevice(x->device);
  if (!x->scheduled) return fail(-1, "nmc_set_schedule first");
  if (iter_begin < 0 || iter_end < iter_begin) return fail(-1, "invalid iteration range");
  if (iter_begin == iter_end) return 0;
  if (x->rng == NMC_RNG_REPLAY && (!x->d.rz || iter_end > x->d.replay_n))
    return fail(-1, "replay variates do not cover the iteration range");
  const bool partial = x->pooling == NMC_POOL_PARTIAL;
  const int P = x->P;
  return with_family(x, [&](auto fam) -> int {
    for (int c0 = iter_begin; c0 < iter_end; c0 += x->d.vcap) {
      const int c1 = c0 + x->d.vcap < iter_end ? c0 + x->d.vcap : iter_end;
      // every variate of iterations [c0, c1) in one fully parallel launch
      x->d.vbase = c0;
      const size_t n = (size_t)(c1 - c0) * P * x->C * (x->G + (partial ? 1 : 0));
      const int blocks = (int)((n + 255) / 256 < 16384 ? (n + 255) / 256 : 16384);
      hipLaunchKernelGGL(nmc_k_fill, dim3(blocks), dim3(256), 0, x->stream, x->d, c0, c1 - c0);
      HIPCHK(hipGetLastError());
      for (int it = c0; it < c1; ++it)
        if (int rc = launch_iter(x, fam, it)) return rc;
      // close the chunk: the last Gibbs update reads this chunk's variates
      if (partial)
        if (int rc = launch_hyper(x, c1 - 1)) return rc;
    }
    return 0;
  });
}

int nmc_synchronize(nmc_ctx* x) {
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  return 0;
}

int nmc_get_samples(nmc_ctx* x, int row_begin, int n_rows, double* out) {
  hipSetDevice(x->device);
  const Dev& d = x->d;
  if (row_begin < 0 || n_rows < 0 || row_begin + n_rows > d.n_rows)
    return fail(-1, "row range out of bounds");
  HIPCHK(hipStreamSynchronize(x->stream));
  const size_t per = (size_t)d.cols * x->C;
  if (n_rows)
    HIPCHK(hipMemcpy(out, d.samples + (size_t)row_begin * per, (size_t)n_rows * per * 8,
                     hipMemcpyDeviceToHost));
  return 0;
}

int nmc_get_accept_counts(nmc_ctx* x, int64_t* out) {
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  HIPCHK(hipMemcpy(out, x->d.tacc, (size_t)x->P * x->G * x->C * 8, hipMemcpyDeviceToHost));
  return 0;
}

int nmc_eval_group_ll(nmc_ctx* x, const double* theta, double* out) {
  hipSetDevice(x->device);
  const size_t PGC = (size_t)x->P * x->G * x->C, GC = (size_t)x->G * x->C;
  double *th = nullptr, *o = nullptr;
  HIPCHK(hipMalloc(&th, PGC * 8));
  HIPCHK(hipMalloc(&o, GC * 8));
  HIPCHK(hipMemcpyAsync(th, theta, PGC * 8, hipMemcpyHostToDevice, x->stream));
  int rc = with_family(x, [&](auto fam) -> int {
    using F = decltype(fam);
    const size_t lds = (size_t)x->d.W * 64 * F::NACC * sizeof(double);
    hipLaunchKernelGGL(nmc_k_group_ll<F>, dim3(x->d.CB * x->G), dim3(64 * x->d.W), lds,
                       x->stream, x->d, fam, x->d.obs, (const double*)th, o);
    HIPCHK(hipGetLastError());
    return 0;
  });
  if (!rc) {
    hipError_t e = hipMemcpyAsync(out, o, GC * 8, hipMemcpyDeviceToHost, x->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
    if (e != hipSuccess) rc = fail(-2, std::string("eval_group_ll: ") + hipGetErrorString(e));
  }
  hipFree(th);
  hipFree(o);
  return rc;
}

int nmc_eval_obs_ll(nmc_ctx* x, double* out) {
  hipSetDevice(x->device);
  const size_t n = (size_t)x->C * x->n_obs;
  double* o = nullptr;
  HIPCHK(hipMalloc(&o, (n ? n : 1) * 8));
  int rc = with_family(x, [&](auto fam) -> int {
    using F = decltype(fam);
    hipLaunchKernelGGL(nmc_k_obs_ll<F>, dim3(x->d.CB * x->G), dim3(64), 0, x->stream, x->d,
                       fam, o, x->n_obs);
    HIPCHK(hipGetLastError());
    return 0;
  });
  if (!rc && n) {
    hipError_t e = hipMemcpyAsync(out, o, n * 8, hipMemcpyDeviceToHost, x->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
    if (e != hipSuccess) rc = fail(-2, std::string("eval_obs_ll: ") + hipGetErrorString(e));
  }
  hipFree(o);
  return rc;
}

int nmc_event_record(nmc_ctx* x, int slot) {
  if (slot < 0 || slot >= 16) return fail(-1, "event slot 0..15");
  hipSetDevice(x->device);
  HIPCHK(hipEventRecord(x->ev[slot], x->stream));
  return 0;
}

int nmc_event_elapsed(nmc_ctx* x, int a, int b, float* ms) {
  if (a < 0 || a >= 16 || b < 0 || b >= 16) return fail(-1, "event slot 0..15");
  hipSetDevice(x->device);
  HIPCHK(hipEventSynchronize(x->ev[b]));
  HIPCHK(hipEventElapsedTime(ms, x->ev[a], x->ev[b]));
  return 0;
}

int nmc_set_kernel_timing(nmc_ctx* x, int enable) {
  x->ktiming = enable != 0;
  x->kev_used = x->hev_used = 0;
  x->step_ms = x->hyper_ms = 0;
  x->step_n = x->hyper_n = 0;
  return 0;
}

int nmc_get_kernel_timing(nmc_ctx* x, double* step_ms, int64_t* step_n, double* hyper_ms,
                          int64_t* hyper_n) {
  hipSetDevice(x->device);
  HIPCHK(hipStreamSynchronize(x->stream));
  for (size_t i = 0; i < x->kev_used; ++i) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, x->kev[i].first, x->kev[i].second));
    x->step_ms += ms;
    x->step_n += 1;
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
  if (hyper_ms) *hyper_ms = x->hyper_ms;
  if (hyper_n) *hyper_n = x->hyper_n;
  return 0;
}

int nmc_launch_config(nmc_ctx* x, int* waves_per_group, int* chain_blocks) {
  *waves_per_group = x->d.W;
  *chain_blocks = x->d.CB;
  return 0;
}

// ---------------------------------------------------------------------------
// CSV output with the reference's formatting (Python "%f" == C "%f" except the
// spelling of NaN, which Python always prints as "nan").
// ---------------------------------------------------------------------------
static inline void put_f(std::string& s, double v) {
  char buf[512];
  if (isnan(v)) { s += "nan"; return; }
  if (isinf(v)) { s += v > 0 ? "inf" : "-inf"; return; }
  int n = snprintf(buf, sizeof(buf), "%f", v);
  if (n >= (int)sizeof(buf)) {
    std::vector<char> big(n + 1);
    snprintf(big.data(), big.size(), "%f", v);
    s += big.data();
  } else {
    s.append(buf, n);
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

int nmc_gather_samples(nmc_ctx* x, void* comm, int root, double* host_out) {
  hipSetDevice(x->device);
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0, rank = 0;
  ncclCommCount(c, &nranks);
  ncclCommUserRank(c, &rank);
  const size_t count = (size_t)x->d.n_rows * x->d.cols * x->C;
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

int nmc_debug_stamps(nmc_ctx* x, int n_blocks, uint64_t* out) {
  // n_blocks > 0: (re)allocate and zero [n_blocks][8]; out != NULL: copy back.
  hipSetDevice(x->device);
  if (n_blocks > 0) {
    dfree(x, x->d.stamps);
    x->d.stamps = nullptr;
    if (int rc = dalloc(x, &x->d.stamps, (size_t)n_blocks * 8)) return rc;
    HIPCHK(hipMemset(x->d.stamps, 0, (size_t)n_blocks * 64));
    x->stamp_blocks = n_blocks;
  }
  if (out) {
    HIPCHK(hipStreamSynchronize(x->stream));
    HIPCHK(hipMemcpy(out, x->d.stamps, (size_t)x->stamp_blocks * 64, hipMemcpyDeviceToHost));
  }
#ifdef NMC_STAMPS
  return 0;
#else
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

}  // extern "C"
