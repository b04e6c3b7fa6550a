/*
 * nestmc.h -- C-ABI of libnestmc.so, the MI355X (gfx950) engine for the MCMC
 * inner loop of tkngch/MCMC-for-Nested-Data.
 *
 * The reference has no FFI: its hot path is Python (posteriorSampling.py).  Each
 * entry point below replaces a piece of that Python, cited file:line, and is
 * bound by the drop-in Python host (mcmc-for-nested-data_amd/nestmc/_lib.py)
 * through ctypes.  Plain C types only; all host buffers are caller-owned and
 * copied; device buffers are owned by the context.  Every function returns 0 on
 * success and a negative code on failure, with the message in nmc_last_error()
 * (thread-local).  A context is used by one host thread at a time.
 *
 * Array layouts (all fp64 unless noted; "c" = local chain, fastest-varying):
 *   value, log_prior, scale  [P][G][C]       ll           [G][C]
 *   (on the device the values after iteration t live in one of two buffers, t & 1)
 *   hyper mu, sigma2         [P][C]          samples      [row][col][C]
 *   replay z, u              [iter][P][G][C] replay hz, hu [iter][P][C]
 *   obs                      [n_obs][n_fields] (group-major, CSR by group_offsets)
 */
#ifndef NESTMC_H
#define NESTMC_H

#ifndef __HIPCC_RTC__
#include <stdint.h>
#else   /* hiprtc (runtime-compiled user families): its own fixed-width types */
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint64_t uintptr_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nmc_ctx nmc_ctx;

/* pooling: StepMethod subclasses, posteriorSampling.py:662-787 */
enum { NMC_POOL_COMPLETE = 0, NMC_POOL_NONE = 1, NMC_POOL_PARTIAL = 2 };

/* likelihood families: device restatements of the user logLikelihoodFunction
 * contract (posteriorSampling.py:61-102) for the models the reference ships or
 * benchmarks (example/regression.py:53-67, example/distribution.py:18-24, cfg 5).
 *   NMC_LL_LINREG    obs = [x_1..x_k, y] (+ implicit ones column if consts[1]=1)
 *                    consts = {k, intercept, sigma (<=0: sigma is the last param)}
 *   NMC_LL_GAUSS_MEAN obs = [m_0..m_{P-1}]; consts = {sd_0..sd_{P-1}}
 *   NMC_LL_LOGISTIC  obs = [x_1..x_k, y]; consts = {k, intercept}              */
enum { NMC_LL_LINREG = 0, NMC_LL_GAUSS_MEAN = 1, NMC_LL_LOGISTIC = 2 };
/* User families (the reference's arbitrary logLikelihoodFunction, :61-102, as device
 * code): ids >= NMC_LL_USER_BASE come from nmc_user_family_compile; consts = the model's
 * constants, passed to the user function as k.                                     */
enum { NMC_LL_USER_BASE = 100 };

/* prior families for none/complete pooling: scipy frozen distributions the
 * reference evaluates with .logpdf (posteriorSampling.py:293-294).
 * params[8] per parameter = {loc, scale, shape, gammaln(shape), log(scale), 0,0,0}
 * (gammaln and log(scale) computed on the host with scipy/numpy).            */
enum { NMC_PRIOR_NORM = 0, NMC_PRIOR_GAMMA = 1, NMC_PRIOR_UNIFORM = 2,
       NMC_PRIOR_EXPON = 3, NMC_PRIOR_HALFNORM = 4, NMC_PRIOR_CAUCHY = 5,
       NMC_PRIOR_LAPLACE = 6, NMC_PRIOR_LOGNORM = 7, NMC_PRIOR_INVGAMMA = 8 };

/* random streams: philox = device Philox4x32-10 (replaces numpy legacy MT19937
 * draws at posteriorSampling.py:306,362,487,498); replay = variates supplied by
 * nmc_set_replay (captured from the reference, for parity).                    */
enum { NMC_RNG_PHILOX = 0, NMC_RNG_REPLAY = 1 };

const char* nmc_last_error(void);
const char* nmc_version(void);
int nmc_device_count(int* n);

/* Replaces the per-chain StepMethod construction (posteriorSampling.py:517-582,
 * :1146-1151): CSR offsets (:554-555), data, priors.  chain_base = global id of
 * local chain 0 (Philox key, posteriorSampling.py:225 seed = chain).           */
/* Compile a user log-likelihood (hiprtc, gfx950) and register it as a family:
 *   source defines  __device__ double nmc_user_loglik(const double* theta,  // [n_params]
 *                                                     const double* row,    // [n_fields]
 *                                                     const double* k);     // consts
 * returning ONE observation's log-likelihood (the reference's logLikelihoodFunction,
 * posteriorSampling.py:61-102, evaluated per row); include_dir = the library's csrc
 * directory (kernels.h, fam_user.h).  *family_id -> pass as nmc_create's ll_family.
 * Errors carry the compiler log (nmc_last_error).                                  */
int nmc_user_family_compile(const char* source, int n_fields, int n_params,
                            const char* include_dir, int* family_id);
int nmc_user_family_shape(int family_id, int* n_fields, int* n_params);

int nmc_create(nmc_ctx** out, int device, int n_chains, int chain_base,
               int n_groups, int n_params, int pooling, int ll_family,
               const double* ll_consts, int n_ll_consts,
               const int64_t* group_offsets, const double* obs, int64_t n_obs,
               int n_fields, const int* prior_family, const double* prior_params,
               uint32_t seed, int rng_mode);
int nmc_destroy(nmc_ctx* ctx);

/* Chain state after initialisation (PartialPooling._initialiseParameters /
 * _determineIndividualStartingPoint :725-758; StepMethod._setStartingPoint
 * :584-592).  hyper_* may be NULL for none/complete; scale NULL -> 1.0.      */
int nmc_set_state(nmc_ctx* ctx, const double* value, const double* log_prior,
                  const double* ll, const double* hyper_mu, const double* hyper_sigma2,
                  const double* scale);
int nmc_get_state(nmc_ctx* ctx, double* value, double* log_prior, double* ll,
                  double* hyper_mu, double* hyper_sigma2, double* scale);

/* Replay variates [n_iter] (RNG mode NMC_RNG_REPLAY). */
int nmc_set_replay(nmc_ctx* ctx, const double* z, const double* u,
                   const double* hz, const double* hu, int n_iter);

/* Sampler.sample schedule (posteriorSampling.py:827-860, MCMC.__init__
 * :1018-1027): allocates the device sample store for every recorded row.     */
int nmc_set_schedule(nmc_ctx* ctx, int n_iter, int burn, int thin, int tune_interval);
int nmc_n_rows(nmc_ctx* ctx, int* rows, int* cols);

/* Optional per-step trace [n_iter][P][G][C]: accept flags (uint8) and the
 * proposal's group log-likelihood; for parity tests.                         */
int nmc_set_trace(nmc_ctx* ctx, int enable);
int nmc_get_trace(nmc_ctx* ctx, uint8_t* accept, double* ll_prop);

/* Sampler._loop (posteriorSampling.py:862-896) for iterations [iter_begin,
 * iter_end): StepMethod.step (:594-613) + HyperParameter.update (:463-498)
 * + the recorder (:887-889) into the device sample store.  Asynchronous on the
 * context's stream; call nmc_synchronize before reading results.
 * The variates of a launch chunk are drawn before it; the next chunk's (the
 * rest of the call, then as many iterations again after it, within the
 * schedule) are drawn on a second stream beside the chunk's step launch and
 * taken by the chunk or call that starts there (NMC_PREFILL=0: off).  The
 * variates depend on (seed, chain, iteration) alone: results are identical.  */
int nmc_run(nmc_ctx* ctx, int iter_begin, int iter_end);
/* Waits for everything nmc_run / nmc_prefill enqueued (both streams).         */
int nmc_synchronize(nmc_ctx* ctx);
/* Draw the variates of iterations [iter_begin, iter_end) (at most one buffer's
 * worth) now, beside whatever runs, for a later nmc_run that starts at
 * iter_begin: a caller that knows its next call's range (replaces nmc_run's
 * own guess).  No effect on results.  iter_end <= the schedule's n_iter.      */
int nmc_prefill(nmc_ctx* ctx, int iter_begin, int iter_end);
/* Iterations drawn by prefills so far / taken by nmc_run from a prefill.      */
int nmc_prefill_stats(nmc_ctx* ctx, int64_t* issued, int64_t* used);
/* Resident step launch for the consecutive nmc_run calls of a sampling loop
 * (Sampler._loop :872-891 driven in chunks, e.g. samplePosterior's progress
 * steps): a call that continues where the previous one ended is handed to the
 * running launch (a command word in pinned host memory) instead of a new launch;
 * the rows and chain state stay in LDS.  Each call completes its results as a
 * launch does -- after nmc_synchronize its sample / trace rows and hyper-
 * parameters are in HBM, bit for bit those of separate launches; the chain
 * state reaches HBM when the launch parks.  Any other entry point parks the
 * launch first (so every read sees the state of separate launches); it parks
 * itself after NMC_RESIDENT_IDLE_US (20 ms) without a call.  No effect where
 * the context's kernel has no resident form (enabled 0 in nmc_resident_stats).
 * No reference counterpart: host plumbing.                                   */
int nmc_set_resident(nmc_ctx* ctx, int enable);
/* enabled: resident launches possible and on; active: one is running now;
 * launches / calls: resident launches made / calls continued inside one;
 * last_refusal: why the latest call not continued was not (1 another start,
 * 2 kernel timing, 3 longer than a chunk, 4 past the launch's variate buffer,
 * 5 variates not prefilled there, 6 counters would wrap, 7 the launch had
 * parked itself after its idle limit, 8 its prefill did not finish beside
 * the launch within 2 ms -- kernels serialized, e.g. by a profiler's counter
 * pass: the resident form is then turned off for the context).               */
int nmc_resident_stats(nmc_ctx* ctx, int* enabled, int* active, int64_t* launches,
                       int64_t* calls, int* last_refusal);

/* Recorded rows [row_begin, row_begin+n_rows) as [row][col][C].
 * Columns follow StepMethod.values / PartialPooling.values (:648-654, :780-787). */
int nmc_get_samples(nmc_ctx* ctx, int row_begin, int n_rows, double* out);
/* Total accepted proposals per (p, g, c) since nmc_set_state. */
int nmc_get_accept_counts(nmc_ctx* ctx, int64_t* out);

/* StepMethod._computeParameterLogLikelihood (:629-635) on device for arbitrary
 * values theta[P][G][C] -> out[G][C] (used by the host init loop :746-758).  */
int nmc_eval_group_ll(nmc_ctx* ctx, const double* theta, double* out);
/* StepMethod.logLikelihood (:656-659): per-observation LL at the current state,
 * out[C][n_obs] (saveLogLikelihood rows, :907-909).                          */
int nmc_eval_obs_ll(nmc_ctx* ctx, double* out);
/* The same at recorded rows [row_begin, row_begin+n_rows) of the sample store -- the
 * state Sampler._printLogLikelihood (:890-891) evaluated at each recorded iteration:
 * out[C][n_rows][n_obs].                                                       */
int nmc_obs_ll_rows(nmc_ctx* ctx, int row_begin, int n_rows, double* out);
/* saveLogLikelihood=True (:890-891, :907-909): logLikelihood.<chain_ids[c]>.csv in dir
 * (a path prefix ending in '/') for every local chain and recorded row, "%f" joined by
 * ",".  Batches of rows are evaluated on the device and copied to pinned memory while
 * the host formats the previous batch with `threads` threads; a chain whose id is
 * negative gets no file (a rank's padding chains).                             */
int nmc_write_ll_csvs(nmc_ctx* ctx, const char* dir, const int32_t* chain_ids, int threads);

/* Timing on the context's stream (hipEvents). */
int nmc_event_record(nmc_ctx* ctx, int slot);                 /* slot 0..15 */
int nmc_event_elapsed(nmc_ctx* ctx, int slot_a, int slot_b, float* ms);
/* Bracket every step launch with events (adds a little overhead): per-kernel
 * average duration for the roofline; step_iters = iterations those launches ran. */
int nmc_set_kernel_timing(nmc_ctx* ctx, int enable);
int nmc_get_kernel_timing(nmc_ctx* ctx, double* step_ms_total, int64_t* step_launches,
                          int64_t* step_iters, double* hyper_ms_total, int64_t* hyper_launches);
/* Cap the iterations one persistent launch covers (0 = the variate chunk, the
 * default); e.g. equal-length launches for profiling.                           */
int nmc_set_launch_iters(nmc_ctx* ctx, int max_iters);
/* Launch geometry of the step kernel: waves per workgroup, chain blocks, whether one
 * resident launch runs a whole chunk of iterations (1) or one launch per iteration
 * (0), chains per workgroup (64, or 32 in the half-lane layout) and the kernel mode
 * (0 none/complete, 1 launch per iteration, 2 persistent sync, 3 LDS Gibbs payload,
 * 4 register Gibbs hand-off, 5 pair); chains_per_block and mode may be NULL.      */
int nmc_launch_config(nmc_ctx* ctx, int* waves_per_group, int* chain_blocks, int* persistent,
                      int* chains_per_block, int* mode);
/* Row split of none/complete pooling (CompletePooling._setGroupIndex :667-671 puts every
 * observation in ONE group): members = workgroups sharing each (chain block, group),
 * exchanging partial sums every step (1: no split); chain blocks per resident launch. */
int nmc_split_config(nmc_ctx* ctx, int* members, int* chain_blocks_per_launch);
/* The step kernel a run launches, e.g. "nmc_k_step<FamLinreg<2>, NMC_MODE_SYNC_REG>"
 * (NUL-terminated, truncated to cap bytes); for the profiles and the bench report.    */
int nmc_kernel_name(nmc_ctx* ctx, char* out, int cap);
/* Where a run's per-step variates come from: *in_kernel = 1 when the step kernel draws
 * them itself (no nmc_k_fill launch for them), 0 when nmc_k_fill writes them to a ring in
 * HBM first.  Both give the same bits (Parameter.propose :304-306, the accept draw :362). */
int nmc_variate_source(nmc_ctx* ctx, int* in_kernel);
/* Partial pooling over G > 128 groups runs the Gibbs update (HyperParameter.update
 * :463-498, once per chain block) as a kernel of its own beside the step kernel; when the
 * two did not run at the same time (a profiler or AMD_SERIALIZE_KERNEL serializes kernels)
 * the step kernel updated that launch's tasks itself, with the same results.  *out = the
 * (launch, chain block) pairs that did so since nmc_create (diagnostics and tests).     */
int nmc_gibbs_fallbacks(nmc_ctx* ctx, int64_t* out);

/* Sampler._printSample (:902-905) + _print (:933-936): append rows of local
 * chain c to a CSV file with the reference's "%i,%i,%f,..." formatting (and the
 * header line of :898-900 when header != NULL).  Host only; thread-safe.     */
int nmc_write_sample_csv(const char* path, int append, const char* header,
                         const double* samples, int n_chains, int c, int cols,
                         const int32_t* row_index, int n_rows, int chain_id);
/* _printLogLikelihood (:907-909): one "%f,..." line per row of ll[n_rows][n]. */
int nmc_write_ll_csv(const char* path, int append, const double* ll, int64_t n,
                     int n_rows);

/* Multi-GPU (replaces the process-per-chain fan-out, posteriorSampling.py:182-201):
 * RCCL communicator over xGMI and ONE gather of every rank's sample store.    */
/* Diagnostic._computeVariogram (sampleDiagnosis.py:189-194) for every lag: x = [K][m][n]
 * (K columns, m half-chains of n samples, host memory), out = [K][n] with
 * out[k][t] = sum_j sum_{i>=t} (x[k][j][i] - x[k][j][i-t])^2 / (m (n - t)), the
 * reference's summation order; runs on `device`; n <= 8192.                          */
int nmc_variogram(int device, const double* x, int K, int m, int n, double* out);

int nmc_comm_unique_id(unsigned char* out /* 128 bytes */);
int nmc_comm_init(void** comm, const unsigned char* id, int nranks, int rank, int device);
int nmc_comm_destroy(void* comm);
/* Rank count and this rank's id of a communicator (ncclCommCount/UserRank). */
int nmc_comm_size(void* comm, int* nranks, int* rank);
/* root receives [rank][row][col][C_local] (all ranks must have equal C_local) in
 * host_out, which must hold host_capacity >= nranks * rows * cols * C_local doubles
 * (ignored on the other ranks, which may pass NULL).                            */
int nmc_gather_samples(nmc_ctx* ctx, void* comm, int root, double* host_out,
                       int64_t host_capacity);

/* Verification hooks (tests only): device numerics on caller inputs.
 *   prior logpdf of family fam with params[8] at xs[n]   (scipy .logpdf)
 *   gammainccinv(a[i], q[i]) with lga[i] = gammaln(a[i]) (scipy.special)
 *   per counter ctr5[i] = (iter, group, param, purpose, chain): out4[i] =
 *   {Box-Muller normal, uniform a, uniform b, Gamma(gamma_shape) draw}.       */
int nmc_debug_prior_logpdf(int fam, const double* params8, const double* xs, int n,
                           double* out);
int nmc_debug_igamci(const double* a, const double* q, const double* lga, int n,
                     double* out);
int nmc_debug_rng(const uint32_t* ctr5, int n, uint32_t seed, double gamma_shape,
                  double* out4);
/* numpy.logaddexp(0, x[i]) as the likelihood kernels evaluate it (csrc/softplus.h): on the
 * host (on_device = 0, no GPU needed) or by a device kernel (on_device = 1); the two are
 * bit-identical by construction (IEEE add / mul / fma / div, rint, ldexp only).          */
int nmc_debug_softplus(const double* x, int n, double* out, int on_device);
/* Diagnostic build only (make stamps -> libnestmc_stamps.so): shader-clock phase
 * stamps of the step kernel, [2 blocks][2 waves][8 iterations][16 slots]; n > 0
 * arms (zeroes) the buffer, out != NULL copies it back.  Error in the shipped lib. */
int nmc_debug_stamps(nmc_ctx* ctx, int n, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* NESTMC_H */
