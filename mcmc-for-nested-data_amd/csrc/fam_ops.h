// fam_ops.h -- the family-templated launches, instantiated once per family TU
// (fam_linreg.hip, fam_gauss_mean.hip, fam_logistic.hip).
#pragma once
#include "ctx.h"

// Iterations [i0, i1) of the step kernel (one launch).
template <class Fam>
static int nmc_launch_run(nmc_ctx* x, const Fam& fam, int i0, int i1, int flags) {
  Dev& d = x->d;
  const size_t lds = run_lds_bytes(x);
  std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
  if (x->ktiming) {
    if (int rc = pop_event_pair(x, x->kev, x->kev_used, &ev)) return rc;
    if (x->kev_iters.size() < x->kev_used) x->kev_iters.resize(x->kev_used);
    x->kev_iters[x->kev_used - 1] = i1 - i0;
    HIPCHK(hipEventRecord(ev->first, x->stream));
  }
  const dim3 grid(d.RB * d.G * d.S), block(64 * d.W);
  switch (run_mode(x)) {
    case NMC_MODE_NOPOOL:
      if (d.S > 1) {   // row split: resident batches of chain blocks
        for (int cb0 = 0; cb0 < d.RB; cb0 += x->split_batch) {
          Dev db = d;
          db.cb0 = cb0;
          const int nb = std::min(x->split_batch, d.RB - cb0);
          hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_NOPOOL>), dim3(nb * d.G * d.S), block, lds,
                             x->stream, db, fam, d.obs, i0, i1, flags);
        }
        break;
      }
      hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_NOPOOL>), grid, block, lds, x->stream, d, fam,
                         d.obs, i0, i1, flags);
      break;
    case NMC_MODE_LAUNCH:
      hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_LAUNCH>), grid, block, lds, x->stream, d, fam,
                         d.obs, i0, i1, flags);
      break;
    case NMC_MODE_SYNC:
      hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_SYNC>), grid, block, lds, x->stream, d, fam,
                         d.obs, i0, i1, flags);
      break;
    case NMC_MODE_PAIR:
      hipLaunchKernelGGL((nmc_k_pair<Fam>), grid, block, lds, x->stream, d, fam, d.obs, i0, i1,
                         flags);
      break;
    case NMC_MODE_SYNC_REG:
      hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_SYNC_REG>), grid, block, lds, x->stream, d, fam,
                         d.obs, i0, i1, flags);
      break;
    default:
      hipLaunchKernelGGL((nmc_k_run<Fam, NMC_MODE_SYNC_LDS>), grid, block, lds, x->stream, d, fam,
                         d.obs, i0, i1, flags);
  }
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev->second, x->stream));
  return 0;
}

// Partial pooling: may every workgroup of the grid be resident at once?  (The
// persistent kernel's chain-block waits need it.)  One block of margin per CU where
// the occupancy query can over-report (MI355X_MICROARCH.md, residency).
template <class Fam>
static bool nmc_can_persist(nmc_ctx* x) {
  if (const char* e = getenv("NMC_PERSIST")) return atoi(e) != 0;
  int nb = 0;
  const void* k = x->d.pair   ? (const void*)nmc_k_pair<Fam>
                  : !x->d.hlds ? (const void*)nmc_k_run<Fam, NMC_MODE_SYNC>
                  : x->d.hreg  ? (const void*)nmc_k_run<Fam, NMC_MODE_SYNC_REG>
                               : (const void*)nmc_k_run<Fam, NMC_MODE_SYNC_LDS>;
  const size_t lds = x->d.pair ? pair_lds_bytes(x) : lds_bytes_for(x, x->d.hlds, x->d.rows_lds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W, lds) !=
      hipSuccess)
    return false;
  // The API can answer one block per CU too many where SGPRs bind (MI355X_MICROARCH.md,
  // residency: min(API, floor(800 / (ceil(sgpr / 16) * 16 + 16))) waves per SIMD); the
  // step kernels use <= 112 SGPRs -> 6 waves per SIMD, i.e. 24 / W blocks of W = 4k waves.
  // Other block sizes keep one block of margin.
  const int W = x->d.W;
  const int safe = W % 4 == 0 ? std::min(nb, 24 / W) : (nb > 1 ? nb - 1 : nb);
  return (int64_t)x->d.RB * x->d.G <= (int64_t)safe * x->ncu;
}

template <class Fam>
static int nmc_fam_call(nmc_ctx* x, const Fam& fam, NmcCall& c) {
  switch (c.op) {
    case NMC_OP_RUN:
      return nmc_launch_run(x, fam, c.i0, c.i1, c.flags);
    case NMC_OP_CAN_PERSIST:
      c.result = nmc_can_persist<Fam>(x) ? 1 : 0;
      return 0;
    case NMC_OP_CAPACITY: {   // resident none/complete step-kernel workgroups (safe count)
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, nmc_k_run<Fam, NMC_MODE_NOPOOL>,
                                                       64 * x->d.W, run_lds_bytes(x)) != hipSuccess)
        return nmc_fail(-2, "occupancy query failed");
      const int W = x->d.W;
      const int safe = W % 4 == 0 ? std::min(nb, 24 / W) : (nb > 1 ? nb - 1 : nb);
      c.result = safe * x->ncu;
      return 0;
    }
    case NMC_OP_GROUP_LL: {
      const size_t lds = (size_t)x->d.W * 64 * Fam::NACC * sizeof(double);
      hipLaunchKernelGGL(nmc_k_group_ll<Fam>, dim3(x->d.CB * x->G), dim3(64 * x->d.W), lds,
                         x->stream, x->d, fam, x->d.obs, c.in, c.out);
      HIPCHK(hipGetLastError());
      return 0;
    }
    case NMC_OP_OBS_LL_ROWS: {
      const int n = c.i1 - c.i0;
      if (n <= 0 || x->n_obs == 0) return 0;
      const dim3 grid((unsigned)((x->n_obs + 255) / 256), (unsigned)x->C, (unsigned)n);
      hipLaunchKernelGGL(nmc_k_obs_ll_rows<Fam>, grid, dim3(256), 0, x->stream, x->d, fam,
                         (const int*)x->gidx, x->n_obs,
                         x->pooling == NMC_POOL_PARTIAL ? 2 : 0, c.i0, n, c.out);
      HIPCHK(hipGetLastError());
      return 0;
    }
    case NMC_OP_OBS_LL:
      hipLaunchKernelGGL(nmc_k_obs_ll<Fam>, dim3(x->d.CB * x->G), dim3(64), 0, x->stream, x->d,
                         fam, c.in, c.out, x->n_obs);
      HIPCHK(hipGetLastError());
      return 0;
  }
  return nmc_fail(-1, "unknown family op");
}

// nmc_call_<family>: (n_fields) -> the concrete functor type, then the op.
#define NMC_DEFINE_FAMILY_CALL(NAME, MAKE)                                  \
  int NAME(nmc_ctx* x, NmcCall& c) {                                        \
    switch (x->nf) {                                                        \
      case 1: return nmc_fam_call(x, MAKE<1>(x->llc), c);                   \
      case 2: return nmc_fam_call(x, MAKE<2>(x->llc), c);                   \
      case 3: return nmc_fam_call(x, MAKE<3>(x->llc), c);                   \
      case 4: return nmc_fam_call(x, MAKE<4>(x->llc), c);                   \
      case 5: return nmc_fam_call(x, MAKE<5>(x->llc), c);                   \
      case 6: return nmc_fam_call(x, MAKE<6>(x->llc), c);                   \
      case 7: return nmc_fam_call(x, MAKE<7>(x->llc), c);                   \
      case 8: return nmc_fam_call(x, MAKE<8>(x->llc), c);                   \
      case 9: return nmc_fam_call(x, MAKE<9>(x->llc), c);                   \
    }                                                                       \
    return nmc_fail(-1, "n_fields must be 1..9");                           \
  }
