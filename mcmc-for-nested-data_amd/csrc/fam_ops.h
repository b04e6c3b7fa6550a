// fam_ops.h -- the family-templated launches, instantiated once per family TU
// (fam_linreg.hip, fam_gauss_mean.hip, fam_logistic.hip).
#pragma once
#include "ctx.h"

// Iterations [i0, i1) of the step kernel (one launch, or one per resident chain-block
// batch under the row split).
// The step kernel instance of (mode, rows in LDS) -- for launches and occupancy queries.
template <class Fam, bool RL>
static const void* nmc_run_kernel_rl(int mode) {
  switch (mode) {
    case NMC_MODE_NOPOOL: return (const void*)nmc_k_run<Fam, NMC_MODE_NOPOOL, RL>;
    case NMC_MODE_LAUNCH: return (const void*)nmc_k_run<Fam, NMC_MODE_LAUNCH, RL>;
    case NMC_MODE_SYNC: return (const void*)nmc_k_run<Fam, NMC_MODE_SYNC, RL>;
    case NMC_MODE_SYNC_REG: return (const void*)nmc_k_run<Fam, NMC_MODE_SYNC_REG, RL>;
    case NMC_MODE_HALF:   // (rows in LDS, row pairs in every block: the host's condition)
      if constexpr (RL && nmc_paired_rows_ok<Fam>())
        return (const void*)nmc_k_run<Fam, NMC_MODE_HALF, true>;
      return nullptr;
    default: return (const void*)nmc_k_run<Fam, NMC_MODE_SYNC_LDS, RL>;
  }
}
template <class Fam>
static const void* nmc_run_kernel(const nmc_ctx* x, int mode) {
  return x->d.rows_lds ? nmc_run_kernel_rl<Fam, true>(mode) : nmc_run_kernel_rl<Fam, false>(mode);
}
// The resident instance (Dev.rcmd: one launch across nmc_run calls) of a mode: rows in LDS,
// families of <= 3 fields, the modes without a per-launch Gibbs pipeline state beyond the
// register hand-off (nullptr: none)
template <class Fam>
static const void* nmc_run_kernel_res(int mode) {
  if constexpr (Fam::NFIELDS <= 3) {
    switch (mode) {
      case NMC_MODE_NOPOOL: return (const void*)nmc_k_run<Fam, NMC_MODE_NOPOOL, true, true>;
      case NMC_MODE_SYNC_REG: return (const void*)nmc_k_run<Fam, NMC_MODE_SYNC_REG, true, true>;
      case NMC_MODE_HALF:
        if constexpr (nmc_paired_rows_ok<Fam>())
          return (const void*)nmc_k_run<Fam, NMC_MODE_HALF, true, true>;
        return nullptr;
    }
  }
  return nullptr;
}

template <class Fam>
static int nmc_launch_run(nmc_ctx* x, const Fam& fam, int i0, int i1, int flags, bool res) {
  return nmc_run_launches(x, i0, i1, [&](int mode, const Dev& d, dim3 grid, dim3 block,
                                         size_t lds) {
    Dev dd = d;
    const double* obs = d.obs;
    void* args[] = {&dd, (void*)&fam, (void*)&obs, &i0, &i1, &flags};
    hipLaunchKernel(res ? nmc_run_kernel_res<Fam>(mode) : nmc_run_kernel<Fam>(x, mode), grid,
                    block, args, lds, x->stream);
  });
}

// Partial pooling: may every workgroup of the grid be resident at once?  (The
// persistent kernel's chain-block waits need it.)
template <class Fam>
static bool nmc_can_persist(nmc_ctx* x) {
  if (const char* e = getenv("NMC_PERSIST")) return atoi(e) != 0;
  int nb = 0;
  const void* k = nmc_run_kernel<Fam>(x, nmc_persist_mode(x));
  if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W,
                                                         nmc_persist_lds(x)) != hipSuccess)
    return false;
  return (int64_t)x->d.RB * x->d.G * x->d.S <= (int64_t)nmc_safe_blocks(x, nb) * x->ncu;
}

template <class Fam>
static int nmc_fam_call(nmc_ctx* x, const Fam& fam, NmcCall& c) {
  switch (c.op) {
    case NMC_OP_RUN:
      return nmc_launch_run(x, fam, c.i0, c.i1, c.flags, c.res != 0);
    case NMC_OP_CAN_PERSIST:
      c.result = nmc_can_persist<Fam>(x) ? 1 : 0;
      return 0;
    case NMC_OP_RES_OK: {   // a resident instance of the run mode, its whole grid co-resident
      const void* k = x->d.rows_lds ? nmc_run_kernel_res<Fam>(run_mode(x)) : nullptr;
      int nb = 0;
      c.result = 0;
      if (k && hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W,
                                                            run_lds_bytes(x)) == hipSuccess)
        c.result = (int64_t)x->d.RB * x->d.G * x->d.S <= (int64_t)nmc_safe_blocks(x, nb) * x->ncu;
      hipFuncAttributes fa{};
      c.result2 = k && hipFuncGetAttributes(&fa, k) == hipSuccess ? fa.numRegs : 0;   // VGPRs
      return 0;
    }
    case NMC_OP_CAPACITY: {   // resident step-kernel workgroups of the run mode (safe count)
      int nb = 0;
      const void* k = nmc_run_kernel<Fam>(x, run_mode(x));
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W, run_lds_bytes(x)) !=
          hipSuccess)
        return nmc_fail(-2, "occupancy query failed");
      c.result = nmc_safe_blocks(x, nb) * x->ncu;
      return 0;
    }
    case NMC_OP_GROUP_LL: {   // c.aux: [S][NACC][G][C] member partials
      const Dev& d = x->d;
      const size_t lds = nmc_group_ll_lds(x);
      const void* k = d.rows_lds ? (const void*)nmc_k_group_part<Fam, true>
                                 : (const void*)nmc_k_group_part<Fam, false>;
      Dev dd = d;
      const double* obs = d.obs;
      const double* in = c.in;
      double* aux = c.aux;
      void* a1[] = {&dd, (void*)&fam, (void*)&obs, (void*)&in, (void*)&aux};
      HIPCHK(hipLaunchKernel(k, dim3(d.CB * d.G * d.S), dim3(64 * std::min(d.W, 8)), a1, lds,
                             x->stream));
      const size_t n = (size_t)d.G * d.C;
      hipLaunchKernelGGL(nmc_k_group_fin<Fam>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                         x->stream, d, fam, c.in, (const double*)c.aux, c.out);
      HIPCHK(hipGetLastError());
      return 0;
    }
    case NMC_OP_OBS_LL_ROWS: {
      const int n = c.i1 - c.i0;
      if (n <= 0 || x->n_obs == 0) return 0;
      const int nc = c.nc > 0 ? c.nc : x->C;
      const dim3 grid((unsigned)((x->n_obs + 255) / 256), (unsigned)nc, (unsigned)n);
      hipLaunchKernelGGL(nmc_k_obs_ll_rows<Fam>, grid, dim3(256), 0, x->stream, x->d, fam,
                         (const int*)x->gidx, x->n_obs,
                         x->pooling == NMC_POOL_PARTIAL ? 2 : 0, c.i0, n, c.c0, c.out);
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
// (NMC_ONLY_NF=k, register-budget experiments only: instantiate one row width)
#ifdef NMC_ONLY_NF
#define NMC_DEFINE_FAMILY_CALL(NAME, MAKE)                                  \
  int NAME(nmc_ctx* x, NmcCall& c) {                                        \
    if (x->nf == NMC_ONLY_NF) return nmc_fam_call(x, MAKE<NMC_ONLY_NF>(x->llc), c); \
    return nmc_fail(-1, "NMC_ONLY_NF build");                               \
  }
#else
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
#endif
