// sweep_ops.h -- the nmc_k_sweep launches (sweep.h), instantiated once per family in their
// own translation units (sweep_*.hip).  Those are built with -mllvm -disable-machine-licm
// (Makefile): left alone, the backend hoists the polynomial constants of the variate draws
// and priors out of the persistent loop into registers for the whole launch and then spills
// them -- 20-70 VGPRs to scratch at the kernel's 168-VGPR budget (three waves per SIMD).
#pragma once
#include "ctx.h"
#include "fam_make.h"

// The sweep kernel instance of a mode (for launches and occupancy queries): SYNC_OWN only
// (partial pooling over G > 128 groups, nestmc.hip choose_geometry)
template <class Fam>
static const void* nmc_sweep_kernel(int mode) {
  return mode == NMC_MODE_SYNC_OWN ? (const void*)nmc_k_sweep<Fam, NMC_MODE_SYNC_OWN> : nullptr;
}

// (four waves: an eight-wave form with two streams per wave needs <= 88 VGPRs to sit beside
//  two likelihood workgroups and spilled at that budget)
template <class Fam>
static const void* nmc_sweep_gibbs_kernel(int) {
  return (const void*)nmc_k_sweep_gibbs<Fam, 4>;
}

// NMC_OP_RUN / NMC_OP_CAN_PERSIST / NMC_OP_CAPACITY of a context whose loop runs nmc_k_sweep.
template <class Fam>
static int nmc_sweep_call_t(nmc_ctx* x, const Fam& fam, NmcCall& c) {
  switch (c.op) {
    case NMC_OP_RUN: {
      const int i0 = c.i0, i1 = c.i1;
      return nmc_run_launches(x, i0, i1, [&](int mode, const Dev& d, dim3 grid, dim3 block,
                                             size_t lds) {
        nmc_sweep_args<Fam> a{d, fam, i0, i1};
        void* args[] = {&a};
        if (mode == NMC_MODE_SYNC_OWN && d.gsep) {
          // the Gibbs workgroups' kernel on the second stream, forked after the work before
          // this launch and joined before the work after it; both kernels resident together
          // (NMC_OP_CAN_PERSIST), each waiting on counters the other advances -- and, when
          // the two do not run at the same time after all, the likelihood workgroups take
          // the launch's Gibbs tasks over (Dev.grole, this launch's epoch gep)
          if (++x->gepoch == 0) ++x->gepoch;   // (0: a role word never written)
          a.d.gep = x->gepoch;
          const unsigned nb = grid.x / (unsigned)d.G;   // chain blocks of this launch
          auto gibbs = [&](hipStream_t s) {
            hipLaunchKernel(nmc_sweep_gibbs_kernel<Fam>(d.gwaves), dim3(nb * d.P),
                            dim3(64 * d.gwaves), args, sweep_gibbs_lds_bytes(x), s);
          };
          if (x->gserial) {   // (tests: both kernels on one stream, serialized; 1: the Gibbs
                              //  kernel first, 2: after the likelihood kernel)
            if (x->gserial == 1) gibbs(x->stream);
            hipLaunchKernel(nmc_sweep_kernel<Fam>(mode), grid, block, args, lds, x->stream);
            if (x->gserial == 2) gibbs(x->stream);
            return;
          }
          hipEventRecord(x->gev[0], x->stream);
          hipStreamWaitEvent(x->gstream, x->gev[0], 0);
          gibbs(x->gstream);
          hipLaunchKernel(nmc_sweep_kernel<Fam>(mode), grid, block, args, lds, x->stream);
          hipEventRecord(x->gev[1], x->gstream);
          hipStreamWaitEvent(x->stream, x->gev[1], 0);
          return;
        }
        // (SYNC_OWN: the Gibbs workgroups after the likelihood ones)
        const dim3 gr(mode == NMC_MODE_SYNC_OWN ? (unsigned)sweep_grid(x) : grid.x);
        hipLaunchKernel(nmc_sweep_kernel<Fam>(mode), gr, block, args, lds, x->stream);
      });
    }
    case NMC_OP_CAN_PERSIST: {   // may every workgroup of the grid be resident at once?
      if (const char* e = getenv("NMC_PERSIST")) {
        c.result = atoi(e) != 0;
        return 0;
      }
      int nb = 0;
      c.result = 0;
      const void* k = nmc_sweep_kernel<Fam>(nmc_persist_mode(x));
      if (k && hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W,
                                                            nmc_persist_lds(x)) == hipSuccess)
        c.result = sweep_grid(x) <= (int64_t)nmc_safe_blocks(x, nb) * x->ncu;
      if (x->d.gsep && k) {
        // the largest batch of chain blocks whose likelihood workgroups are co-resident and
        // leave, on the CUs holding the most of them, the LDS and the wave slots (<= 168
        // VGPRs: three waves per SIMD) for one four-wave Gibbs workgroup; the launches run
        // the chain blocks in such batches (nmc_run_launches)
        int ng = 0;
        const void* gk = nmc_sweep_gibbs_kernel<Fam>(x->d.gwaves);
        const int gw = x->d.gwaves;
        hipFuncAttributes am{}, ag{};
        const bool gok = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                             &ng, gk, 64 * gw, sweep_gibbs_lds_bytes(x)) == hipSuccess &&
                         ng >= 1 && hipFuncGetAttributes(&am, k) == hipSuccess &&
                         hipFuncGetAttributes(&ag, gk) == hipSuccess;
        // VGPRs per SIMD (512 per lane, allocated in 8s) and wave slots (8 per SIMD)
        auto vg = [](int r) { return (r + 7) / 8 * 8; };
        const int64_t cap = (int64_t)nmc_safe_blocks(x, nb) * x->ncu;
        int best = 0;
        for (int b = 1; gok && b <= x->d.RB; ++b) {
          const int64_t wg = (int64_t)b * x->d.G;
          const int64_t per = (wg + x->ncu - 1) / x->ncu;
          const int64_t mw = (per * x->d.W + 3) / 4, gws = (gw + 3) / 4;   // waves per SIMD
          if (wg <= cap &&
              per * (int64_t)nmc_persist_lds(x) + sweep_gibbs_lds_bytes(x) <= (size_t)160 * 1024 &&
              mw * vg(am.numRegs) + gws * vg(ag.numRegs) <= 512 && mw + gws <= 8)
            best = b;
        }
        x->sweep_batch = best;
        c.result = best >= 1;
      }
      return 0;
    }
    case NMC_OP_CAPACITY: {
      int nb = 0;
      const void* k = nmc_sweep_kernel<Fam>(run_mode(x));
      if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 64 * x->d.W,
                                                             run_lds_bytes(x)) != hipSuccess)
        return nmc_fail(-2, "occupancy query failed");
      c.result = nmc_safe_blocks(x, nb) * x->ncu;
      return 0;
    }
  }
  return nmc_fail(-1, "sweep: unknown op");
}

#ifdef NMC_ONLY_NF
#define NMC_DEFINE_SWEEP_CALL(NAME, MAKE)                                              \
  int NAME(nmc_ctx* x, NmcCall& c) {                                                   \
    if (x->nf == NMC_ONLY_NF) return nmc_sweep_call_t(x, MAKE<NMC_ONLY_NF>(x->llc), c); \
    return nmc_fail(-1, "NMC_ONLY_NF build");                                          \
  }
#else
#define NMC_DEFINE_SWEEP_CALL(NAME, MAKE)                                   \
  int NAME(nmc_ctx* x, NmcCall& c) {                                        \
    switch (x->nf) {                                                        \
      case 1: return nmc_sweep_call_t(x, MAKE<1>(x->llc), c);               \
      case 2: return nmc_sweep_call_t(x, MAKE<2>(x->llc), c);               \
      case 3: return nmc_sweep_call_t(x, MAKE<3>(x->llc), c);               \
      case 4: return nmc_sweep_call_t(x, MAKE<4>(x->llc), c);               \
      case 5: return nmc_sweep_call_t(x, MAKE<5>(x->llc), c);               \
      case 6: return nmc_sweep_call_t(x, MAKE<6>(x->llc), c);               \
      case 7: return nmc_sweep_call_t(x, MAKE<7>(x->llc), c);               \
      case 8: return nmc_sweep_call_t(x, MAKE<8>(x->llc), c);               \
      case 9: return nmc_sweep_call_t(x, MAKE<9>(x->llc), c);               \
    }                                                                       \
    return nmc_fail(-1, "n_fields must be 1..9");                           \
  }
#endif
