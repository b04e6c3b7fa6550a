// pair.h -- the two-parameter step kernel (P == 2, partial pooling, persistent, G <= 64).
//
// An iteration of the reference is two Metropolis steps (StepMethod.step :594-613):
// step 0 proposes theta_0' = theta_0 + s_0 z_0 against theta_1, step 1 proposes
// theta_1' = theta_1 + s_1 z_1 against whatever step 0 decided.  Both proposals are
// known when the iteration starts (the scales only change at their own step, the
// variates are pre-drawn), so ONE pass over the group's rows evaluates the three
// likelihoods the iteration can need:
//     A = LL(theta_0', theta_1)     step 0
//     B = LL(theta_0,  theta_1')    step 1 if step 0 rejected
//     C = LL(theta_0', theta_1')    step 1 if step 0 accepted
// and the control wave then decides step 0 (with A) and step 1 (with B or C, per chain)
// back to back.  Every sum is the one nmc_k_run forms for that step -- same tiles
// (nmc_tiles), same per-tile accumulation order, same fixed slot combine -- so the
// results are bit-identical to the one-step-per-pass kernel; the rows are streamed
// once per iteration instead of twice and the serial decision/barrier section is paid
// once per iteration.  The step-1 variant that is not taken is the only extra work
// (three likelihoods per iteration instead of two; the pass is VALU-bound).
//
// Waves: 0 control (decisions, state, variate DMA; takes tiles), 1 and 2 the Gibbs
// waves of parameters 0 and 1 (publishing the workgroup's decided value of their
// parameter, then HyperParameter.update :463-498 from a register copy of the chain
// block's published values, nmc_hyper_compute_reg), the rest likelihood tiles.  Gibbs task (t-1, q) is published at the end of iteration t-1
// and needed by the decision of step (t, q): the Gibbs wave of q polls, fetches and
// updates it during iteration t's pass and evaluates step (t, q)'s priors.
#pragma once
#include "kernels.h"

// LDS carve of the pair kernel, in columns of 64 doubles (the host computes the same).
struct nmc_pair_layout {
  int th;      // [2]            current values
  int part;    // [3][NACC][NSLOT]  tile partials of A, B, C (unused slots: -0.0)
  int st;      // [5][2]         scale, log prior, n acc, n rej, total acc
  int hyp;     // [6][2]         hyper state (NMC_HY_*)
  int zl;      // [2 parity][2 steps][2]  {z, log u} of the steps of iterations t, t+1
  int cw;      // [16]           control-wave / Gibbs-wave values across the barriers
  int flag;    // [1]            verdict words, tile counters
  int rows;    // [nrows][NF]    the group's rows (+1 column of prefetch pad)
  int total;
};
__host__ __device__ inline nmc_pair_layout nmc_pair_lds(int nacc, int row_doubles) {
  nmc_pair_layout L;
  L.th = 0;
  L.part = L.th + 2;
  L.st = L.part + 3 * nacc * NMC_NSLOT;
  L.hyp = L.st + 5 * 2;
  L.zl = L.hyp + 6 * 2;
  L.cw = L.zl + 8;
  L.flag = L.cw + 16;
  L.rows = L.flag + 1;
  L.total = L.rows + (row_doubles + 63) / 64 + 1;
  return L;
}
// cw columns: priors from the Gibbs waves, both outcomes of each step's counters
enum { NMC_PW_LPC0 = 0, NMC_PW_LPP0, NMC_PW_LPC1, NMC_PW_LPP1, NMC_PW_CNT = 4 };  // + 5 per step

// The regression row loop (FamLinreg<2>, rows {x, y}) for the three parameter sets at
// once, with nmc_rows_lds_linreg2's blocks and residual e = fma(x, b1, b0 - y) per set.
// For P == 2 sets A and C always share their intercept (b0 = theta_0' with an
// intercept, 0 without), so b0 - y is formed once for both: per row two subtractions,
// three fmas and three squares instead of three of each.  Row j of a block: x in
// v[b+4j:+1], y in v[b+4j+2:+3]; temporaries U_j = v[160+2j] (set B), T_j = v[176+2j]
// (set A); set C's residual ends in y's register.  nb: even number of 8-row blocks.
#define NMC_PX(b, j) "v[" #b "+4*" #j ":" #b "+4*" #j "+1]"
#define NMC_PY(b, j) "v[" #b "+4*" #j "+2:" #b "+4*" #j "+3]"
#define NMC_PU(j) "v[160+2*" #j ":160+2*" #j "+1]"
#define NMC_PT(j) "v[176+2*" #j ":176+2*" #j "+1]"
#define NMC_PSUB(b, j)                                                       \
  "v_add_f64 " NMC_PU(j) ", %[b0b], -" NMC_PY(b, j) "\n"                     \
  "v_add_f64 " NMC_PY(b, j) ", %[b0a], -" NMC_PY(b, j) "\n"
#define NMC_PFMA(b, j)                                                       \
  "v_fma_f64 " NMC_PU(j) ", " NMC_PX(b, j) ", %[b1b], " NMC_PU(j) "\n"        \
  "v_fma_f64 " NMC_PT(j) ", " NMC_PX(b, j) ", %[b1a], " NMC_PY(b, j) "\n"     \
  "v_fma_f64 " NMC_PY(b, j) ", " NMC_PX(b, j) ", %[b1c], " NMC_PY(b, j) "\n"
#define NMC_PSQ(b, j, k)                                                          \
  "v_fma_f64 %[a" #k "], " NMC_PT(j) ", " NMC_PT(j) ", %[a" #k "]\n"              \
  "v_fma_f64 %[c" #k "], " NMC_PU(j) ", " NMC_PU(j) ", %[c" #k "]\n"              \
  "v_fma_f64 %[e" #k "], " NMC_PY(b, j) ", " NMC_PY(b, j) ", %[e" #k "]\n"
#define NMC_PB8(b)                                                                        \
  NMC_PSUB(b, 0) NMC_PSUB(b, 1) NMC_PSUB(b, 2) NMC_PSUB(b, 3) NMC_PSUB(b, 4) NMC_PSUB(b, 5) \
  NMC_PSUB(b, 6) NMC_PSUB(b, 7) NMC_PFMA(b, 0) NMC_PFMA(b, 1) NMC_PFMA(b, 2) NMC_PFMA(b, 3) \
  NMC_PFMA(b, 4) NMC_PFMA(b, 5) NMC_PFMA(b, 6) NMC_PFMA(b, 7) NMC_PSQ(b, 0, 0)              \
  NMC_PSQ(b, 1, 1) NMC_PSQ(b, 2, 2) NMC_PSQ(b, 3, 3) NMC_PSQ(b, 4, 0) NMC_PSQ(b, 5, 1)      \
  NMC_PSQ(b, 6, 2) NMC_PSQ(b, 7, 3)
__device__ __forceinline__ void nmc_rows_lds_linreg2x3(const double* p, int nb, double b0a,
                                                       double b0b, double b1a, double b1b,
                                                       double b1c, double (&a)[3][4]) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nb;
  asm volatile(
      NMC_L8(192, 0)
      "L_nmc_prows_%=:\n"
      NMC_L8(224, 128)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_PB8(192)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_nmc_plast_%=\n"
      NMC_L8(192, 0)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_PB8(224)
      "s_branch L_nmc_prows_%=\n"
      "L_nmc_plast_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_PB8(224)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [a0] "+v"(a[0][0]), [a1] "+v"(a[0][1]),
        [a2] "+v"(a[0][2]), [a3] "+v"(a[0][3]), [c0] "+v"(a[1][0]), [c1] "+v"(a[1][1]),
        [c2] "+v"(a[1][2]), [c3] "+v"(a[1][3]), [e0] "+v"(a[2][0]), [e1] "+v"(a[2][1]),
        [e2] "+v"(a[2][2]), [e3] "+v"(a[2][3])
      : [b0a] "v"(b0a), [b0b] "v"(b0b), [b1a] "v"(b1a), [b1b] "v"(b1b), [b1c] "v"(b1c)
      : "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170",
        "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181",
        "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192",
        "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203",
        "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214",
        "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225",
        "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236",
        "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247",
        "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255", "scc", "memory");
}

// nmc_ll_rows_lds for three parameter sets over the same rows: every block is read once
// and accumulated per set exactly as nmc_ll_rows_lds would (same blocks, same accumulator
// per row, same tail), so each set's sum is bit-identical to the single-set loop.
template <class Fam>
__device__ __forceinline__ void nmc_ll_rows_lds3(const Fam& fam, const typename Fam::Reg (&reg)[3],
                                                 const double* __restrict__ p, int n,
                                                 double (&acc)[3][Fam::NACC]) {
  constexpr int NF = Fam::NFIELDS;
  constexpr int BD = NF <= 2 ? NMC_LDS_ROW_DOUBLES : 8;
  constexpr int R = (BD / NF) > 0 ? (BD / NF) : 1;
  double a[3][4][Fam::NACC];
#pragma unroll
  for (int v = 0; v < 3; ++v)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < Fam::NACC; ++k) a[v][s][k] = 0.0;
  const int nb2 = (n / R) & ~1;
  if constexpr (Fam::ASM_ROWS) {
    static_assert(R == 8 && NF == 2, "the asm row loop is the 8-row {x, y} block");
    if (nb2 > 0) {
      double aa[3][4];
#pragma unroll
      for (int v = 0; v < 3; ++v)
#pragma unroll
        for (int s = 0; s < 4; ++s) aa[v][s] = 0.0;
      // (reg[2].b0 == reg[0].b0: see nmc_rows_lds_linreg2x3)
      nmc_rows_lds_linreg2x3(p, nb2, reg[0].b0, reg[1].b0, reg[0].b[0], reg[1].b[0], reg[2].b[0],
                             aa);
#pragma unroll
      for (int v = 0; v < 3; ++v)
#pragma unroll
        for (int s = 0; s < 4; ++s) a[v][s][0] = aa[v][s];
    }
  } else {
    for (int b = 0; b < nb2; ++b) {
      double A[R * NF];
#pragma unroll
      for (int j = 0; j < R * NF; ++j) A[j] = p[(size_t)b * (R * NF) + j];
#pragma unroll
      for (int v = 0; v < 3; ++v) fam.template accumN<R>(reg[v], A, a[v]);
    }
  }
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
    for (int v = 0; v < 3; ++v)
#pragma unroll
      for (int i = 0; i < TB; ++i)
        if (r0 + i < n) fam.accum(reg[v], tv + i * NF, a[v][0]);
  }
#pragma unroll
  for (int v = 0; v < 3; ++v)
#pragma unroll
    for (int k = 0; k < Fam::NACC; ++k)
      acc[v][k] = (a[v][0][k] + a[v][1][k]) + (a[v][2][k] + a[v][3][k]);
}

// The Metropolis decision of Parameter.step (:334-367), branch order exact.
__device__ __forceinline__ bool nmc_mh_accept(double lpc, double ll, double lpp, double llp,
                                              double lu) {
  const double postp = lpp + llp;
  const double post = lpc + ll;
  const double diff = postp - post;
  if (!isfinite(post) && isfinite(postp)) return true;   // :347-352
  if (!isfinite(llp)) return false;                     // :354-356
  if (!isfinite(diff)) return false;                    // :358-360
  return lu < diff;                                     // :362-364
}

template <class Fam>
__global__ void __launch_bounds__(512)
nmc_k_pair(Dev d, Fam fam, const double* __restrict__ obs, int i0, int i1, int flags) {
  constexpr int NA = Fam::NACC;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = d.G, C = d.C;
  const int W = blockDim.x >> 6;   // (diagnostic stamps)
  (void)W;
  const int b = blockIdx.x;
  const int g = b % G, cb = b / G;
  const int c = cb * 64 + lane;
  const bool live = c < C;
  const int cc = live ? c : C - 1;
  const int row_doubles = d.nmax * Fam::NFIELDS;
  const nmc_pair_layout L = nmc_pair_lds(NA, row_doubles);
  double* th = lds + L.th * 64 + lane;     // th[q * 64]
  double* st = lds + L.st * 64 + lane;     // st[(k * 2 + q) * 64]
  double* hy = lds + L.hyp * 64 + lane;    // hy[(k * 2 + q) * 64]
  double* cwv = lds + L.cw * 64 + lane;
  unsigned* tcnt = (unsigned*)(lds + L.flag * 64 + 4);   // tile counters by iteration parity
  const int64_t r0 = d.off[g];
  const int nrow = (int)(d.off[g + 1] - r0);
  const nmc_tiling TI = nmc_tiles(nrow, d.tile);
  const int nt = TI.nt;
  const size_t GC = (size_t)G * C;
  const size_t gc = (size_t)g * C + cc;
  const bool ctl = w == 0;
  const bool gw = w == 1 || w == 2;
  const int gq = w - 1;   // the Gibbs wave's parameter
  if ((ctl || gw) && !(d.noprio & 1)) __builtin_amdgcn_s_setprio(3);

  // ---- prologue: values, state, hyper-parameters after i0-1 -> LDS; rows -> LDS ----
  const double* vin = ((i0 - 1) & 1) ? d.vb1 : d.vb0;
  if (w < 2) {
    const int q = w;
    const size_t ip = (size_t)q * GC + gc;
    th[q * 64] = vin[ip];
    st[(NMC_ST_S * 2 + q) * 64] = d.scale[ip];
    st[(NMC_ST_LP * 2 + q) * 64] = d.lp[ip];
    st[(NMC_ST_NA * 2 + q) * 64] = (double)d.nacc[ip];
    st[(NMC_ST_NR * 2 + q) * 64] = (double)d.nrej[ip];
    st[(NMC_ST_TA * 2 + q) * 64] = (double)d.tacc[ip];
    const size_t ho = nmc_hslot(d, i0 - 1) + (size_t)q * C + cc;
    const double s2 = d.s2[ho];
    hy[(NMC_HY_MU * 2 + q) * 64] = d.mu[ho];
    hy[(NMC_HY_SD * 2 + q) * 64] = d.hsd[ho];
    hy[(NMC_HY_LSD * 2 + q) * 64] = d.hlsd[ho];
    hy[(NMC_HY_S2 * 2 + q) * 64] = s2;
    hy[(NMC_HY_SDM * 2 + q) * 64] = sqrt(s2 / G);
    hy[(NMC_HY_ISD * 2 + q) * 64] = 1.0 / d.hsd[ho];
  }
  const double gcst = fam.gconst((long)nrow);
  double* lrows = lds + L.rows * 64;
  {
    const double* grows = obs + r0 * Fam::NFIELDS;
    const int nd = nrow * Fam::NFIELDS;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
  }
  const size_t PGC = 2 * GC;
  auto zl_src = [&](int tn, int q) -> const double* {
    return d.vzl + ((size_t)(tn - d.vbase) * PGC + (size_t)q * GC + gc) * 2;
  };
  auto zl_slot = [&](int tn, int q) -> double* {   // {z, log u} of step (tn, q), lane-interleaved
    return lds + (L.zl + 2 * (2 * (tn & 1) + q)) * 64;
  };
  // One pass over the rows for iteration t: every wave that runs it takes row tiles
  // from the iteration's LDS counter until none is left, writing the tile partials of
  // A, B and C.
  auto pass = [&](int t) {
    const double v0 = th[0], v1 = th[64];
    const double p0 = v0 + (1.0 * st[(NMC_ST_S * 2 + 0) * 64]) * zl_slot(t, 0)[2 * lane];
    const double p1 = v1 + (1.0 * st[(NMC_ST_S * 2 + 1) * 64]) * zl_slot(t, 1)[2 * lane];
    double thp[Fam::MAXP];
#pragma unroll
    for (int q = 0; q < Fam::MAXP; ++q) thp[q] = 0.0;
    typename Fam::Reg reg[3];
    thp[0] = p0; thp[1] = v1; reg[0] = fam.prepare(thp);
    thp[0] = v0; thp[1] = p1; reg[1] = fam.prepare(thp);
    thp[0] = p0; thp[1] = p1; reg[2] = fam.prepare(thp);
    const int sp = t & 1;
    auto grab = [&]() -> unsigned {
      unsigned k = 0;
      if (lane == 0)
        k = __hip_atomic_fetch_add(tcnt + sp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return k;
    };
    int k = (int)__builtin_amdgcn_readlane(grab(), 0);
    while (k < nt) {
      const unsigned kn = grab();
      const int ra = TI.start(k);
      const int rn = TI.len(k);
      double acc[3][NA];
      nmc_ll_rows_lds3(fam, reg, lrows + (size_t)ra * Fam::NFIELDS, rn, acc);
#pragma unroll
      for (int v = 0; v < 3; ++v)
#pragma unroll
        for (int j = 0; j < NA; ++j) lds[(L.part + (v * NA + j) * NMC_NSLOT + k) * 64 + lane] = acc[v][j];
      k = (int)__builtin_amdgcn_readlane(kn, 0);
    }
  };
  if (ctl) {
    nmc_dma16(zl_src(i0, 0), zl_slot(i0, 0));
    nmc_dma16(zl_src(i0, 1), zl_slot(i0, 1));
    for (int v = 0; v < 3 * NA; ++v)   // x + (-0.0) == x: the fixed slot sums
      for (int k = nt; k < NMC_NSLOT; ++k) lds[(L.part + v * NMC_NSLOT + k) * 64 + lane] = -0.0;
    nmc_drain_vm();
    lds[L.flag * 64 + lane] = 0.0;   // verdict words and both tile counters
  }
  __syncthreads();

  bool ok = true;
  // ---- the Gibbs waves: task (t-1, gq) during iteration t, then step (t, gq)'s priors ----
  if (gw) {
    for (int t = i0; t < i1 && ok; ++t) {
      const bool due = t > i0;
      if (due) {
        const bool r = nmc_poll_published(d, cb, gq, (unsigned)G * (unsigned)(t - i0));
        if (lane == 0)
          __hip_atomic_store(lds + L.flag * 64 + 1 + gq, r ? 2.0 * ((double)t + 1) : -2.0 * ((double)t + 1),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (gq == 0) NMC_STAMP_AUX(t, 13);
        if (r) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          double xv[64], fz, fx;
          nmc_hyper_fetch_reg(d, t - 1, gq, cc, xv, fz, fx);
#ifdef NMC_STAMPS
          nmc_drain_vm();
          if (gq == 0) NMC_STAMP_AUX(t, 14);
#endif
          nmc_hyper_compute_reg(d, cb, t - 1, gq, lds, L.hyp, g == 0, fz, fx, xv);
          if (gq == 0) NMC_STAMP_AUX(t, 15);
          const double v = th[gq * 64];
          const double prop = v + (1.0 * st[(NMC_ST_S * 2 + gq) * 64]) * zl_slot(t, gq)[2 * lane];
          const double m = hy[(NMC_HY_MU * 2 + gq) * 64], sd = hy[(NMC_HY_SD * 2 + gq) * 64];
          const double lsd = hy[(NMC_HY_LSD * 2 + gq) * 64], isd = hy[(NMC_HY_ISD * 2 + gq) * 64];
          cwv[(NMC_PW_LPC0 + 2 * gq) * 64] = nmc_norm_logpdf_r(v, m, sd, isd, lsd);   // t > 0
          cwv[(NMC_PW_LPP0 + 2 * gq) * 64] = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
        }
      }
      __syncthreads();   // A
      if (due) {
        ok = lds[L.flag * 64 + 1] == 2.0 * ((double)t + 1) &&
             lds[L.flag * 64 + 2] == 2.0 * ((double)t + 1);
        if (!ok) break;
      }
      __syncthreads();   // B
      // publish this workgroup's decided value of gq write-through, then count it (the
      // store drain stays off the control wave's path)
      if (live)
        __hip_atomic_store(((t & 1) ? d.vb1 : d.vb0) + (size_t)gq * GC + gc, th[gq * 64],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nmc_drain_vm();
      if (lane == 0)
        __hip_atomic_fetch_add(nmc_counter(d, cb, gq, g & 7), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    // closing: task (i1-1, gq), written and recorded by the group-0 workgroups
    if (ok && g == 0 && nmc_poll_published(d, cb, gq, (unsigned)G * (unsigned)(i1 - i0))) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double xv[64], fz, fx;
      nmc_hyper_fetch_reg(d, i1 - 1, gq, cc, xv, fz, fx);
      nmc_hyper_compute_reg(d, cb, i1 - 1, gq, lds, L.hyp, true, fz, fx, xv);
    }
    nmc_drain_vm();
    return;
  }

  // ---- control and likelihood waves ----
  double c_LL = ctl ? d.ll[gc] : 0.0;
  bool q_acc[2] = {false, false};
  double q_plp[2] = {0, 0}, q_pll[2] = {0, 0};
  int pend_t = -1;       // iteration whose two decided steps await their state update
  auto apply_pending = [&]() {
    for (int q = 0; q < 2; ++q) {
      const int o = NMC_PW_CNT + 5 * q;
      st[(NMC_ST_LP * 2 + q) * 64] = q_plp[q];
      st[(NMC_ST_NA * 2 + q) * 64] = cwv[(o + (q_acc[q] ? 0 : 2)) * 64];
      st[(NMC_ST_NR * 2 + q) * 64] = cwv[(o + (q_acc[q] ? 1 : 3)) * 64];
      st[(NMC_ST_TA * 2 + q) * 64] = cwv[(o + 4) * 64] + (q_acc[q] ? 1.0 : 0.0);
      if (live) {
        const int row = nmc_record_row(d, pend_t);
        if (row >= 0) d.samples[((size_t)row * d.cols + q * (G + 2) + 2 + g) * C + c] = th[q * 64];
        if (pend_t < d.trace_n) {
          const size_t it = (((size_t)pend_t * 2 + q) * G + g) * C + c;
          d.tflag[it] = q_acc[q] ? 1 : 0;
          d.tllp[it] = q_pll[q];
        }
      }
    }
    pend_t = -1;
  };
  for (int t = i0; t < i1 && ok; ++t) {
    NMC_STAMP(t, 0);
    const bool tune = t > 0 && t < d.burn && t % d.tune_interval == 0;
    double c_prop[2], c_v[2], c_lu[2], c_lpc[2], c_lpp[2], c_sA[2], c_sR[2];
    if (ctl) {
      if (pend_t >= 0) apply_pending();
      for (int q = 0; q < 2; ++q) {
        const double* zs = zl_slot(t, q);
        c_v[q] = th[q * 64];
        const double s = st[(NMC_ST_S * 2 + q) * 64];
        c_prop[q] = c_v[q] + (1.0 * s) * zs[2 * lane];   // propose (:304-306)
        c_lu[q] = zs[2 * lane + 1];
        const double na = st[(NMC_ST_NA * 2 + q) * 64], nr = st[(NMC_ST_NR * 2 + q) * 64];
        double naA = na + 1.0, nrA = nr, naR = na, nrR = nr + 1.0;
        c_sA[q] = s;
        c_sR[q] = s;
        if (tune) {
          nmc_tune(c_sA[q], naA, nrA);
          nmc_tune(c_sR[q], naR, nrR);
        }
        const int o = NMC_PW_CNT + 5 * q;
        cwv[o * 64] = naA;
        cwv[(o + 1) * 64] = nrA;
        cwv[(o + 2) * 64] = naR;
        cwv[(o + 3) * 64] = nrR;
        cwv[(o + 4) * 64] = st[(NMC_ST_TA * 2 + q) * 64];
        if (t == i0) {   // no Gibbs task lands in the launch's first iteration: own priors
          const double m = hy[(NMC_HY_MU * 2 + q) * 64], sd = hy[(NMC_HY_SD * 2 + q) * 64];
          const double lsd = hy[(NMC_HY_LSD * 2 + q) * 64], isd = hy[(NMC_HY_ISD * 2 + q) * 64];
          c_lpc[q] = t > 0 ? nmc_norm_logpdf_r(c_v[q], m, sd, isd, lsd) : st[(NMC_ST_LP * 2 + q) * 64];
          c_lpp[q] = nmc_norm_logpdf_r(c_prop[q], m, sd, isd, lsd);
        }
      }
      if (t + 1 < i1) {
        nmc_dma16(zl_src(t + 1, 0), zl_slot(t + 1, 0));
        nmc_dma16(zl_src(t + 1, 1), zl_slot(t + 1, 1));
      }
    }
    // ---- one pass over the rows: A, B and C (:615-635), tile by tile ----
    pass(t);
    NMC_STAMP(t, 1);
    if (ctl) nmc_drain_vm();   // the next iteration's variates have landed
    __syncthreads();   // A
    NMC_STAMP(t, 2);
    if (t > i0) {   // the Gibbs waves' verdicts
      ok = lds[L.flag * 64 + 1] == 2.0 * ((double)t + 1) &&
           lds[L.flag * 64 + 2] == 2.0 * ((double)t + 1);
      if (!ok) break;
    }
    // ---- control wave: step 0 with A, step 1 with B or C (:334-383, :608-610) ----
    if (ctl) {
      if (lane == 0) tcnt[(t & 1) ^ 1] = 0u;   // the next iteration's tile counter
      double sA[NA], sB[NA], sC[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        sA[j] = nmc_sum_slots(lds + (L.part + (0 * NA + j) * NMC_NSLOT) * 64 + lane);
        sB[j] = nmc_sum_slots(lds + (L.part + (1 * NA + j) * NMC_NSLOT) * 64 + lane);
        sC[j] = nmc_sum_slots(lds + (L.part + (2 * NA + j) * NMC_NSLOT) * 64 + lane);
      }
      if (t > i0) {
        c_lpc[0] = cwv[NMC_PW_LPC0 * 64];
        c_lpp[0] = cwv[NMC_PW_LPP0 * 64];
        c_lpc[1] = cwv[NMC_PW_LPC1 * 64];
        c_lpp[1] = cwv[NMC_PW_LPP1 * 64];
      }
      double thp[Fam::MAXP];
#pragma unroll
      for (int q = 0; q < Fam::MAXP; ++q) thp[q] = 0.0;
      thp[0] = c_prop[0]; thp[1] = c_v[1];
      const double llA = fam.finish_fast(fam.prepare(thp), sA, (long)nrow, gcst);
      const bool acc0 = nmc_mh_accept(c_lpc[0], c_LL, c_lpp[0], llA, c_lu[0]);
      thp[0] = c_v[0]; thp[1] = c_prop[1];
      const double llB = fam.finish_fast(fam.prepare(thp), sB, (long)nrow, gcst);
      thp[0] = c_prop[0];
      const double llC = fam.finish_fast(fam.prepare(thp), sC, (long)nrow, gcst);
      const double ll1 = acc0 ? llC : llB;
      const double LL1 = acc0 ? llA : c_LL;
      const bool acc1 = nmc_mh_accept(c_lpc[1], LL1, c_lpp[1], ll1, c_lu[1]);
      const double vn0 = acc0 ? c_prop[0] : c_v[0];
      const double vn1 = acc1 ? c_prop[1] : c_v[1];
      th[0] = vn0;     // published by the Gibbs waves after barrier B
      th[64] = vn1;
      st[(NMC_ST_S * 2 + 0) * 64] = acc0 ? c_sA[0] : c_sR[0];
      st[(NMC_ST_S * 2 + 1) * 64] = acc1 ? c_sA[1] : c_sR[1];
      q_acc[0] = acc0;
      q_acc[1] = acc1;
      q_plp[0] = acc0 ? c_lpp[0] : c_lpc[0];
      q_plp[1] = acc1 ? c_lpp[1] : c_lpc[1];
      q_pll[0] = llA;
      q_pll[1] = ll1;
      c_LL = acc1 ? ll1 : LL1;
      pend_t = t;
      NMC_STAMP(t, 3);
    }
    __syncthreads();   // B: the new values are visible to every wave
  }
  if (ctl) {
    if (pend_t >= 0) apply_pending();
    if (live && ok) {   // ---- epilogue: state back to HBM (values were published) ----
      for (int q = 0; q < 2; ++q) {
        const size_t ip = (size_t)q * GC + gc;
        d.lp[ip] = st[(NMC_ST_LP * 2 + q) * 64];
        d.scale[ip] = st[(NMC_ST_S * 2 + q) * 64];
        d.nacc[ip] = (int)st[(NMC_ST_NA * 2 + q) * 64];
        d.nrej[ip] = (int)st[(NMC_ST_NR * 2 + q) * 64];
        d.tacc[ip] = (long long)st[(NMC_ST_TA * 2 + q) * 64];
      }
      d.ll[gc] = c_LL;
    }
  }
}
