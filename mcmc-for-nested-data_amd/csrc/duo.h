// duo.h -- nmc_k_duo: the partial-pooling step loop without step barriers.
//
// nmc_k_run steps its 64 chains of one group in lock step: every parameter step is a tile
// phase (all waves on the group's rows) followed by a serial phase -- barrier, the control
// wave's sum and Metropolis decision, barrier, restart -- during which the CU's SIMDs
// idle (~5k of ~9k cycles per step at cfg 3).  nmc_k_duo splits the
// workgroup's 64 chains into two independent half blocks of 32 chains (h = 0, 1) that
// step on their own, so one half's tiles fill the SIMDs while the other half decides:
//
//   * tickets: every (half, step) release appends a record to an LDS ring; a wave takes
//     the next ticket (one LDS atomic), ticket n = tile n % nt of record n / nt, and waits
//     only when every released tile is taken -- first come, first served, whichever half;
//   * the wave that completes a (half, step)'s last tile decides it (posteriorSampling.py
//     :334-383, branch order exact), forms the half's next proposal and releases its next
//     step before doing the step's bookkeeping (counters, tuning, publication, sample and
//     trace rows); there is no barrier after the prologue;
//   * one Gibbs wave per half (waves 0 and 1) runs the half's hyper updates
//     (HyperParameter.update :463-498) in task order, as soon as the publication count of
//     the chain block's G groups is full, in numpy's pairwise order (nmc_pairwise_reg);
//     a decision waits (LDS flag) only if its update has not landed yet;
//   * quad row layout: lane (r, j) = (lane >> 4, lane & 15) holds the half's chains j and
//     j + 16 and reads rows 4i + r of a tile -- one ds_read_b128 feeds 128 (chain, row)
//     terms, as the paired loop -- and accumulates exactly the residue-r accumulator a[r]
//     of nmc_ll_rows_lds (rows = r mod 4, in order; the < 16-row tail into a[0]); the
//     tile sum (a0 + a1) + (a2 + a3) is two lane swaps (v_permlane16/32_swap).  Same
//     tiles, same order: every sum is bit-identical to nmc_k_run's.
//
// Scope: partial pooling over G <= 64 groups (the register Gibbs update), rows in LDS, no
// row split, the {x, y} regression rows (Fam::ASM_ROWS); nmc_k_run covers the rest.
#pragma once
#include "kernels.h"

#ifndef NMC_DUO_THREADS
#define NMC_DUO_THREADS 768   // 12 waves (three per SIMD, <= 168 VGPRs): 2 Gibbs + 10 likelihood
#endif
#ifndef NMC_DUO_GIBBS_PRIO
#define NMC_DUO_GIBBS_PRIO 0   // issue priority of the Gibbs wave's arithmetic
#endif
enum { NMC_MODE_DUO = 7 };    // (run_mode / nmc_kernel_name)

// LDS carve (doubles).  Per half (32 chains; columns of 32 doubles): thp [P] the step's
// likelihood parameters (the proposal in place; pair-interleaved: position 2j + (L >> 4)
// holds chain L = j or j + 16, so a tile lane reads both of its chains with one
// ds_read_b128), th [P] current values, st [5][P] scale / log prior / n acc / n rej /
// total acc, ll the group log-likelihood of the current state, hyp [6][P] hyper state
// (NMC_HY_*), part [NSLOT] tile partials (pair-interleaved, unused slots -0.0), zl [4]
// {z, log u} ring (LDS-DMA, 16 B per chain).  Then the control words, the release ring
// and the group's rows.
struct nmc_duo_layout {
  int thp, hyp, part, zl, half;
  int ctl, rows, total;
};
__host__ __device__ inline nmc_duo_layout nmc_duo_lds(int P, int row_doubles) {
  nmc_duo_layout L;
  int o = 0;
  L.thp = o; o += 32 * P;
  L.hyp = o; o += 32 * 4 * P;
  L.part = o; o += 32 * NMC_NSLOT;
  L.zl = o; o += 4 * 64;
  L.half = o;
  L.ctl = 2 * o;                       // 32 u32 words
  L.rows = (L.ctl + 16 + 63) & ~63;
  L.total = L.rows + row_doubles;
  return L;
}
// control words (u32): per half h at 8 h + {tiles done, Gibbs tasks done, tickets taken, steps
// released}; the abort word at 16
enum { NMC_DUO_DONE = 0, NMC_DUO_HREADY = 2, NMC_DUO_TAKE = 3, NMC_DUO_REL = 4,
       NMC_DUO_ABORT = 16 };

__device__ __forceinline__ int nmc_duo_pos(int L) { return 2 * (L & 15) + (L >> 4); }

// Even / odd 16-lane row of each row pair (rows 0/1 and 2/3) in every lane (gfx950
// v_permlane16_swap); nmc_halves is the 32-lane form.
__device__ __forceinline__ nmc_pair2 nmc_rows16(double v) {
  const unsigned l = (unsigned)__double2loint(v), h = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(l, l, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(h, h, false, false);
  nmc_pair2 r;
  r.lo = __hiloint2double((int)b[0], (int)a[0]);
  r.hi = __hiloint2double((int)b[1], (int)a[1]);
  return r;
}

// The quad form of the regression row loop: p = this lane's first row (tile start + r
// rows); nq >= 1 blocks of 16 rows, each lane taking rows 0, 4, 8, 12 of a block (its
// residue) for chain A (b0, b1) into uA and chain B (c0, c1) into uB, in row order --
// the same e = fma(x, b1, b0 - y), acc = fma(e, e, acc) as nmc_rows_lds_linreg2(_paired).
// Two register sets (rows v[120:135] / v[144:159], chain-B residuals v[136:143] /
// v[160:167]); the next block's four reads are in flight while a block is consumed.
#define NMC_Q4(b, off)                                                     \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"         \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+64\n"        \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+128\n"      \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+192\n"
#define NMC_QB(b, t)                                                                        \
  NMC_PDX(b, t, 0, 0) NMC_PDX(b, t, 4, 2) NMC_PDX(b, t, 8, 4) NMC_PDX(b, t, 12, 6)           \
  NMC_PDO(b, 0) NMC_PDO(b, 4) NMC_PDO(b, 8) NMC_PDO(b, 12)                                   \
  NMC_PEO(b, 0) NMC_PEO(b, 4) NMC_PEO(b, 8) NMC_PEO(b, 12)                                   \
  NMC_PEX(b, t, 0, 0) NMC_PEX(b, t, 4, 2) NMC_PEX(b, t, 8, 4) NMC_PEX(b, t, 12, 6)           \
  NMC_PSO(b, 0, u0) NMC_PSX(t, 0, w0) NMC_PSO(b, 4, u0) NMC_PSX(t, 2, w0)                   \
  NMC_PSO(b, 8, u0) NMC_PSX(t, 4, w0) NMC_PSO(b, 12, u0) NMC_PSX(t, 6, w0)
__device__ __forceinline__ void nmc_rows_lds_linreg2_quad(const double* p, int nq, double b0,
                                                          double b1, double c0, double c1,
                                                          double& uA, double& uB) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nq;
  asm volatile(
      NMC_Q4(120, 0)
      "L_nmc_q_%=:\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_eq_u32 %[cnt], 0\n"
      "s_cbranch_scc1 L_nmc_qla_%=\n"
      NMC_Q4(144, 256)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_QB(120, 136)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_eq_u32 %[cnt], 0\n"
      "s_cbranch_scc1 L_nmc_qlb_%=\n"
      NMC_Q4(120, 256)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_QB(144, 160)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_branch L_nmc_q_%=\n"
      "L_nmc_qla_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QB(120, 136)
      "s_branch L_nmc_qdone_%=\n"
      "L_nmc_qlb_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QB(144, 160)
      "L_nmc_qdone_%=:\n"
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(uA), [w0] "+v"(uB)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130",
        "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141",
        "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152",
        "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163",
        "v164", "v165", "v166", "v167", "scc", "memory");
}

// Two full tiles of one ticket in one pass (both of nq >= 1 blocks of 16 rows, no tail):
// each block iteration reads four rows of each tile (eight ds_read_b128 in flight) and feeds
// four accumulators (chains A / B of tile 1: u0 / w0, of tile 2: u1 / w1) in the tiles' own
// row orders -- each tile's sums exactly nmc_rows_lds_linreg2_quad's.  Stage A rows
// v[72:103] (tile 2 from v88), chain-B residuals v[104:119]; stage B v[120:151] / v[152:167].
#define NMC_Q8(b, off)                                                     \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[a1] offset:" #off "+0\n"           \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[a1] offset:" #off "+64\n"          \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[a1] offset:" #off "+128\n"        \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[a1] offset:" #off "+192\n"       \
  "ds_read_b128 v[" #b "+16:" #b "+19], %[a2] offset:" #off "+0\n"         \
  "ds_read_b128 v[" #b "+20:" #b "+23], %[a2] offset:" #off "+64\n"        \
  "ds_read_b128 v[" #b "+24:" #b "+27], %[a2] offset:" #off "+128\n"       \
  "ds_read_b128 v[" #b "+28:" #b "+31], %[a2] offset:" #off "+192\n"
#define NMC_QSO(b, k4, a) \
  "v_fma_f64 %[" #a "], v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], v[" #b "+" #k4 "+2:" #b "+" #k4 "+3], %[" #a "]\n"
#define NMC_QSX(t, k2, a) \
  "v_fma_f64 %[" #a "], v[" #t "+" #k2 ":" #t "+" #k2 "+1], v[" #t "+" #k2 ":" #t "+" #k2 "+1], %[" #a "]\n"
// one tile's four rows of a block: residuals, then the accumulators U (chain A) / W (chain B)
#define NMC_QT(b, t, U, W)                                                                  \
  NMC_PDX(b, t, 0, 0) NMC_PDX(b, t, 4, 2) NMC_PDX(b, t, 8, 4) NMC_PDX(b, t, 12, 6)           \
  NMC_PDO(b, 0) NMC_PDO(b, 4) NMC_PDO(b, 8) NMC_PDO(b, 12)                                   \
  NMC_PEO(b, 0) NMC_PEO(b, 4) NMC_PEO(b, 8) NMC_PEO(b, 12)                                   \
  NMC_PEX(b, t, 0, 0) NMC_PEX(b, t, 4, 2) NMC_PEX(b, t, 8, 4) NMC_PEX(b, t, 12, 6)           \
  NMC_QSO(b, 0, U) NMC_QSX(t, 0, W) NMC_QSO(b, 4, U) NMC_QSX(t, 2, W)                       \
  NMC_QSO(b, 8, U) NMC_QSX(t, 4, W) NMC_QSO(b, 12, U) NMC_QSX(t, 6, W)
#define NMC_QB2(b, t) NMC_QT(b, t, u0, w0) NMC_QT(b + 16, t + 8, u1, w1)
__device__ __forceinline__ void nmc_rows_lds_linreg2_quad2(const double* p1, const double* p2,
                                                           int nq, double b0, double b1,
                                                           double c0, double c1, double& uA1,
                                                           double& uB1, double& uA2,
                                                           double& uB2) {
  unsigned a1 = (unsigned)(uintptr_t)(nmc_lds_cptr)p1;
  unsigned a2 = (unsigned)(uintptr_t)(nmc_lds_cptr)p2;
  int cnt = nq;
  asm volatile(
      NMC_Q8(72, 0)
      "L_nmc_q2_%=:\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_eq_u32 %[cnt], 0\n"
      "s_cbranch_scc1 L_nmc_q2la_%=\n"
      NMC_Q8(120, 256)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_QB2(72, 104)
      "v_add_u32 %[a1], 0x100, %[a1]\n"
      "v_add_u32 %[a2], 0x100, %[a2]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_eq_u32 %[cnt], 0\n"
      "s_cbranch_scc1 L_nmc_q2lb_%=\n"
      NMC_Q8(72, 256)
      "s_waitcnt lgkmcnt(8)\n"
      NMC_QB2(120, 152)
      "v_add_u32 %[a1], 0x100, %[a1]\n"
      "v_add_u32 %[a2], 0x100, %[a2]\n"
      "s_branch L_nmc_q2_%=\n"
      "L_nmc_q2la_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QB2(72, 104)
      "s_branch L_nmc_q2done_%=\n"
      "L_nmc_q2lb_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_QB2(120, 152)
      "L_nmc_q2done_%=:\n"
      : [a1] "+v"(a1), [a2] "+v"(a2), [cnt] "+s"(cnt), [u0] "+v"(uA1), [w0] "+v"(uB1),
        [u1] "+v"(uA2), [w1] "+v"(uB2)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83",
        "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95",
        "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
        "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117",
        "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128",
        "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139",
        "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150",
        "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161",
        "v162", "v163", "v164", "v165", "v166", "v167", "scc", "memory");
}

// (a0 + a1) + (a2 + a3) of the lane's residue accumulators, in every lane of the quad
__device__ __forceinline__ double nmc_duo_reduce(double u) {
  const nmc_pair2 a16 = nmc_rows16(u);
  const nmc_pair2 a32 = nmc_halves(a16.lo + a16.hi);
  return a32.lo + a32.hi;
}

// Tile [ra, ra + rn) of the group's rows (LDS) for the lane's two chains: the 4-way part
// (the first 8 * nb2 rows, nb2 = (rn / 8) & ~1 as nmc_ll_rows_lds) by residue, the tail in
// order into residue 0, then (a0 + a1) + (a2 + a3) in every lane.  Returns {A, B}.
template <class Fam>
__device__ __forceinline__ nmc_pair2 nmc_duo_tile(const Fam& fam, const typename Fam::Reg& ra_,
                                                  const typename Fam::Reg& rb_,
                                                  const double* rows, int rn) {
  constexpr int NF = Fam::NFIELDS;
  static_assert(Fam::ASM_ROWS && NF == 2, "nmc_k_duo: the {x, y} regression rows");
  const int lane = threadIdx.x & 63;
  const int r = lane >> 4;
  double uA = 0.0, uB = 0.0;
  const int nb2 = (rn / 8) & ~1;
  if (nb2 > 0)
    nmc_rows_lds_linreg2_quad(rows + (size_t)r * NF, nb2 >> 1, ra_.b0, ra_.b[0], rb_.b0, rb_.b[0],
                              uA, uB);
  if (r == 0) {   // the < 16-row tail, in order, into residue 0 (nmc_ll_rows_lds: a[0])
    for (int i = nb2 * 8; i < rn; ++i) {
      const double* q = rows + (size_t)i * NF;
      fam.accum(ra_, q, &uA);
      fam.accum(rb_, q, &uB);
    }
  }
  nmc_pair2 out;
  out.lo = nmc_duo_reduce(uA);
  out.hi = nmc_duo_reduce(uB);
  return out;
}

// numpy's pairwise sum of x[0..G) (G <= 64; nmc_pairwise_reg's order and operations) with
// the values split over the lane halves: lanes 0-31 hold x[0..31] of their chain, lanes
// 32-63 x[32..63] of the same chain (32 registers each instead of 64).  The eight streams
// r_j = x_j + x_{j+8} + ... run blocks 0-3 in the low lanes, are handed over (lane swap) and
// continue with blocks 4-7 in the high lanes; the G % 8 tail is added in order there.  The
// result reaches every lane.
__device__ __forceinline__ double nmc_pairwise_split(const double (&x)[32], int G, bool sq,
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
#pragma unroll
  for (int u = 1; u < 4; ++u)
    if (u < cnt) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + tr(x[8 * u + j]);
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = nmc_halves(r[j]).lo;   // the low lanes' streams
#pragma unroll
  for (int u = 4; u < 8; ++u)
    if (u < cnt) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + tr(x[8 * (u - 4) + j]);
    }
  double res = cnt ? ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])) : 0.0;
  // the G % 8 tail (G < 8: the whole sum from 0), block m8 / 8 of the low or high lanes
  double tv[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) tv[k] = 0.0;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (8 * u == (m8 & 31)) {
#pragma unroll
      for (int k = 0; k < 7; ++k) tv[k] = x[8 * u + k];
    }
  const bool tail_hi = m8 >= 32;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const nmc_pair2 e = nmc_halves(tv[k]);
    tv[k] = tail_hi ? e.hi : e.lo;
  }
  const int nt = G - m8;
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if (k < nt) res += tr(tv[k]);
  return nmc_halves(res).hi;   // (the high lanes hold it)
}

// The tile partials of one sum in nmc_sum_slots' order, from the pair-interleaved columns
// of a half (stride 32).
__device__ __forceinline__ double nmc_duo_sum_slots(const double* pt) {
  double v[NMC_NSLOT];
#pragma unroll
  for (int u = 0; u < NMC_NSLOT; ++u) v[u] = pt[u * 32];
  double a4[4];
#pragma unroll
  for (int u = 0; u < NMC_NSLOT; ++u) a4[u & 3] = u < 4 ? v[u] : a4[u & 3] + v[u];
  return (a4[0] + a4[1]) + (a4[2] + a4[3]);
}

// Diagnostic build only (make duostamps -> libnestmc_ds.so, never shipped): shader-clock
// stamps of workgroup 0 -- decisions [h][s < 64][4] at 0 (detected, waits done, released,
// bookkeeping done), Gibbs tasks [h][s < 64][4] at 640 (loop top, poll done, computed),
// tickets [record < 128][first tile < 16][3] at 1152 (start, done, wave).
#ifdef NMC_DUO_STAMPS
#define NMC_DS(idx)                                                                        \
  do {                                                                                     \
    if (d.stamps && blockIdx.x == 0 && lane == 0)                                          \
      d.stamps[(idx)] = __builtin_amdgcn_s_memtime();                                      \
  } while (0)
#define NMC_DS_DEC(h, s, k) do { if ((s) < 64) NMC_DS(((h) * 64 + (s)) * 5 + (k)); } while (0)
#define NMC_DS_GIB(h, s, k) do { if ((s) < 64) NMC_DS(640 + ((h) * 64 + (s)) * 4 + (k)); } while (0)
#define NMC_DS_TILE(r, k, e)                                                               \
  do {                                                                                     \
    if ((r) < 128 && (k) < 16) {                                                           \
      NMC_DS(1152 + ((r) * 16 + (k)) * 3 + (e));                                           \
      if ((e) == 1 && d.stamps && blockIdx.x == 0 && lane == 0)                             \
        d.stamps[1152 + ((r) * 16 + (k)) * 3 + 2] = (unsigned long long)w;                 \
    }                                                                                      \
  } while (0)
#else
#define NMC_DS_DEC(h, s, k) do {} while (0)
#define NMC_DS_GIB(h, s, k) do {} while (0)
#define NMC_DS_TILE(r, k, e) do {} while (0)
#endif

// Bounded LDS spin until control word k reaches target: false once the abort word is set
// or after NMC_SPIN_LIMIT polls (then the timeout word and the abort word are set, so every
// wave of the workgroup leaves and the host reports the timeout).
__device__ __forceinline__ bool nmc_duo_spin(const Dev& d, unsigned* ctl, int k, unsigned target) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = __hip_atomic_load(ctl + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (v >= target) return true;
    if (__hip_atomic_load(ctl + NMC_DUO_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
      return false;
    if (spins >= NMC_SPIN_LIMIT) {
      __hip_atomic_store(d.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(ctl + NMC_DUO_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <class Fam>
__global__ void __launch_bounds__(NMC_DUO_THREADS)
nmc_k_duo(Dev d_arg, Fam fam, const double* __restrict__ obs, int i0, int i1, int flags) {
  // (flags: nmc_k_run's; a persistent launch always starts from the hyper state of i0 - 1)
  (void)d_arg;   // (read through nmc_kdev(): the same bytes)
  (void)flags;
  constexpr int MP = Fam::MAXP;
  const Dev* dP = nmc_kdev();
#define d (*dP)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = d.P, G = d.G, C = d.C;
  const int b = blockIdx.x;
  const int g = b % G, cb = b / G + d.cb0;
  const int ngrp = (int)(d.off[g + 1] - d.off[g]);
  const nmc_tiling TI = nmc_tiles(ngrp, d.tile);
  const int nt = TI.nt;
  const int nsteps = (i1 - i0) * P;
  // half blocks with at least one chain (a chain block of <= 32 chains runs half 0 only)
  const int nh = cb * 64 + 32 < C ? 2 : 1;
  const nmc_duo_layout L = nmc_duo_lds(P, d.nmax * Fam::NFIELDS);
  unsigned* ctl = (unsigned*)(lds + L.ctl);
  double* lrows = lds + L.rows;
  const size_t PGC = (size_t)P * G * C;
  const int Lc = lane & 31;   // a role wave's chain within its half (lanes 32-63 mirror 0-31)
  const bool lo = lane < 32;

  // Roles: wave h (h < 2) the Gibbs wave of half h, wave 2 + h its control wave, waves 4..
  // the likelihood tiles.
  const bool gibbs = w < 2, control = w >= 2 && w < 4;
  const int hr = gibbs ? w : w - 2;   // the role wave's half
  const int c = cb * 64 + 32 * hr + Lc;
  const int cc = c < C ? c : C - 1;
  const bool live = lo && c < C;
  double* H = lds + hr * L.half;

  // ---- prologue (every wave meets one barrier, in its role's branch) ----
  {
    const int nd = ngrp * Fam::NFIELDS;
    const double* grows = obs + d.off[g] * Fam::NFIELDS;
    for (int i = threadIdx.x; i < nd; i += blockDim.x) lrows[i] = grows[i];
  }

  // ---- the Gibbs wave of half hr: the half's hyper updates in task order ----
  if (gibbs) {
    const int h = hr;
    const int hb = 2 * cb + h;   // publication counters per 32-chain half block
    double s2v[MP];               // sigma2 of each parameter's last update
#pragma unroll
    for (int q = 0; q < MP; ++q)
      s2v[q] = q < P ? d.s2[nmc_hslot(d, i0 - 1) + (size_t)q * C + cc] : 0.0;
    __syncthreads();
    if (h >= nh) return;   // (an empty half block)
    __builtin_amdgcn_s_setprio(3);
    // (the parameter loop unrolled: every per-parameter register is indexed by a constant)
    for (int t = i0; t < i1; ++t)
#pragma unroll
    for (int p = 0; p < MP; ++p) {
      if (p >= P) break;
      const int s = (t - i0) * P + p;
      dP = nmc_kdev();
      const bool needed = s + P < nsteps;   // the decision of step s + P uses it
      const int jl = s - (nsteps - P);      // the launch's closing tasks: group jl % G writes
      const bool writer = needed ? g == 0 : g == jl % G;
      if (!needed && !writer) continue;
      NMC_DS_GIB(h, s, 0);
      if (!nmc_poll_published(d, hb, p, (unsigned)G * (unsigned)(t - i0 + 1))) {
        if (lane == 0)
          __hip_atomic_store(ctl + NMC_DUO_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        goto gibbs_done;
      }
      // keep the payload loads below the poll (no instruction: wavefront scope)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      NMC_DS_GIB(h, s, 1);
      // (the update's arithmetic at the likelihood waves' priority: at priority 3 its ~2k
      //  cycles of sqrt / log / divisions held back the two likelihood waves of its SIMD)
      __builtin_amdgcn_s_setprio(NMC_DUO_GIBBS_PRIO);
      // the chain block's values of p after t: groups 0-31 in the low lanes, 32-63 in the
      // high ones (sc1 loads, all in flight; groups >= G read the buffers' slack)
      double xv[32];
      {
        const double* src = ((t & 1) ? d.vb1 : d.vb0) + (size_t)p * G * C + cc +
                            (lo ? (size_t)0 : (size_t)32 * C);
#pragma unroll
        for (int k = 0; k < 32; ++k) xv[k] = nmc_ldv<NMC_SRC_SC1>(src + (size_t)k * C);
      }
      const size_t hvi = (((size_t)(t - d.vbase) * P + p) * C + cc) * 2;
      const double hz = d.vh[hvi], hx = d.vh[hvi + 1];
      const double sdm = sqrt(s2v[p] / G);
      const double tot = nmc_pairwise_split(xv, G, false, 0.0);
      const double mu = tot / G + sdm * hz;                        // mu ~ N(mean(x), sqrt(s2/G))
      const double ss = nmc_pairwise_split(xv, G, true, mu);
      const double hat = ss / (double)(G - 1);
      const double scl = d.ha * hat;
      // scipy invgamma.rvs: (1/gammainccinv(a, U)) * scale + loc; loc when scale == 0
      const double s2n = scl == 0.0 ? 0.0 : (1.0 / hx) * scl;
      const double sdn = sqrt(s2n);
      const double lsd = log(sdn);
      s2v[p] = s2n;
      if (lo) {   // the half's hyper state of p for its control wave (setPrior :273-282)
        double* hy = H + L.hyp + Lc;
        hy[32 * (0 * P + p)] = mu;
        hy[32 * (1 * P + p)] = sdn;
        hy[32 * (2 * P + p)] = lsd;
        hy[32 * (3 * P + p)] = 1.0 / sdn;
      }
      if (writer && live) {
        // the global hyper slot (t & 1) is what the next launch starts from: written by the
        // launch's closing tasks only, one writer per address -- two workgroups' write-back
        // stores to one address (tasks t - 2 and t) land in their XCDs' L2s in any order
        if (!needed) {
          const size_t ho = nmc_hslot(d, t) + (size_t)p * C + c;
          d.mu[ho] = mu;
          d.s2[ho] = s2n;
          d.hsd[ho] = sdn;
          d.hlsd[ho] = lsd;
        }
        const int row = nmc_record_row(d, t);
        if (row >= 0) {
          double* out = d.samples + ((size_t)row * d.cols + (size_t)p * (G + 2)) * C + c;
          out[0] = mu;
          out[C] = s2n;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      NMC_DS_GIB(h, s, 2);
      if (lane == 0)
        __hip_atomic_store(ctl + 8 * h + NMC_DUO_HREADY, (unsigned)(s + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      __builtin_amdgcn_s_setprio(3);
    }
  gibbs_done:
    nmc_drain_vm();
    return;
  }

  // ---- the control wave of half hr: every decision of the half (:334-383) ----
  if (control) {
    const int h = hr;
    const int pos = nmc_duo_pos(Lc);
    const size_t gc = (size_t)g * C + c;
    // the half's chains, one per lane (posteriorSampling.py :234-437 per (chain, p)):
    // values, scale, log prior, counters since the last tune and in total, the group LL,
    // the hyper-prior of each parameter (mu, sd, log sd, 1 / sd), the step's proposal
    double th[MP], sc[MP], lpv[MP], na[MP], nr[MP], ta[MP], hm[MP], hs[MP], hl[MP], hi[MP];
    {
      const double* vin = ((i0 - 1) & 1) ? d.vb1 : d.vb0;
#pragma unroll
      for (int q = 0; q < MP; ++q) {
        const int qq = q < P ? q : 0;
        const size_t ip = ((size_t)qq * G + g) * C + cc;
        const size_t ho = nmc_hslot(d, i0 - 1) + (size_t)qq * C + cc;   // after i0 - 1
        th[q] = vin[ip];
        sc[q] = d.scale[ip];
        lpv[q] = d.lp[ip];
        na[q] = (double)d.nacc[ip];
        nr[q] = (double)d.nrej[ip];
        ta[q] = (double)d.tacc[ip];
        hm[q] = d.mu[ho];
        hs[q] = d.hsd[ho];
        hl[q] = d.hlsd[ho];
        hi[q] = 1.0 / hs[q];
      }
    }
    double LL = d.ll[(size_t)g * C + cc];
    if (lo) {
      for (int k = nt; k < NMC_NSLOT; ++k) H[L.part + 32 * k + Lc] = -0.0;
      // {z, log u} of the first three steps -> zl slots 0..2 (this wave's own DMAs)
      for (int s = 0; s < 3 && s < nsteps; ++s) {
        const int t = i0 + s / P, p = s % P;
        nmc_dma16(d.vzl + ((size_t)(t - d.vbase) * PGC + ((size_t)p * G + g) * C + cc) * 2,
                  H + L.zl + 64 * s);
      }
    }
    nmc_drain_vm();
    // step 0's likelihood parameters: the proposal of parameter 0
    double prop = th[0] + (1.0 * sc[0]) * H[L.zl + 2 * Lc];
    if (lo) {
#pragma unroll
      for (int q = 0; q < MP; ++q)
        if (q < P) H[L.thp + 32 * q + nmc_duo_pos(Lc)] = q == 0 ? prop : th[q];
    }
    if (lane == 0) {   // (LDS is not cleared between workgroups: every word is set here)
      ctl[8 * h + NMC_DUO_DONE] = 0;
      ctl[8 * h + NMC_DUO_HREADY] = 0;
      ctl[8 * h + NMC_DUO_TAKE] = 0;
      ctl[8 * h + NMC_DUO_REL] = 1;   // step 0 released
      if (h == 0) ctl[NMC_DUO_ABORT] = 0;
    }
    __syncthreads();
    if (h >= nh) return;   // (an empty half block)
    __builtin_amdgcn_s_setprio(3);
    bool ok = true;
    // (the parameter loop unrolled: every per-parameter register is indexed by a constant)
    for (int t = i0; t < i1 && ok; ++t)
#pragma unroll
    for (int p = 0; p < MP; ++p) {
      if (p >= P || !ok) break;
      const int s = (t - i0) * P + p;
      dP = nmc_kdev();
      const bool last = s + 1 == nsteps;
      const bool wrap = p + 1 >= P;   // the next step proposes parameter 0
      // -- before the step's tiles are done: the update after iteration t - 1 (task s - P),
      //    the priors of the current value and the proposal (:293-294), the variates --
      if (s >= P) {
        if (!nmc_duo_spin(d, ctl, 8 * h + NMC_DUO_HREADY, (unsigned)(s - P + 1))) {
          ok = false;
          break;
        }
        const double* hy = H + L.hyp + Lc;
        hm[p] = hy[32 * (0 * P + p)];
        hs[p] = hy[32 * (1 * P + p)];
        hl[p] = hy[32 * (2 * P + p)];
        hi[p] = hy[32 * (3 * P + p)];
      }
      const double v = th[p];
      const double m = hm[p], sd = hs[p], lsd = hl[p], isd = hi[p];
      const double lpc = t > 0 ? nmc_norm_logpdf_r(v, m, sd, isd, lsd) : lpv[p];
      const double lpp = nmc_norm_logpdf_r(prop, m, sd, isd, lsd);
      // this wave's DMAs of steps s and s + 1 have landed (issued two or more steps ago)
      nmc_drain_vm();
      const double lu = H[L.zl + 64 * (s & 3) + 2 * Lc + 1];
      const double zn = last ? 0.0 : H[L.zl + 64 * ((s + 1) & 3) + 2 * Lc];
      const bool tune = t > 0 && t < d.burn && t % d.tune_interval == 0;
      // -- the tiles of step s --
      if (!nmc_duo_spin(d, ctl, 8 * h + NMC_DUO_DONE, (unsigned)nt * (unsigned)(s + 1))) {
        ok = false;
        break;
      }
      NMC_DS_DEC(h, s, 0);
      // -- the decision: group LL of the proposal (tiles in order), Metropolis test --
      double acc[Fam::NACC];
      acc[0] = nmc_duo_sum_slots(H + L.part + pos);
      double thq[MP];
#pragma unroll
      for (int q = 0; q < MP; ++q) thq[q] = q == p ? prop : th[q];
      const double llp = fam.finish_fast(fam.prepare(thq), acc, (long)ngrp, fam.gconst((long)ngrp));
      const double postp = lpp + llp;
      const double post = lpc + LL;
      const double diff = postp - post;
      bool accept;
      if (!isfinite(post) && isfinite(postp)) accept = true;        // :347-352
      else if (!isfinite(llp)) accept = false;                      // :354-356
      else if (!isfinite(diff)) accept = false;                     // :358-360
      else accept = lu < diff;                                      // :362-364
      const double vn = accept ? prop : v;                          // :369-383
      double sN = sc[p], naN = na[p], nrN = nr[p];
      naN = accept ? naN + 1.0 : naN;
      nrN = accept ? nrN : nrN + 1.0;
      if (tune) nmc_tune(sN, naN, nrN);                             // :385-437
      th[p] = vn;
      sc[p] = sN;
      // -- the next step's likelihood parameters (the proposal of pn, :304-306), released --
      if (!last) {
        const int pn1 = p + 1 < MP ? p + 1 : 0;   // (a constant once unrolled)
        prop = (wrap ? th[0] : th[pn1]) + (1.0 * (wrap ? sc[0] : sc[pn1])) * zn;
        if (lo) {
#pragma unroll
          for (int q = 0; q < MP; ++q)
            if (q < P) H[L.thp + 32 * q + pos] = q == (wrap ? 0 : pn1) ? prop : th[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the parameters are in LDS
        if (lane == 0)   // release step s + 1 of the half
          __hip_atomic_store(ctl + 8 * h + NMC_DUO_REL, (unsigned)(s + 2), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      NMC_DS_DEC(h, s, 2);
      // -- the rest of the update (:369-383, :608-610), off the critical path --
      na[p] = naN;
      nr[p] = nrN;
      ta[p] = ta[p] + (accept ? 1.0 : 0.0);
      lpv[p] = accept ? lpp : lpc;
      if (accept) LL = llp;
      if (lo && s + 3 < nsteps) {   // {z, log u} of step s + 3 -> the slot step s - 1 used
        const int t3 = i0 + (s + 3) / P, p3 = (s + 3) % P;
        nmc_dma16(d.vzl + ((size_t)(t3 - d.vbase) * PGC + ((size_t)p3 * G + g) * C + cc) * 2,
                  H + L.zl + 64 * ((s + 3) & 3));
      }
      if (live) {
        // publish write-through; counted below once stored (the Gibbs waves poll the count)
        __hip_atomic_store(((t & 1) ? d.vb1 : d.vb0) + (size_t)p * G * C + gc, vn,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int row = nmc_record_row(d, t);
        if (row >= 0)
          d.samples[((size_t)row * d.cols + (size_t)p * (G + 2) + 2 + g) * C + c] = vn;
        if (t < d.trace_n) {
          const size_t it = (((size_t)t * P + p) * G + g) * C + c;
          d.tflag[it] = accept ? 1 : 0;
          d.tllp[it] = llp;
        }
      }
      nmc_drain_vm();   // the value is stored before it is counted
      if (lane == 0)
        __hip_atomic_fetch_add(nmc_counter(d, 2 * cb + h, p, g & 7), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      NMC_DS_DEC(h, s, 3);
    }
    if (ok && live) {   // the half's state after the launch
#pragma unroll
      for (int q = 0; q < MP; ++q) {
        if (q < P) {
          const size_t ip = (size_t)q * G * C + gc;
          d.lp[ip] = lpv[q];
          d.scale[ip] = sc[q];
          d.nacc[ip] = (int)na[q];
          d.nrej[ip] = (int)nr[q];
          d.tacc[ip] = (long long)ta[q];
        }
      }
      d.ll[gc] = LL;
    }
    nmc_drain_vm();
    return;
  }

  // ---- every other wave: tickets of KT likelihood tiles of its half (waves 4..7: half 0,
  //      8..11: half 1 -- one of each half on every SIMD, whose waves a workgroup fills in
  //      the cyclic order 0, 2, 1, 3), or of half 0 when the chain block has one half ----
  __syncthreads();
  const int j16 = lane & 15;
  const int KT = d.dkt > 0 ? d.dkt : 1;
  const int ntk = (nt + KT - 1) / KT;
  const int ntw = (int)(blockDim.x >> 6) - 4;   // likelihood waves
  const int h = nh == 2 && (w - 4) >= ntw / 2 ? 1 : 0;
  double* Ht = lds + h * L.half;
  int cur_s = -1;
  typename Fam::Reg regA{}, regB{};
  for (;;) {
    dP = nmc_kdev();
    unsigned n = 0;
    if (lane == 0)
      n = __hip_atomic_fetch_add(ctl + 8 * h + NMC_DUO_TAKE, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
    n = __builtin_amdgcn_readlane(n, 0);
    const int s = (int)(n / (unsigned)ntk), kk = (int)(n % (unsigned)ntk);
    if (s >= nsteps) break;   // every ticket of the half's launch is taken
    if (s != cur_s) {   // wait for the step's release, then its likelihood parameters
      if (!nmc_duo_spin(d, ctl, 8 * h + NMC_DUO_REL, (unsigned)(s + 1))) break;
      double tA[MP], tB[MP];
#pragma unroll
      for (int q = 0; q < MP; ++q) {
        tA[q] = 0.0;
        tB[q] = 0.0;
        if (q < P) {
          const double2 v2 = *(const double2*)(Ht + L.thp + 32 * q + 2 * j16);
          tA[q] = v2.x;
          tB[q] = v2.y;
        }
      }
      regA = fam.prepare(tA);
      regB = fam.prepare(tB);
      cur_s = s;
    }
    // a step's tickets from its last tiles back: the group's short last tile (its own
    // loop, the slowest ticket) starts first instead of ending the step
    const int k0 = (ntk - 1 - kk) * KT, k1 = k0 + KT < nt ? k0 + KT : nt;
    NMC_DS_TILE(h * nsteps + s, k0, 0);
    int k = k0;
    if (k1 - k0 == 2 && TI.len(k0) == TI.len(k0 + 1) && TI.len(k0) % 16 == 0) {
      // two full tiles (no tail): one fused pass
      const int rn = TI.len(k0);
      const double* r1 = lrows + ((size_t)TI.start(k0) + (size_t)(lane >> 4)) * Fam::NFIELDS;
      const double* r2 = lrows + ((size_t)TI.start(k0 + 1) + (size_t)(lane >> 4)) * Fam::NFIELDS;
      double uA1 = 0.0, uB1 = 0.0, uA2 = 0.0, uB2 = 0.0;
      nmc_rows_lds_linreg2_quad2(r1, r2, rn >> 4, regA.b0, regA.b[0], regB.b0, regB.b[0], uA1,
                                 uB1, uA2, uB2);
      const double tA1 = nmc_duo_reduce(uA1), tB1 = nmc_duo_reduce(uB1);
      const double tA2 = nmc_duo_reduce(uA2), tB2 = nmc_duo_reduce(uB2);
      if (lane < 16) {
        *(double2*)(Ht + L.part + 32 * k0 + 2 * j16) = make_double2(tA1, tB1);
        *(double2*)(Ht + L.part + 32 * (k0 + 1) + 2 * j16) = make_double2(tA2, tB2);
      }
      k = k1;
    }
    for (; k < k1; ++k) {
      const int ra = TI.start(k), rn = TI.len(k);
      const nmc_pair2 tot = nmc_duo_tile(fam, regA, regB, lrows + (size_t)ra * Fam::NFIELDS, rn);
      if (lane < 16) *(double2*)(Ht + L.part + 32 * k + 2 * j16) = make_double2(tot.lo, tot.hi);
    }
    // (LDS executes a wave's operations in order: the partials land before the count)
    asm volatile("" ::: "memory");
    if (lane == 0)
      __hip_atomic_fetch_add(ctl + 8 * h + NMC_DUO_DONE, (unsigned)(k1 - k0), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    NMC_DS_TILE(h * nsteps + s, k0, 1);
  }
#undef d
}
