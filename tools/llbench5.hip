// llbench5.hip -- the likelihood tile loop of the step kernel in isolation (diagnostics,
// not shipped): one (64-chain block, group) per workgroup, W waves taking the 16 tiles of a
// 1000-row {x, y} group from an LDS counter, NPASS passes with a barrier between passes --
// the tile phase of nmc_k_step without the roles and the decision.
//   V  no loads: the same three fp64 VALU ops per (chain, row) on register operands
//   P  the shipped paired loop: nmc_ll_rows_lds<FamLinreg<2>, true> (2 chains per lane)
//   B  the broadcast loop: nmc_ll_rows_lds<FamLinreg<2>, false> (1 chain per lane)
//   Q  quad: lane groups of 16 read rows 4m + g, every lane evaluates its row for 4 chains
//      (its own and lanes ^16, ^32, ^48) -- a quarter of the broadcast loop's LDS reads
// Prints cycles per pass (s_memtime, workgroup 0) and checks Q's tile sums against B's.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

constexpr int N = 1000, TILE = 64, NSL = 16;

// Quad row loop over nq (>= 2, even) 16-row granules from this lane group's first row p:
// per granule four ds_read_b128 (rows p, p + 4, p + 8, p + 12 of the granule), each row
// evaluated for the four chains k with parameters (b0[k], b1[k]) into acc[k].
#define Q_LD(b, off)                                                  \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"    \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+64\n"   \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+128\n" \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+192\n"
// row r of register set b: x = v[b+4r : b+4r+1], y = v[b+4r+2 : b+4r+3]; residual temps
// t[2k : 2k+1] for chain k
#define Q_ROW(b, r)                                                                                  \
  "v_add_f64 v[176:177], %[c0], -v[" #b "+" #r "*4+2:" #b "+" #r "*4+3]\n"                           \
  "v_add_f64 v[178:179], %[c1], -v[" #b "+" #r "*4+2:" #b "+" #r "*4+3]\n"                           \
  "v_add_f64 v[180:181], %[c2], -v[" #b "+" #r "*4+2:" #b "+" #r "*4+3]\n"                           \
  "v_add_f64 v[182:183], %[c3], -v[" #b "+" #r "*4+2:" #b "+" #r "*4+3]\n"                           \
  "v_fma_f64 v[176:177], v[" #b "+" #r "*4:" #b "+" #r "*4+1], %[d0], v[176:177]\n"                  \
  "v_fma_f64 v[178:179], v[" #b "+" #r "*4:" #b "+" #r "*4+1], %[d1], v[178:179]\n"                  \
  "v_fma_f64 v[180:181], v[" #b "+" #r "*4:" #b "+" #r "*4+1], %[d2], v[180:181]\n"                  \
  "v_fma_f64 v[182:183], v[" #b "+" #r "*4:" #b "+" #r "*4+1], %[d3], v[182:183]\n"                  \
  "v_fma_f64 %[a0], v[176:177], v[176:177], %[a0]\n"                                                 \
  "v_fma_f64 %[a1], v[178:179], v[178:179], %[a1]\n"                                                 \
  "v_fma_f64 %[a2], v[180:181], v[180:181], %[a2]\n"                                                 \
  "v_fma_f64 %[a3], v[182:183], v[182:183], %[a3]\n"
#define Q_G(b) Q_ROW(b, 0) Q_ROW(b, 1) Q_ROW(b, 2) Q_ROW(b, 3)
__device__ __forceinline__ void quad_rows(const double* p, int nq, const double (&b0)[4],
                                          const double (&b1)[4], double (&a)[4]) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nq;
  asm volatile(
      Q_LD(184, 0)
      "L_q_%=:\n"
      Q_LD(200, 256)
      "s_waitcnt lgkmcnt(4)\n"
      Q_G(184)
      "v_add_u32 %[addr], 0x200, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_qlast_%=\n"
      Q_LD(184, 0)
      "s_waitcnt lgkmcnt(4)\n"
      Q_G(200)
      "s_branch L_q_%=\n"
      "L_qlast_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      Q_G(200)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]),
        [a3] "+v"(a[3])
      : [c0] "v"(b0[0]), [c1] "v"(b0[1]), [c2] "v"(b0[2]), [c3] "v"(b0[3]), [d0] "v"(b1[0]),
        [d1] "v"(b1[1]), [d2] "v"(b1[2]), [d3] "v"(b1[3])
      : "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186",
        "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197",
        "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208",
        "v209", "v210", "v211", "v212", "v213", "v214", "v215", "scc", "memory");
}

__device__ __forceinline__ double shx(double v, int m) { return __shfl_xor(v, m, 64); }

// the quad form of nmc_ll_rows_lds<FamLinreg<2>>: same rows into the same accumulators in
// the same order (row r of the tile -> a[r & 3] of its chain), tail rows into a[0]
__device__ __forceinline__ double quad_tile(const double* rows, int n, double b0, double b1) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  double c0[4], c1[4], a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // chain of lane ^ 16k
    c0[k] = k ? shx(b0, 16 * k) : b0;
    c1[k] = k ? shx(b1, 16 * k) : b1;
  }
  // an even number of 16-row granules; nmc_ll_rows_lds covers nb2 = (n / 8) & ~1 8-row
  // blocks, the rows in between (if any) go through the per-lane loop below
  const int nq = (n / 16) & ~1;
  if (nq > 0) quad_rows(rows + (size_t)g * 2, nq, c0, c1, a);
  // a[k] = this lane group's accumulator a[g] of chain lane ^ 16k -> chain-own a[0..3]
  double own[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const double v = d ? shx(a[d], 16 * d) : a[d];   // lane ^ 16d's slot d = a[g ^ d] of mine
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j == d) own[j] = v;
  }
  double acc4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {   // a[j] = own[j ^ g]
    double v = own[0];
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if ((j ^ g) == d) v = own[d];
    acc4[j] = v;
  }
  // rows [16 nq, n): whole 8-row blocks (pairs) of the broadcast loop, then the tail, in order
  const int nb2 = (n / 8) & ~1;
  for (int r = 16 * nq; r < nb2 * 8; ++r) {
    double e = b0 - rows[2 * r + 1];
    e = fma(rows[2 * r], b1, e);
    acc4[r & 3] = fma(e, e, acc4[r & 3]);
  }
  for (int r = nb2 * 8; r < n; ++r) {
    double e = b0 - rows[2 * r + 1];
    e = fma(rows[2 * r], b1, e);
    acc4[0] = fma(e, e, acc4[0]);
  }
  return (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
}

template <int V>
__global__ void __launch_bounds__(512) kbench(const double* obs, int npass, double* out,
                                              unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double lrows[N * 2 + 128];
  __shared__ double part[NSL * 64];
  __shared__ unsigned tc[2];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < N * 2; i += blockDim.x) lrows[i] = obs[i];
  if (threadIdx.x < 2) tc[threadIdx.x] = 0;
  FamLinreg<2> fam;
  fam.intercept = 1;
  fam.sigma_known = 1.0;
  fam.log_sigma_known = 0.0;
  fam.inv_s2_known = 1.0;
  const nmc_tiling TI = nmc_tiles(N, TILE);
  double th[3] = {0.3 + 1e-3 * lane, 1.9 - 1e-3 * blockIdx.x, 0.0};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double chk = 0.0;
  for (int ps = 0; ps < npass; ++ps) {
    const int sp = ps & 1;
    th[0] += 1e-9;
    const FamLinreg<2>::Reg reg = fam.prepare(th);
    FamLinreg<2>::Reg preg = reg;
    {
      double pth[3];
      for (int q = 0; q < 3; ++q) {
        const nmc_pair2 e = nmc_halves(th[q]);
        pth[q] = lane >= 32 ? e.lo : e.hi;
      }
      preg = fam.prepare(pth);
    }
    auto grab = [&]() -> unsigned {
      unsigned k = 0;
      if (lane == 0) k = __hip_atomic_fetch_add(tc + sp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return k;
    };
    int k = (int)__builtin_amdgcn_readlane(grab(), 0);
    while (k < TI.nt) {
      const unsigned kn = grab();
      const int ra = TI.start(k), rn = TI.len(k);
      double s;
      if constexpr (V == 0) {   // VALU only
        double a[4] = {0, 0, 0, 0};
        double x = 0.5 + 1e-3 * k, y = 0.25;
        for (int r = 0; r < rn; r += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            double e = reg.b0 - y;
            e = fma(x, reg.b[0], e);
            a[u] = fma(e, e, a[u]);
            x += 1e-12;
          }
        }
        s = (a[0] + a[1]) + (a[2] + a[3]);
      } else if constexpr (V == 1) {
        double acc[1];
        nmc_ll_rows_lds<FamLinreg<2>, true>(fam, reg, lrows + (size_t)ra * 2, rn, acc, &preg);
        s = acc[0];
      } else if constexpr (V == 2) {
        double acc[1];
        nmc_ll_rows_lds<FamLinreg<2>, false>(fam, reg, lrows + (size_t)ra * 2, rn, acc);
        s = acc[0];
      } else {
        s = quad_tile(lrows + (size_t)ra * 2, rn, reg.b0, reg.b[0]);
      }
      part[k * 64 + lane] = s;
      k = (int)__builtin_amdgcn_readlane(kn, 0);
    }
    __syncthreads();
    if (w == 0) {
      if (lane == 0) tc[sp] = 0;
      chk += nmc_sum_slots(part + lane);
      if (ps == 0 && out)
        for (int t = 0; t < TI.nt; ++t) out[((size_t)blockIdx.x * NSL + t) * 64 + lane] = part[t * 64 + lane];
    }
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  if (w == 0 && chk == 12345.678) out[lane] = chk;   // keep the work
}

int main() {
  double* h = (double*)malloc(N * 2 * 8);
  srand(3);
  for (int i = 0; i < N; ++i) {
    h[2 * i] = (rand() / (double)RAND_MAX) * 2 - 1;
    h[2 * i + 1] = (rand() / (double)RAND_MAX) * 4 - 2;
  }
  double *obs, *outB, *outQ;
  unsigned long long* cyc;
  hipMalloc(&obs, N * 2 * 8);
  hipMalloc(&outB, 256 * NSL * 64 * 8);
  hipMalloc(&outQ, 256 * NSL * 64 * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(obs, h, N * 2 * 8, hipMemcpyHostToDevice);
  const int npass = 400;
  const char* names[4] = {"V", "P", "B", "Q"};
  for (int W : {4, 8}) {
    for (int v = 0; v < 4; ++v) {
      auto kern = v == 0 ? kbench<0> : v == 1 ? kbench<1> : v == 2 ? kbench<2> : kbench<3>;
      double* o = v == 2 ? outB : v == 3 ? outQ : nullptr;
      hipLaunchKernelGGL(kern, dim3(256), dim3(64 * W), 0, 0, obs, 10, o, cyc);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(256), dim3(64 * W), 0, 0, obs, npass, o, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("{\"variant\": \"%s\", \"waves\": %d, \"cycles_per_pass\": %.0f, \"us_per_pass\": %.3f, "
             "\"clock_ghz\": %.3f}\n",
             names[v], W, (double)c / npass, ms * 1e3 / npass, (double)c / (ms * 1e6));
    }
  }
  // bit identity of the quad tiles against the broadcast tiles (pass 0)
  double* hb = (double*)malloc(256 * NSL * 64 * 8);
  double* hq = (double*)malloc(256 * NSL * 64 * 8);
  hipMemcpy(hb, outB, 256 * NSL * 64 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hq, outQ, 256 * NSL * 64 * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (size_t i = 0; i < (size_t)256 * NSL * 64; ++i)
    if (memcmp(&hb[i], &hq[i], 8) != 0) ++bad;
  printf("{\"quad_vs_broadcast_mismatches\": %d}\n", bad);
  return bad != 0;
}
