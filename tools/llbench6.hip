// llbench6.hip -- where the paired row loop loses its VALU issue rate (diagnostics, not
// shipped).  Same harness as llbench5 (one (64-chain block, group) per workgroup, W waves
// taking tiles of a 1000-row {x, y} group, a barrier per pass), with:
//   PR  the shipped paired asm body with its LDS reads removed (registers only): the
//       instruction schedule's own VALU efficiency
//   P   the shipped paired loop (nmc_ll_rows_lds<FamLinreg<2>, true>)
//   P16 the paired loop on 16-row super-blocks, one super-block in flight (twice the
//       shipped prefetch distance), the two 8-row halves' independent residual work
//       interleaved ahead of their accumulations
// at tile targets of 64, 128 and 256 rows (16, 8 and 4 tiles per pass).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

constexpr int N = 1000, NSL = 16;

// registers-only form of nmc_rows_lds_linreg2_paired (same VALU instructions, no reads)
__device__ __forceinline__ void paired_regs(int nb, double b0, double b1, double c0, double c1,
                                            double& u0, double& u1, double& w0, double& w1) {
  int cnt = nb;
  asm volatile(
      "L_pr_%=:\n"
      NMC_PB(208, 224)
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      NMC_PB(232, 248)
      "s_cbranch_scc1 L_pr_%=\n"
      : [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0), [w1] "+v"(w1)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218",
        "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229",
        "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240",
        "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251",
        "v252", "v253", "v254", "v255", "scc", "memory");
}

// the shipped paired loop with its fixed registers moved to v[120:167] (so a kernel can stay
// within 168 VGPRs: three waves per SIMD)
__device__ __forceinline__ void paired_low(const double* p, int nb, double b0, double b1,
                                           double c0, double c1, double& u0, double& u1,
                                           double& w0, double& w1) {
  unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)p;
  int cnt = nb;
  asm volatile(
      NMC_P4(120, 0)
      "L_pl_%=:\n"
      NMC_P4(144, 128)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_PB(120, 136)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_pllast_%=\n"
      NMC_P4(120, 0)
      "s_waitcnt lgkmcnt(4)\n"
      NMC_PB(144, 160)
      "s_branch L_pl_%=\n"
      "L_pllast_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      NMC_PB(144, 160)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0),
        [w1] "+v"(w1)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130",
        "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141",
        "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152",
        "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163",
        "v164", "v165", "v166", "v167", "scc", "memory");
}

// 16-row super-block: rows of two 8-row blocks in v[b : b+31], temps v[t : t+15]; the
// residual work of both halves first (independent), then the accumulations in row order
#define S_RES(b, t)                                                                           \
  NMC_PDX(b, t, 0, 0) NMC_PDX(b, t, 4, 2) NMC_PDX(b, t, 8, 4) NMC_PDX(b, t, 12, 6)             \
  NMC_PDX(b+16, t+8, 0, 0) NMC_PDX(b+16, t+8, 4, 2) NMC_PDX(b+16, t+8, 8, 4)                  \
  NMC_PDX(b+16, t+8, 12, 6)                                                                   \
  NMC_PDO(b, 0) NMC_PDO(b, 4) NMC_PDO(b, 8) NMC_PDO(b, 12)                                     \
  NMC_PDO(b+16, 0) NMC_PDO(b+16, 4) NMC_PDO(b+16, 8) NMC_PDO(b+16, 12)                         \
  NMC_PEO(b, 0) NMC_PEO(b, 4) NMC_PEO(b, 8) NMC_PEO(b, 12)                                     \
  NMC_PEO(b+16, 0) NMC_PEO(b+16, 4) NMC_PEO(b+16, 8) NMC_PEO(b+16, 12)                         \
  NMC_PEX(b, t, 0, 0) NMC_PEX(b, t, 4, 2) NMC_PEX(b, t, 8, 4) NMC_PEX(b, t, 12, 6)             \
  NMC_PEX(b+16, t+8, 0, 0) NMC_PEX(b+16, t+8, 4, 2) NMC_PEX(b+16, t+8, 8, 4)                  \
  NMC_PEX(b+16, t+8, 12, 6)
#define S_ACC(b, t)                                                                           \
  NMC_PSO(b, 0, u0) NMC_PSX(t, 0, w0) NMC_PSO(b, 4, u1) NMC_PSX(t, 2, w1)                     \
  NMC_PSO(b, 8, u0) NMC_PSX(t, 4, w0) NMC_PSO(b, 12, u1) NMC_PSX(t, 6, w1)                    \
  NMC_PSO(b+16, 0, u0) NMC_PSX(t+8, 0, w0) NMC_PSO(b+16, 4, u1) NMC_PSX(t+8, 2, w1)           \
  NMC_PSO(b+16, 8, u0) NMC_PSX(t+8, 4, w0) NMC_PSO(b+16, 12, u1) NMC_PSX(t+8, 6, w1)
#define S_LD(b, off) NMC_P4(b, off) NMC_P4(b+16, off+128)
#define S_CLOB                                                                                  \
  "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170",      \
      "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181",  \
      "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192",  \
      "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203",  \
      "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214",  \
      "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225",  \
      "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236",  \
      "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247",  \
      "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255", "scc", "memory"
// one super-block (nsb odd: the first one alone)
__device__ __forceinline__ void p16_one(unsigned& addr, double b0, double b1, double c0, double c1,
                                        double& u0, double& u1, double& w0, double& w1) {
  asm volatile(
      S_LD(160, 0)
      "s_waitcnt lgkmcnt(0)\n"
      S_RES(160, 224) S_ACC(160, 224)
      "v_add_u32 %[addr], 0x100, %[addr]\n"
      : [addr] "+v"(addr), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0), [w1] "+v"(w1)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : S_CLOB);
}
// an even number nsb >= 2 of super-blocks, one in flight
__device__ __forceinline__ void p16_loop(unsigned& addr, int nsb, double b0, double b1, double c0,
                                         double c1, double& u0, double& u1, double& w0,
                                         double& w1) {
  int cnt = nsb;
  asm volatile(
      S_LD(160, 0)
      "L_s16_%=:\n"
      S_LD(192, 256)
      "s_waitcnt lgkmcnt(8)\n"
      S_RES(160, 224) S_ACC(160, 224)
      "v_add_u32 %[addr], 0x200, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc0 L_s16last_%=\n"
      S_LD(160, 0)
      "s_waitcnt lgkmcnt(8)\n"
      S_RES(192, 240) S_ACC(192, 240)
      "s_branch L_s16_%=\n"
      "L_s16last_%=:\n"
      "s_waitcnt lgkmcnt(0)\n"
      S_RES(192, 240) S_ACC(192, 240)
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0),
        [w1] "+v"(w1)
      : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
      : S_CLOB);
}

// nmc_ll_rows_lds<FamLinreg<2>, true> with the 16-row super-block body (same sums)
__device__ __forceinline__ double p16_tile(const double* p, int n, const FamLinreg<2>::Reg& reg,
                                           const FamLinreg<2>::Reg& preg, int variant) {
  const int h = (threadIdx.x >> 5) & 1;
  const double* ph = p + (size_t)h * 2;
  double u0 = 0, u1 = 0, w0 = 0, w1 = 0;
  const int nb2 = (n / 8) & ~1;
  if (variant == 2) {   // registers only
    if (nb2 > 0) paired_regs(nb2, reg.b0, reg.b[0], preg.b0, preg.b[0], u0, u1, w0, w1);
  } else if (variant == 3) {   // the shipped loop on low registers
    if (nb2 > 0) paired_low(ph, nb2, reg.b0, reg.b[0], preg.b0, preg.b[0], u0, u1, w0, w1);
  } else if (nb2 > 0) {
    unsigned addr = (unsigned)(uintptr_t)(nmc_lds_cptr)ph;
    int nsb = nb2 / 2;
    if (nsb & 1) {
      p16_one(addr, reg.b0, reg.b[0], preg.b0, preg.b[0], u0, u1, w0, w1);
      --nsb;
    }
    if (nsb > 0) p16_loop(addr, nsb, reg.b0, reg.b[0], preg.b0, preg.b[0], u0, u1, w0, w1);
  }
  double a[4];
  const nmc_pair2 e = nmc_halves(w0), o = nmc_halves(w1);
  const double p0 = h ? e.lo : e.hi, p1 = h ? o.lo : o.hi;
  a[0] = h ? p0 : u0;
  a[1] = h ? u0 : p0;
  a[2] = h ? p1 : u1;
  a[3] = h ? u1 : p1;
  for (int r = nb2 * 8; r < n; ++r) {
    double x = p[2 * r], y = p[2 * r + 1];
    double ee = reg.b0 - y;
    ee = fma(x, reg.b[0], ee);
    a[0] = fma(ee, ee, a[0]);
  }
  return (a[0] + a[1]) + (a[2] + a[3]);
}

__device__ unsigned long long g_tl[16 * 4 + 16 * 2];   // pass-5 timeline of workgroup 0
template <int V, int LB>
__global__ void __launch_bounds__(LB) kbench(const double* obs, int npass, int tile, double* out,
                                             unsigned long long* cyc, int idle) {
  __shared__ __attribute__((aligned(16))) double lrows[N * 2 + 256];
  __shared__ double part[NSL * 64];
  __shared__ unsigned tc[2];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < N * 2 + 256; i += blockDim.x) lrows[i] = i < N * 2 ? obs[i] : 0.0;
  if (threadIdx.x < 2) tc[threadIdx.x] = 0;
  FamLinreg<2> fam;
  fam.intercept = 1;
  fam.sigma_known = 1.0;
  fam.log_sigma_known = 0.0;
  fam.inv_s2_known = 1.0;
  const nmc_tiling TI = nmc_tiles(N, tile);
  for (int k = TI.nt + w; k < NSL; k += blockDim.x >> 6) part[k * 64 + lane] = -0.0;
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
    int k = w < idle ? TI.nt : (int)__builtin_amdgcn_readlane(grab(), 0);
    while (k < TI.nt) {
      const unsigned kn = grab();
      const int ra = TI.start(k), rn = TI.len(k);
      if (ps == 5 && blockIdx.x == 0 && lane == 0) {
        g_tl[k * 4 + 0] = __builtin_amdgcn_s_memtime();
        g_tl[k * 4 + 2] = (unsigned long long)w;
      }
      double s;
      if constexpr (V == 0) {
        double acc[1];
        nmc_ll_rows_lds<FamLinreg<2>, true>(fam, reg, lrows + (size_t)ra * 2, rn, acc, &preg);
        s = acc[0];
      } else {
        s = p16_tile(lrows + (size_t)ra * 2, rn, reg, preg, V);
      }
      part[k * 64 + lane] = s;
      if (ps == 5 && blockIdx.x == 0 && lane == 0) g_tl[k * 4 + 1] = __builtin_amdgcn_s_memtime();
      k = (int)__builtin_amdgcn_readlane(kn, 0);
    }
    if (ps == 5 && blockIdx.x == 0 && lane == 0) g_tl[64 + w * 2] = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (ps == 5 && blockIdx.x == 0 && lane == 0) g_tl[64 + w * 2 + 1] = __builtin_amdgcn_s_memtime();
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
  if (w == 0 && chk == 12345.678) out[lane] = chk;
}

int main() {
  double* h = (double*)malloc(N * 2 * 8);
  srand(3);
  for (int i = 0; i < N; ++i) {
    h[2 * i] = (rand() / (double)RAND_MAX) * 2 - 1;
    h[2 * i + 1] = (rand() / (double)RAND_MAX) * 4 - 2;
  }
  double *obs, *outP, *outS;
  unsigned long long* cyc;
  (void)hipMalloc(&obs, N * 2 * 8);
  (void)hipMalloc(&outP, 256 * NSL * 64 * 8);
  (void)hipMalloc(&outS, 256 * NSL * 64 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(obs, h, N * 2 * 8, hipMemcpyHostToDevice);
  const int npass = 400;
  int bad = 0;
  struct Cfg { const char* name; const void* k; int W; int idle; };
  const Cfg cfgs[] = {
      {"P", (const void*)kbench<0, 512>, 8, 0},   {"P", (const void*)kbench<0, 512>, 8, 2},
      {"PL", (const void*)kbench<3, 512>, 8, 0},  {"PL", (const void*)kbench<3, 512>, 8, 2},
      {"PL", (const void*)kbench<3, 768>, 12, 0}, {"PL", (const void*)kbench<3, 768>, 12, 2},
      {"PR", (const void*)kbench<2, 512>, 8, 0},  {"P16", (const void*)kbench<1, 512>, 8, 0}};
  for (int tile : {64, 128}) {
    for (const Cfg& cf : cfgs) {
      double* o = nullptr;
      int np = 10;
      void* a1[] = {&obs, &np, &tile, &o, &cyc, (void*)&cf.idle};
      (void)hipLaunchKernel(cf.k, dim3(256), dim3(64 * cf.W), a1, 0, 0);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      int npp = npass;
      void* a2[] = {&obs, &npp, &tile, &o, &cyc, (void*)&cf.idle};
      hipError_t err = hipLaunchKernel(cf.k, dim3(256), dim3(64 * cf.W), a2, 0, 0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c = 0;
      (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      unsigned long long tl[96];
      (void)hipMemcpyFromSymbol(tl, HIP_SYMBOL(g_tl), sizeof(tl));
      unsigned long long t0 = ~0ull;
      for (int q = 0; q < 16; ++q) if (tl[q * 4] && tl[q * 4] < t0) t0 = tl[q * 4];
      char buf[4096];
      int n = 0;
      for (int q = 0; q < 16; ++q)
        if (tl[q * 4 + 1]) n += snprintf(buf + n, sizeof(buf) - n, "%s[%d,%lld,%lld]", n ? "," : "",
                                          (int)tl[q * 4 + 2], (long long)(tl[q * 4] - t0),
                                          (long long)(tl[q * 4 + 1] - t0));
      n += snprintf(buf + n, sizeof(buf) - n, "], \"barrier_arrive\": [");
      for (int q = 0; q < cf.W; ++q)
        n += snprintf(buf + n, sizeof(buf) - n, "%s%lld", q ? "," : "", (long long)(tl[64 + q * 2] - t0));
      printf("{\"variant\": \"%s\", \"waves\": %d, \"idle_waves\": %d, \"tile\": %d, "
             "\"cycles_per_pass\": %.0f, \"us_per_pass\": %.3f, \"launch\": \"%s\", "
             "\"tiles_wave_start_end\": [%s]}\n",
             cf.name, cf.W, cf.idle, tile, (double)c / npass, ms * 1e3 / npass,
             hipGetErrorString(err), buf);
    }
  }
  {   // bit identity: PL and P16 tiles against the shipped loop (pass 0)
    double* hp = (double*)malloc(256 * NSL * 64 * 8);
    double* hs = (double*)malloc(256 * NSL * 64 * 8);
    for (int v : {1, 3}) {
      int np = 1, tile = 64, idle = 0;
      void* a0[] = {&obs, &np, &tile, &outP, &cyc, &idle};
      (void)hipLaunchKernel((const void*)kbench<0, 512>, dim3(256), dim3(512), a0, 0, 0);
      void* a1[] = {&obs, &np, &tile, &outS, &cyc, &idle};
      (void)hipLaunchKernel(v == 1 ? (const void*)kbench<1, 512> : (const void*)kbench<3, 512>,
                            dim3(256), dim3(512), a1, 0, 0);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(hp, outP, 256 * NSL * 64 * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(hs, outS, 256 * NSL * 64 * 8, hipMemcpyDeviceToHost);
      for (size_t i = 0; i < (size_t)256 * NSL * 64; ++i)
        if (memcmp(&hp[i], &hs[i], 8) != 0) ++bad;
    }
  }
  printf("{\"p16_vs_paired_mismatches\": %d}\n", bad);
  return bad != 0;
}
