// fp64issue.hip -- fp64 VALU issue rate on gfx950 by waves per SIMD (diagnostics, not
// shipped).  256 workgroups (one per CU) of 64 x 4 x WPS threads; every wave runs REPS trips
// of an asm body; each wave stamps s_memtime at its start and end.  Reported per variant and
// WPS: shader cycles per fp64 wave-instruction per SIMD over workgroup 0's span (first start
// to last end of its waves), and the event-timed chip rate.
//   indep16 / indep4 : independent v_fma_f64 chains (16 / 4 per wave)
//   dep1             : one dependent chain (latency)
//   pb_regs          : the shipped paired linreg body (24 fp64 per 8-row block), registers only
//   pb_lds           : the shipped paired loop with its ds_read_b128 row reads
//   pb_lds3          : the same with three register sets, the reads two blocks ahead
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

#define FC(r) "v_fma_f64 v[" #r ":" #r "+1], v[" #r ":" #r "+1], %[m], %[a]\n"
#define FC4 FC(64) FC(66) FC(68) FC(70)
#define FC16 FC4 FC(72) FC(74) FC(76) FC(78) FC(80) FC(82) FC(84) FC(86) FC(88) FC(90) FC(92) FC(94)
#define CL64_111                                                                              \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76",   \
      "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88",      \
      "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100",     \
      "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111"
#define CL112_135                                                                              \
  "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",      \
      "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133",  \
      "v134", "v135"

enum { V_INDEP16 = 0, V_INDEP4, V_DEP1, V_PB_REGS, V_PB_LDS, V_PB_LDS3, NV };
static const char* vname[NV] = {"indep16", "indep4", "dep1", "pb_regs", "pb_lds", "pb_lds3"};
// fp64 wave-instructions per loop trip (pb_lds / pb_lds3: per two 8-row blocks)
static const int vper[NV] = {48, 48, 48, 48, 48, 48};

template <int V, int LB>
__global__ void __launch_bounds__(LB) k(const double* obs, int reps, unsigned long long* ts,
                                        double* out) {
  __shared__ __attribute__((aligned(16))) double lrows[2048 + 512];
  if (V == V_PB_LDS || V == V_PB_LDS3) {
    for (int i = threadIdx.x; i < 2048 + 512; i += blockDim.x) lrows[i] = obs[i & 2047];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  double u0 = 0, u1 = 0, w0 = 0, w1 = 0;
  const double b0 = 0.1 + lane * 1e-3, b1 = 1.9, c0 = 0.2, c1 = 2.1;
  const double m = 1.0000001, a = 1e-9;
  int n = reps;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (V == V_INDEP16) {
    asm volatile("L_a_%=:\n" FC16 FC16 FC16
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L_a_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CL64_111, "scc");
  } else if constexpr (V == V_INDEP4) {
    asm volatile("L_b_%=:\n" FC4 FC4 FC4 FC4 FC4 FC4 FC4 FC4 FC4 FC4 FC4 FC4
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L_b_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CL64_111, "scc");
  } else if constexpr (V == V_DEP1) {
#define D8 FC(64) FC(64) FC(64) FC(64) FC(64) FC(64) FC(64) FC(64)
    asm volatile("L_c_%=:\n" D8 D8 D8 D8 D8 D8
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L_c_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CL64_111, "scc");
  } else if constexpr (V == V_PB_REGS) {
    asm volatile("L_d_%=:\n" NMC_PB(64, 80) NMC_PB(88, 104)
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L_d_%=\n"
                 : [n] "+s"(n), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0), [w1] "+v"(w1)
                 : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
                 : CL64_111, "scc");
  } else if constexpr (V == V_PB_LDS3) {
    // three register sets, the reads of blocks i+1 and i+2 in flight while block i is
    // consumed; 132 blocks per trip (64 two-block trips' worth of rows, counted as 66)
    const int h = (threadIdx.x >> 5) & 1;
    const unsigned base = (unsigned)(uintptr_t)(nmc_lds_cptr)(lrows + 2 * h);
    for (int r = 0; r < reps; r += 66) {
      unsigned addr = base;
      int cnt = 132;
      asm volatile(
          NMC_P4(64, 0)
          NMC_P4(88, 128)
          "L_f_%=:\n"
          NMC_P4(112, 256)
          "s_waitcnt lgkmcnt(8)\n"
          NMC_PB(64, 80)
          NMC_P4(64, 384)
          "s_waitcnt lgkmcnt(8)\n"
          NMC_PB(88, 104)
          NMC_P4(88, 512)
          "s_waitcnt lgkmcnt(8)\n"
          NMC_PB(112, 128)
          "v_add_u32 %[addr], 0x180, %[addr]\n"
          "s_sub_u32 %[cnt], %[cnt], 3\n"
          "s_cmp_gt_i32 %[cnt], 0\n"
          "s_cbranch_scc1 L_f_%=\n"
          "s_waitcnt lgkmcnt(0)\n"
          : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0),
            [w1] "+v"(w1)
          : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
          : CL64_111, CL112_135, "scc", "memory");
    }
  } else {
    // the shipped loop's structure (two register sets, next block's reads in flight), over
    // 128 blocks of rows per trip, the address wrapping back each trip
    const int h = (threadIdx.x >> 5) & 1;
    const unsigned base = (unsigned)(uintptr_t)(nmc_lds_cptr)(lrows + 2 * h);
    for (int r = 0; r < reps; r += 64) {
      unsigned addr = base;
      int cnt = 128;
      asm volatile(
          NMC_P4(64, 0)
          "L_e_%=:\n"
          NMC_P4(88, 128)
          "s_waitcnt lgkmcnt(4)\n"
          NMC_PB(64, 80)
          "v_add_u32 %[addr], 0x100, %[addr]\n"
          "s_sub_u32 %[cnt], %[cnt], 2\n"
          "s_cmp_gt_i32 %[cnt], 0\n"
          "s_cbranch_scc0 L_el_%=\n"
          NMC_P4(64, 0)
          "s_waitcnt lgkmcnt(4)\n"
          NMC_PB(88, 104)
          "s_branch L_e_%=\n"
          "L_el_%=:\n"
          "s_waitcnt lgkmcnt(0)\n"
          NMC_PB(88, 104)
          : [addr] "+v"(addr), [cnt] "+s"(cnt), [u0] "+v"(u0), [u1] "+v"(u1), [w0] "+v"(w0),
            [w1] "+v"(w1)
          : [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1)
          : CL64_111, "scc", "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int wg = threadIdx.x >> 6;
  if (lane == 0) {
    ts[((size_t)blockIdx.x * 16 + wg) * 2] = t0;
    ts[((size_t)blockIdx.x * 16 + wg) * 2 + 1] = t1;
  }
  if (u0 + u1 + w0 + w1 == 1.2345) out[threadIdx.x] = u0;
}

template <int V>
static void run(const double* obs, unsigned long long* ts, double* out) {
  // pb_lds: 128 blocks (64 trips) per rep; pb_lds3: 132 blocks (66 trips)
  const int reps = V == V_PB_LDS ? 64 * 40 : V == V_PB_LDS3 ? 66 * 40 : 4000;
  for (int wps = 1; wps <= 4; ++wps) {
    auto kern = wps == 1 ? k<V, 256> : wps == 2 ? k<V, 512> : wps == 3 ? k<V, 768> : k<V, 1024>;
    hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, obs,
                       V == V_PB_LDS ? 64 : V == V_PB_LDS3 ? 66 : 10, ts, out);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, obs, reps, ts, out);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) {
      printf("{\"variant\": \"%s\", \"wps\": %d, \"error\": \"%s\"}\n", vname[V], wps,
             hipGetErrorString(hipGetLastError()));
      return;
    }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(256 * 16 * 2);
    (void)hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
    const int nw = 4 * wps;
    unsigned long long lo = ~0ull, hi = 0, first_end = ~0ull;
    for (int w = 0; w < nw; ++w) {
      lo = std::min(lo, h[w * 2]);
      hi = std::max(hi, h[w * 2 + 1]);
      first_end = std::min(first_end, h[w * 2 + 1]);
    }
    // trips per wave: pb_lds runs 64 trips (128 blocks) per rep/64
    const double trips = V == V_PB_LDS ? (double)reps : (double)reps;
    const double per_simd = trips * vper[V] * wps;   // fp64 wave-instructions per SIMD
    const double span = (double)(hi - lo);
    const double chip = (double)256 * 4 * per_simd * 64 / (ms * 1e-3);   // lane-ops/s
    printf("{\"variant\": \"%s\", \"wps\": %d, \"cyc_per_fp64_per_simd\": %.3f, "
           "\"first_wave_cyc_per_instr\": %.3f, \"ms\": %.4f, \"clock_ghz\": %.3f, "
           "\"chip_T_lane_ops\": %.2f}\n",
           vname[V], wps, span / per_simd, (double)(first_end - lo) / (trips * vper[V]), ms,
           span / (ms * 1e6), chip / 1e12);
  }
}

int main() {
  std::vector<double> hobs(2048);
  for (int i = 0; i < 2048; ++i) hobs[i] = (i % 7) * 0.1;
  double *obs, *out;
  unsigned long long* ts;
  (void)hipMalloc(&obs, 2048 * 8);
  (void)hipMalloc(&out, 1024 * 8);
  (void)hipMalloc(&ts, 256 * 16 * 2 * 8);
  (void)hipMemcpy(obs, hobs.data(), 2048 * 8, hipMemcpyHostToDevice);
  run<V_INDEP16>(obs, ts, out);
  run<V_INDEP4>(obs, ts, out);
  run<V_DEP1>(obs, ts, out);
  run<V_PB_REGS>(obs, ts, out);
  run<V_PB_LDS>(obs, ts, out);
  run<V_PB_LDS3>(obs, ts, out);
  return 0;
}
