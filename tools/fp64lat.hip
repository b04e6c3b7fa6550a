// fp64lat.hip -- fp64 VALU issue and dependent latency on gfx950 (diagnostics, not shipped).
// 256 workgroups (one per CU) of 64 x WPS x 4 threads (WPS waves per SIMD); each wave runs
// K independent v_fma_f64 accumulation chains written in asm (no compiler reordering):
// cycles per fma per SIMD = how many chains a wave (or two) needs to fill the pipe.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define F(r) "v_fma_f64 v[" #r ":" #r "+1], v[" #r ":" #r "+1], %[m], %[a]\n"
#define F1 F(128)
#define F2 F(128) F(130)
#define F4 F2 F(132) F(134)
#define F8 F4 F(136) F(138) F(140) F(142)
#define F16 F8 F(144) F(146) F(148) F(150) F(152) F(154) F(156) F(158)
#define CLOB                                                                                  \
  "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138",     \
      "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", \
      "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "scc"

template <int K>
__global__ void __launch_bounds__(1024) k(int iters, double m, double a, unsigned long long* cyc) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int n = iters;
  // K chains, each instruction group of K repeated until 16 instructions per loop trip
  if constexpr (K == 0)   // 1 chain: every fma depends on the previous one
    asm volatile("L0_%=:\n" F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L0_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CLOB);
  if constexpr (K == 2)
    asm volatile("L2_%=:\n" F2 F2 F2 F2 F2 F2 F2 F2
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L2_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CLOB);
  if constexpr (K == 4)
    asm volatile("L4_%=:\n" F4 F4 F4 F4
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L4_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CLOB);
  if constexpr (K == 8)
    asm volatile("L8_%=:\n" F8 F8
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L8_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CLOB);
  if constexpr (K == 16)
    asm volatile("L16_%=:\n" F16
                 "s_sub_u32 %[n], %[n], 1\ns_cmp_gt_i32 %[n], 0\ns_cbranch_scc1 L16_%=\n"
                 : [n] "+s"(n) : [m] "v"(m), [a] "v"(a) : CLOB);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  unsigned long long* cyc;
  (void)hipMalloc(&cyc, 8);
  const int iters = 4000;
  for (int wps : {1, 2, 3, 4}) {
    for (int K : {0, 2, 4, 8, 16}) {
      auto kern = K == 0 ? k<0> : K == 2 ? k<2> : K == 4 ? k<4> : K == 8 ? k<8> : k<16>;
      hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, 10, 1.0, 0.0, cyc);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, iters, 1.0, 0.0, cyc);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c = 0;
      (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const double per_fma_simd = (double)c / (iters * 16.0 * wps);
      printf("{\"waves_per_simd\": %d, \"chains\": %d, \"cycles_per_fma_per_simd\": %.2f, "
             "\"clock_ghz\": %.3f}\n",
             wps, K == 0 ? 1 : K, per_fma_simd, (double)c / (ms * 1e6));
    }
  }
  return 0;
}
