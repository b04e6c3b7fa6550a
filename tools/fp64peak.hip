// fp64peak.hip -- measured fp64 VALU throughput on this GPU (diagnostics):
// independent v_fma_f64 / v_add_f64 chains, 256 x 1024-thread workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ void __launch_bounds__(1024) k(double* out, int iters, double a, double b) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) x[i] = fma(x[i], a, b);
      else x[i] = x[i] + b;
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 1024 * 8 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int op = 0; op < 2; ++op)
    for (int wg : {256, 512, 1024}) {
      auto kern = op == 0 ? k<0> : k<1>;
      hipLaunchKernelGGL(kern, dim3(wg), dim3(1024), 0, 0, out, 100, 1.0000001, 1e-9);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(wg), dim3(1024), 0, 0, out, iters, 1.0000001, 1e-9);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)wg * 1024 * iters * 8;
      printf("{\"op\": \"%s\", \"workgroups\": %d, \"ms\": %.3f, \"Gops_per_s\": %.1f, "
             "\"lane_ops_per_clk_per_CU_at_2.4GHz\": %.2f}\n",
             op == 0 ? "v_fma_f64" : "v_add_f64", wg, ms, ops / ms / 1e6,
             ops / (ms * 1e-3) / 256 / 2.4e9);
    }
  return 0;
}
