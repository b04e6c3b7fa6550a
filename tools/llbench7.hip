// llbench7.hip -- steady-state issue rate of the paired row loop with no step structure
// (diagnostics, not shipped): every wave of W runs the shipped asm loop over the same LDS
// rows REPS times back to back, no barriers, no tiles.  cycles per fp64 VALU instruction
// per SIMD = cycles / (24 per 8-row block x blocks x REPS x waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

template <int LB>
__global__ void __launch_bounds__(LB) k(const double* obs, int reps, unsigned long long* cyc,
                                        double* out) {
  __shared__ __attribute__((aligned(16))) double lrows[1024 * 2 + 64];
  for (int i = threadIdx.x; i < 1024 * 2 + 64; i += blockDim.x) lrows[i] = i < 2048 ? obs[i] : 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  double u0 = 0, u1 = 0, w0 = 0, w1 = 0;
  const double b0 = 0.1 + lane * 1e-3, b1 = 1.9, c0 = 0.2, c1 = 2.1;
  const int h = (threadIdx.x >> 5) & 1;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
    nmc_rows_lds_linreg2_paired(lrows + 2 * h, 128, b0, b1, c0, c1, u0, u1, w0, w1);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  if (u0 + u1 + w0 + w1 == 1.2345) out[threadIdx.x] = u0;
}

int main() {
  double* h = (double*)malloc(2048 * 8);
  for (int i = 0; i < 2048; ++i) h[i] = (i % 7) * 0.1;
  double *obs, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&obs, 2048 * 8);
  (void)hipMalloc(&out, 1024 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(obs, h, 2048 * 8, hipMemcpyHostToDevice);
  const int reps = 100;
  for (int W : {4, 8}) {
    auto kern = W == 4 ? k<256> : k<512>;
    hipLaunchKernelGGL(kern, dim3(256), dim3(64 * W), 0, 0, obs, 2, cyc, out);
    hipLaunchKernelGGL(kern, dim3(256), dim3(64 * W), 0, 0, obs, reps, cyc, out);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double dp = 24.0 * 128 * reps * (W / 4);   // per SIMD
    printf("{\"waves\": %d, \"cycles\": %llu, \"cycles_per_dp_per_simd\": %.3f}\n", W, c, c / dp);
  }
  return 0;
}
