// llbench2.hip -- the step kernel's likelihood phase in isolation (diagnostics).
//
// 256 workgroups x 16 waves; 15 waves split one group's 1000 (x, y) rows, the same
// rows every pass; NPASS passes per launch with a barrier between passes (like the
// per-parameter steps of nmc_k_run).  Variants of the row loop:
//   0  LDS rows, nmc_ll_rows_lds (4-row blocks, next block prefetched)
//   1  LDS rows, plain 8-row blocks (no prefetch)
//   2  LDS rows, 8-row blocks, next block prefetched
//   3  global rows, scalar loads (nmc_ll_rows, 8-row blocks)
//   4  LDS rows, 16-row blocks, two block loads in flight
// Prints cycles per pass (s_memtime, workgroup 0) and us per pass (events).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

template <int R, bool PF>
__device__ __forceinline__ double rows_lds_r(const double* __restrict__ p, int n, double b0, double b1) {
  double a[4] = {0, 0, 0, 0};
  const int nb = n / R;
  if (PF) {
    double cur[2 * R];
#pragma unroll
    for (int j = 0; j < 2 * R; ++j) cur[j] = p[j];
    for (int b = 0; b < nb; ++b) {
      const int bn = b + 1 < nb ? b + 1 : b;
      double nxt[2 * R];
#pragma unroll
      for (int j = 0; j < 2 * R; ++j) nxt[j] = p[bn * 2 * R + j];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double e = fma(cur[2 * i], b1, b0) - cur[2 * i + 1];
        a[i & 3] = fma(e, e, a[i & 3]);
      }
#pragma unroll
      for (int j = 0; j < 2 * R; ++j) cur[j] = nxt[j];
    }
  } else {
    for (int b = 0; b < nb; ++b) {
      double cur[2 * R];
#pragma unroll
      for (int j = 0; j < 2 * R; ++j) cur[j] = p[b * 2 * R + j];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double e = fma(cur[2 * i], b1, b0) - cur[2 * i + 1];
        a[i & 3] = fma(e, e, a[i & 3]);
      }
    }
  }
  for (int r = nb * R; r < n; ++r) {
    const double e = fma(p[2 * r], b1, b0) - p[2 * r + 1];
    a[0] = fma(e, e, a[0]);
  }
  return (a[0] + a[1]) + (a[2] + a[3]);
}

template <int V>
__global__ void __launch_bounds__(1024) k_ll(const double* __restrict__ obs, int N, int npass,
                                             double* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const double* src = obs + (size_t)(blockIdx.x % 64) * N * 2;
  for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) lds[i] = src[i];
  __syncthreads();
  FamLinreg<2> fam{};
  fam.intercept = 1;
  fam.sigma_known = 1.0;
  double tot = 0.0;
  double b0 = 0.1 + 1e-3 * lane, b1 = 2.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int ps = 0; ps < npass; ++ps) {
    if (w >= 1) {
      int64_t ra;
      int rn;
      nmc_chunk(0, N, w - 1, W - 1, &ra, &rn);
      double acc[1];
      if (V == 0) {
        double th[3] = {b0, b1, 1.0};
        nmc_ll_rows_lds(fam, fam.prepare(th), lds + ra * 2, rn, acc);
      } else if (V == 1) {
        acc[0] = rows_lds_r<8, false>(lds + ra * 2, rn, b0, b1);
      } else if (V == 2) {
        acc[0] = rows_lds_r<8, true>(lds + ra * 2, rn, b0, b1);
      } else if (V == 3) {
        double th[3] = {b0, b1, 1.0};
        nmc_ll_rows(fam, fam.prepare(th), src + ra * 2, rn, acc);
      } else {
        acc[0] = rows_lds_r<16, true>(lds + ra * 2, rn, b0, b1);
      }
      tot += acc[0];
    }
    __syncthreads();
    b0 += 1e-6;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = tot;
}

int main() {
  const int N = 1000, npass = 400;
  std::vector<double> h((size_t)64 * N * 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  double *obs, *out;
  unsigned long long* cyc;
  hipMalloc(&obs, h.size() * 8);
  hipMemcpy(obs, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMalloc(&out, 256 * 1024 * 8);
  hipMalloc(&cyc, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int V = 0; V < 5; ++V) {
    auto kern = V == 0 ? k_ll<0> : V == 1 ? k_ll<1> : V == 2 ? k_ll<2> : V == 3 ? k_ll<3> : k_ll<4>;
    const size_t lds = (size_t)N * 16;
    hipLaunchKernelGGL(kern, dim3(256), dim3(1024), lds, 0, obs, N, 10, out, cyc);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(256), dim3(1024), lds, 0, obs, N, npass, out, cyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // fp64 lane-op floor per pass: 1000 rows x 64 lanes x 3 ops per workgroup at the
    // measured 44.5 lane-ops/clk/CU
    printf("{\"variant\": %d, \"cycles_per_pass\": %.0f, \"us_per_pass\": %.3f, "
           "\"floor_cycles\": %.0f}\n", V, (double)c / npass, ms * 1e3 / npass,
           1000.0 * 64 * 3 / 44.5);
  }
  return 0;
}
