// llbench3.hip -- row-loop variants of the likelihood phase in isolation (diagnostics).
//
// 256 workgroups x 16 waves; 15 waves split one group's N (x, y) rows (the rows of
// group blockIdx % 64), NPASS passes per launch with a barrier between passes.
//   0  LDS rows, nmc_ll_rows_lds (the shipped loop: 4-row blocks, copy-based prefetch)
//   1  LDS rows, R-row blocks, ping-pong prefetch unrolled by two (no register copies), R=4
//   2  the same, R=8
//   3  global rows through scalar loads (SGPR operands), 8-row blocks, ping-pong prefetch
//   4  global rows, scalar loads, the shipped nmc_ll_rows
//   5  global rows, scalar loads, 4-row blocks, ping-pong prefetch
// Prints cycles per pass (s_memtime, workgroup 0) and us per pass (events).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#include "../mcmc-for-nested-data_amd/csrc/kernels.h"

template <int R>
__device__ __forceinline__ void blk_load(const double* __restrict__ p, double (&v)[2 * R]) {
#pragma unroll
  for (int j = 0; j < 2 * R; ++j) v[j] = p[j];
}

template <int R>
__device__ __forceinline__ void blk_acc(const double (&v)[2 * R], double b0, double b1,
                                        double (&a)[4]) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const double e = fma(v[2 * i], b1, b0) - v[2 * i + 1];
    a[i & 3] = fma(e, e, a[i & 3]);
  }
}

// ping-pong: block b in A, b+1 in B; no copies between the two register sets
template <int R>
__device__ __forceinline__ double rows_pp(const double* __restrict__ p, int n, double b0,
                                          double b1) {
  double a[4] = {0, 0, 0, 0};
  const int nb = n / R;
  double A[2 * R], B[2 * R];
  int b = 0;
  if (nb > 0) blk_load<R>(p, A);
  for (; b + 1 < nb; b += 2) {
    blk_load<R>(p + (size_t)(b + 1) * 2 * R, B);
    blk_acc<R>(A, b0, b1, a);
    if (b + 2 < nb) blk_load<R>(p + (size_t)(b + 2) * 2 * R, A);
    blk_acc<R>(B, b0, b1, a);
  }
  if (b < nb) blk_acc<R>(A, b0, b1, a);
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
  double b0 = 0.1 + 1e-3 * lane, b1 = 2.0 + 1e-4 * (lane & 7);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int64_t ra;
  int rn;
  nmc_chunk(0, N, w - 1, W - 1, &ra, &rn);
  for (int ps = 0; ps < npass; ++ps) {
    if (w >= 1) {
      double acc[1];
      if (V == 0) {
        double th[3] = {b0, b1, 1.0};
        nmc_ll_rows_lds(fam, fam.prepare(th), lds + ra * 2, rn, acc);
      } else if (V == 1) {
        acc[0] = rows_pp<4>(lds + ra * 2, rn, b0, b1);
      } else if (V == 2) {
        acc[0] = rows_pp<8>(lds + ra * 2, rn, b0, b1);
      } else if (V == 3) {
        acc[0] = rows_pp<8>(src + ra * 2, rn, b0, b1);
      } else if (V == 4) {
        double th[3] = {b0, b1, 1.0};
        nmc_ll_rows(fam, fam.prepare(th), src + ra * 2, rn, acc);
      } else {
        acc[0] = rows_pp<4>(src + ra * 2, rn, b0, b1);
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
  const int npass = 400;
  for (int N : {1000, 4000}) {
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
    for (int V = 0; V < 6; ++V) {
      auto kern = V == 0 ? k_ll<0> : V == 1 ? k_ll<1> : V == 2 ? k_ll<2> : V == 3 ? k_ll<3>
                : V == 4 ? k_ll<4> : k_ll<5>;
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
      printf("{\"N\": %d, \"variant\": %d, \"cycles_per_pass\": %.0f, \"us_per_pass\": %.3f}\n", N,
             V, (double)c / npass, ms * 1e3 / npass);
    }
    hipFree(obs);
    hipFree(out);
    hipFree(cyc);
  }
  return 0;
}
