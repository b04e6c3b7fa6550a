// llbench.hip -- microbenchmark of the per-group log-likelihood loop (diagnostics).
//
// One workgroup = 64 chains (lanes) x one group of N rows (x, y fp64); W waves split
// the rows; every wave evaluates sum (b0 + b1 x - y)^2 for P passes.  Variants:
//   0  rows staged in LDS, wave-uniform ds_read_b128 (broadcast)
//   1  rows read with scalar loads (s_load_dwordx16, SGPR operands)
//   2  half the waves LDS, half scalar
//   3/5 scalar loads, explicit prefetch of the next 4/8-row block
//   4  empty body (launch + geometry overhead)
// Prints us per launch and per-row cycles.  Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

template <class T>
__device__ __forceinline__ double rows_ll(const T* __restrict__ q, int r0, int r1, int P,
                                          double b0, double b1) {
  double tot = 0.0;
  for (int p = 0; p < P; ++p) {
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int r = r0;
    for (; r + 8 <= r1; r += 8) {
      double x[8], y[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) { x[i] = q[2 * (r + i)]; y[i] = q[2 * (r + i) + 1]; }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        double e = fma(x[i], b1, b0) - y[i];
        if ((i & 3) == 0) a0 = fma(e, e, a0);
        if ((i & 3) == 1) a1 = fma(e, e, a1);
        if ((i & 3) == 2) a2 = fma(e, e, a2);
        if ((i & 3) == 3) a3 = fma(e, e, a3);
      }
    }
    for (; r < r1; ++r) {
      double e = fma(q[2 * r], b1, b0) - q[2 * r + 1];
      a0 = fma(e, e, a0);
    }
    tot += (a0 + a1) + (a2 + a3);
    b0 += 1e-3;
  }
  return tot;
}

// explicit software pipeline: block b+1 requested before block b is consumed
template <int R>
__device__ __forceinline__ double rows_ll_pf(const double* __restrict__ q, int r0, int r1, int P,
                                             double b0, double b1) {
  double tot = 0.0;
  for (int p = 0; p < P; ++p) {
    double a[4] = {0, 0, 0, 0};
    const int nb = (r1 - r0) / R;
    int r = r0;
    if (nb > 0) {
      double cur[2 * R];
#pragma unroll
      for (int j = 0; j < 2 * R; ++j) cur[j] = q[2 * r0 + j];
      for (int b = 0; b < nb; ++b) {
        const int bn = b + 1 < nb ? b + 1 : b;
        double nxt[2 * R];
#pragma unroll
        for (int j = 0; j < 2 * R; ++j) nxt[j] = q[2 * (r0 + bn * R) + j];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double e = fma(cur[2 * i], b1, b0) - cur[2 * i + 1];
          a[i & 3] = fma(e, e, a[i & 3]);
        }
#pragma unroll
        for (int j = 0; j < 2 * R; ++j) cur[j] = nxt[j];
      }
      r = r0 + nb * R;
    }
    for (; r < r1; ++r) {
      double e = fma(q[2 * r], b1, b0) - q[2 * r + 1];
      a[0] = fma(e, e, a[0]);
    }
    tot += (a[0] + a[1]) + (a[2] + a[3]);
    b0 += 1e-3;
  }
  return tot;
}

template <int V>
__global__ void __launch_bounds__(1024) k_ll(const double* __restrict__ obs, int G, int N, int P,
                                             const double* __restrict__ theta, double* out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int g = blockIdx.x % G;
  const double* src = obs + (size_t)g * N * 2;
  const bool use_lds = V == 0 || (V == 2 && (w & 1));
  if (V == 0 || V == 2) {
    for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) lds[i] = src[i];
    __syncthreads();
  }
  double b0 = theta[lane], b1 = theta[64 + lane];
  const int per = (N + W - 1) / W;
  const int r0 = w * per;
  const int r1 = r0 + per < N ? r0 + per : N;
  double tot;
  if (V == 3) tot = rows_ll_pf<4>(src, r0, r1, P, b0, b1);
  else if (V == 5) tot = rows_ll_pf<8>(src, r0, r1, P, b0, b1);
  else if (V == 4) tot = b0 + b1;
  else tot = use_lds ? rows_ll(lds, r0, r1, P, b0, b1) : rows_ll(src, r0, r1, P, b0, b1);
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = tot;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 64;
  const int N = argc > 2 ? atoi(argv[2]) : 1000;
  const int CB = argc > 3 ? atoi(argv[3]) : 4;
  const int P = 2, reps = 200;
  std::vector<double> h((size_t)G * N * 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  double *obs, *th, *out;
  hipMalloc(&obs, h.size() * 8);
  hipMemcpy(obs, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  std::vector<double> t(128, 0.5);
  hipMalloc(&th, 128 * 8);
  hipMemcpy(th, t.data(), 128 * 8, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)CB * G * 1024 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double work = (double)CB * G * N * P;  // wave-rows x 64
  for (int V = 0; V < 6; ++V) {
    for (int W : {4, 8, 16}) {
      auto kern = V == 0 ? k_ll<0> : V == 1 ? k_ll<1> : V == 2 ? k_ll<2> : V == 3 ? k_ll<3> : V == 4 ? k_ll<4> : k_ll<5>;
      const size_t lds = (V == 0 || V == 2) ? (size_t)N * 16 : 0;
      for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL(kern, dim3(CB * G), dim3(64 * W), lds, 0, obs, G, N, P, th, out);
      hipEventRecord(a);
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(kern, dim3(CB * G), dim3(64 * W), lds, 0, obs, G, N, P, th, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / reps;
      // VALU ceiling: 3 fp64 ops x 4 cycles per wave-row, 1024 SIMDs, 2.4 GHz
      const double floor_us = work * 12.0 / 1024 / 2.4e3;
      printf("{\"variant\": %d, \"waves\": %d, \"G\": %d, \"N\": %d, \"CB\": %d, \"us\": %.3f, "
             "\"valu_floor_us\": %.3f}\n", V, W, G, N, CB, us, floor_us);
    }
  }
  return 0;
}
