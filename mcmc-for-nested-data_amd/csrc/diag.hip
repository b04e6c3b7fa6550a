// diag.hip -- the convergence diagnostic's variogram on the GPU.
//
// The reference's effective sample size (Diagnostic._computeVariogram,
// sampleDiagnosis.py:189-194, called for every lag t < n by _computeAutocorrelation
// :196-208) is
//   V_t = sum_j sum_{i=t}^{n-1} (x_j[i] - x_j[i-t])^2 / (m (n - t))
// over the m half-chains j of each column: O(m n^2) pure-Python work per column, the
// part that does not scale (16k-66k columns at cfg 4/5).  Here one thread owns one
// (column, lag) and adds in the reference's order: i ascending inside a half-chain, the
// half-chains' sums in j order, then one division.  A block stages one half-chain row
// of its column in LDS at a time; thread t reads row[s + t] (consecutive lanes) and
// row[s] (a broadcast) for s = i - t.  Squares are d * d, correctly rounded; the
// reference's numpy float64 ** 2 goes through libm pow, which rounds a few in 10^4
// squares the other way, so V_t agree to a few ulp (the printed %.3f values agree).
#include <hip/hip_runtime.h>

#include <string>

#include "ctx.h"

// x: [K][m][n] columns' half-chains; out: [K][n].  grid = (ceil(n / 256), K), 256 threads;
// dynamic LDS = n doubles.
__global__ void __launch_bounds__(256) nmc_k_variogram(const double* __restrict__ x, int m, int n,
                                                       double* __restrict__ out) {
  extern __shared__ double row[];
  const int k = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const double* xk = x + (size_t)k * m * n;
  double total = 0.0;
  for (int j = 0; j < m; ++j) {
    __syncthreads();   // the previous row is no longer read
    for (int i = threadIdx.x; i < n; i += 256) row[i] = xk[(size_t)j * n + i];
    __syncthreads();
    if (t < n) {
      double s = 0.0;
      for (int q = 0; q + t < n; ++q) {   // i = q + t, i - t = q
        const double d = row[q + t] - row[q];
        s = s + d * d;
      }
      total = j == 0 ? s : total + s;
    }
  }
  if (t < n) out[(size_t)k * n + t] = total / ((double)m * (double)(n - t));
}

extern "C" int nmc_variogram(int device, const double* x, int K, int m, int n, double* out) {
  if (K < 0 || m < 1 || n < 1) return nmc_fail(-1, "variogram: need K >= 0, m >= 1, n >= 1");
  if ((size_t)n * 8 > (size_t)64 * 1024) return nmc_fail(-1, "variogram: n > 8192 half-chain rows");
  if (K == 0) return 0;
  HIPCHK(hipSetDevice(device));
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  double *dx = nullptr, *dout = nullptr;
  const size_t nx = (size_t)K * m * n, no = (size_t)K * n;
  hipError_t e = hipMalloc(&dx, nx * 8);
  if (e == hipSuccess) e = hipMalloc(&dout, no * 8);
  if (e == hipSuccess) e = hipMemcpyAsync(dx, x, nx * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(nmc_k_variogram, dim3((n + 255) / 256, K), dim3(256), (size_t)n * 8, st,
                       dx, m, n, dout);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, no * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  hipFree(dx);
  hipFree(dout);
  hipStreamDestroy(st);
  if (e != hipSuccess) return nmc_fail(-2, std::string("variogram: ") + hipGetErrorString(e));
  return 0;
}
