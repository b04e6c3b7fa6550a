// fillbench.hip -- where nmc_k_fill's time goes (diagnostics, not shipped): the shipped fill
// kernel (kernels_misc.h) on cfg-3 sizes (P = 2, G = 64, C = 256, partial pooling) for
// T = 1, 5, 20, 100 iterations, in three forms:
//   full   the shipped launch (hyper Gamma elements first, then the step elements)
//   step   step elements only (no hyper elements: none pooling)
//   hyper  hyper elements only (Dev.zin: the step elements skipped)
// and an empty kernel of the same grid (launch + drain floor).  hipEvent timing, median of 20.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//     -I mcmc-for-nested-data_amd/csrc tools/fillbench.hip -o tools/fillbench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "kernels_misc.h"

// candidate step-element fills: a grid-stride loop over (t, p, g, c) on a resident grid,
// U elements per thread-iteration computed side by side (independent dependency chains)
template <int U>
__global__ void __launch_bounds__(256) k_step_gs(Dev d, int iter0, int T) {
  const unsigned C = (unsigned)d.C, GC = (unsigned)d.G * C, PGC = (unsigned)d.P * GC;
  const unsigned n1 = (unsigned)T * PGC;
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < n1; e0 += U * stride) {
    double z[U], lu[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      unsigned e = e0 + k * stride;
      if (e >= n1) e = e0;
      const unsigned t = e / PGC, r = e - t * PGC;
      const unsigned p = r / GC, q = r - p * GC;
      const unsigned g = q / C, c = q - g * C;
      nmc_step_variate(d, iter0 + (int)t, (int)p, (int)g, (int)c, z[k], lu[k]);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned e = e0 + k * stride;
      if (e < n1) {
        d.vzl[2 * (size_t)e] = z[k];
        d.vzl[2 * (size_t)e + 1] = lu[k];
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_empty(double* out, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && out[0] == 12345.0) out[i] = 1.0;
}

int main() {
  const int P = 2, G = 64, C = 256, TMAX = 100;
  Dev d{};
  d.C = C; d.G = G; d.P = P; d.pooling = NMC_POOL_PARTIAL; d.rng_mode = 0; d.seed = 1234;
  d.chain_base = 0; d.ha = (G - 1) / 2.0; d.hlga = lgamma(d.ha); d.vbase = 0;
  hipMalloc(&d.vzl, (size_t)TMAX * P * G * C * 2 * 8);
  hipMalloc(&d.vh, (size_t)TMAX * P * C * 2 * 8);
  double* junk;
  hipMalloc(&junk, 8);
  hipMemset(junk, 0, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("{\"rows\": [\n");
  const int Ts[] = {1, 5, 20, 100};
  bool first = true;
  for (int T : Ts) {
    for (int form = 0; form < 8; ++form) {
      Dev dd = d;
      if (form == 1) dd.pooling = 1;   // step only
      if (form == 2) dd.zin = 1;       // hyper only
      if (form >= 4) dd.pooling = 1;   // (the candidates: step elements only)
      const size_t n = (size_t)T * P * C * ((dd.zin ? 0 : G) + (dd.pooling == NMC_POOL_PARTIAL ? 1 : 0));
      int blocks = (int)((n + 255) / 256 < 16384 ? (n + 255) / 256 : 16384);
      if (form >= 4) {   // resident grids: 2 / 3 / 4 blocks per CU
        const int per = form == 4 ? 3 : form == 5 ? 3 : form == 6 ? 4 : 6;
        blocks = std::min(blocks, 256 * per);
      }
      std::vector<float> ms;
      for (int r = 0; r < 22; ++r) {
        hipEventRecord(a, 0);
        if (form < 3)
          hipLaunchKernelGGL(nmc_k_fill<false>, dim3(blocks), dim3(256), 0, 0, dd, 0, T);
        else if (form == 4)
          hipLaunchKernelGGL(k_step_gs<1>, dim3(blocks), dim3(256), 0, 0, dd, 0, T);
        else if (form == 5)
          hipLaunchKernelGGL(k_step_gs<2>, dim3(blocks), dim3(256), 0, 0, dd, 0, T);
        else if (form == 6)
          hipLaunchKernelGGL(k_step_gs<2>, dim3(blocks), dim3(256), 0, 0, dd, 0, T);
        else if (form == 7)
          hipLaunchKernelGGL(k_step_gs<4>, dim3(blocks), dim3(256), 0, 0, dd, 0, T);
        else
          hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, 0, junk, (unsigned)n);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float t = 0;
        hipEventElapsedTime(&t, a, b);
        if (r >= 2) ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      const char* names[] = {"full", "step", "hyper", "empty", "gs1_3pcu", "gs2_3pcu", "gs2_4pcu", "gs4_6pcu"};
      printf("%s{\"T\": %d, \"form\": \"%s\", \"elements\": %zu, \"blocks\": %d, \"us_median\": %.2f, \"us_min\": %.2f}",
             first ? "" : ",\n", T, names[form], n, blocks, ms[ms.size() / 2] * 1e3, ms[0] * 1e3);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
