// latency.hip -- round-trip latencies the sweep kernel's step path pays (diagnostics, not
// shipped): one wave per workgroup, 256 workgroups, dependent chains of REPS operations,
// shader cycles (s_memtime) per operation, median over workgroups.
//   karg   : s_load of a kernel-argument field through a laundered pointer (as sweep.h)
//   gscal  : s_load of a uniform word of a device buffer (dependent address)
//   ldsrd  : ds_read_b32 + v_readfirstlane (dependent address)
//   ldsat  : ds_add_rtn_u32 + v_readfirstlane (the tile queue's take)
//   memtime: s_memtime back to back
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

struct Args { int pad[64]; int f[64]; const int* buf; unsigned long long* out; int reps; };

template <int V>
__global__ void __launch_bounds__(64) k(Args a_) {
  __shared__ int lds[1024];
  const Args* A = (const Args*)__builtin_amdgcn_kernarg_segment_ptr();
  const int reps = A->reps;
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = (i + 1) & 1023;
  __syncthreads();
  int x = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if constexpr (V == 0) {
      const Args* P = A;
      asm volatile("" : "+s"(P));
      x = P->f[x & 63];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (V == 1) {
      const int* b = A->buf;
      asm volatile("" : "+s"(b));
      x = __builtin_amdgcn_readfirstlane(b[x & 1023]);
    } else if constexpr (V == 2) {
      x = __builtin_amdgcn_readfirstlane(lds[x & 1023]);
    } else if constexpr (V == 3) {
      unsigned v = 0;
      if ((threadIdx.x & 63) == 0)
        v = __hip_atomic_fetch_add((unsigned*)&lds[x & 1023], 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
      x = __builtin_amdgcn_readlane((int)v, 0);
    } else {
      x += (int)__builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) A->out[blockIdx.x] = (t1 - t0) * 1000 / reps + (x == 12345678 ? 1 : 0);
}

int main() {
  const char* names[] = {"karg", "gscal", "ldsrd", "ldsat", "memtime"};
  Args a{};
  for (int i = 0; i < 64; ++i) a.f[i] = (i + 1) & 63;
  std::vector<int> hb(1024);
  for (int i = 0; i < 1024; ++i) hb[i] = (i * 17 + 1) & 1023;
  int* db; unsigned long long* dout;
  hipMalloc(&db, 4096); hipMalloc(&dout, 256 * 8);
  hipMemcpy(db, hb.data(), 4096, hipMemcpyHostToDevice);
  a.buf = db; a.out = dout; a.reps = 4096;
  void (*ks[])(Args) = {k<0>, k<1>, k<2>, k<3>, k<4>};
  printf("{");
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(ks[v], dim3(256), dim3(64), 0, 0, a);
    hipDeviceSynchronize();
    std::vector<unsigned long long> o(256);
    hipMemcpy(o.data(), dout, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(o.begin(), o.end());
    printf("%s\"%s_cycles\": %.1f", v ? ", " : "", names[v], o[128] / 1000.0);
  }
  printf("}\n");
  return 0;
}
