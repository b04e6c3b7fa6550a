// llbench4.hip -- floors of the likelihood row loop (diagnostics, not shipped).
//
// 256 workgroups of W waves; the likelihood waves of a workgroup split one group's
// N (x, y) rows; NPASS passes per launch with a barrier between passes (the step
// structure of nmc_k_run).  Inner loops are hand-written (inline asm) so the
// compiler's scheduling and register allocation are out of the picture:
//   L  rows in LDS, 8-row blocks, two fixed register sets (ds_read_b128 broadcast)
//   S  rows in global memory through scalar loads (s_load_dwordx16, SGPR operands)
//   V  no loads: the same three fp64 VALU ops per row on register operands (VALU floor)
//   M  mixed: even likelihood waves L, odd waves S
// Per row and chain: e = fma(x, b1, b0) - y; acc = fma(e, e, acc).
// Prints cycles per pass (s_memtime, workgroup 0, wave 0).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define ROW8(A, O) \
  "v_fma_f64 v[" #A ":" #A "+1], v[" #A ":" #A "+1], %[b1], %[b0]\n"

// one 8-row block in v[base .. base+31] = 8 x {x, y}: 24 VALU ops, 4 accumulators
#define BLK(b)                                                                              \
  "v_fma_f64 v[" #b "+0:" #b "+1], v[" #b "+0:" #b "+1], %[b1], %[b0]\n"                    \
  "v_fma_f64 v[" #b "+4:" #b "+5], v[" #b "+4:" #b "+5], %[b1], %[b0]\n"                    \
  "v_fma_f64 v[" #b "+8:" #b "+9], v[" #b "+8:" #b "+9], %[b1], %[b0]\n"                    \
  "v_fma_f64 v[" #b "+12:" #b "+13], v[" #b "+12:" #b "+13], %[b1], %[b0]\n"                \
  "v_fma_f64 v[" #b "+16:" #b "+17], v[" #b "+16:" #b "+17], %[b1], %[b0]\n"                \
  "v_fma_f64 v[" #b "+20:" #b "+21], v[" #b "+20:" #b "+21], %[b1], %[b0]\n"                \
  "v_fma_f64 v[" #b "+24:" #b "+25], v[" #b "+24:" #b "+25], %[b1], %[b0]\n"                \
  "v_fma_f64 v[" #b "+28:" #b "+29], v[" #b "+28:" #b "+29], %[b1], %[b0]\n"                \
  "v_add_f64 v[" #b "+0:" #b "+1], v[" #b "+0:" #b "+1], -v[" #b "+2:" #b "+3]\n"           \
  "v_add_f64 v[" #b "+4:" #b "+5], v[" #b "+4:" #b "+5], -v[" #b "+6:" #b "+7]\n"           \
  "v_add_f64 v[" #b "+8:" #b "+9], v[" #b "+8:" #b "+9], -v[" #b "+10:" #b "+11]\n"         \
  "v_add_f64 v[" #b "+12:" #b "+13], v[" #b "+12:" #b "+13], -v[" #b "+14:" #b "+15]\n"     \
  "v_add_f64 v[" #b "+16:" #b "+17], v[" #b "+16:" #b "+17], -v[" #b "+18:" #b "+19]\n"     \
  "v_add_f64 v[" #b "+20:" #b "+21], v[" #b "+20:" #b "+21], -v[" #b "+22:" #b "+23]\n"     \
  "v_add_f64 v[" #b "+24:" #b "+25], v[" #b "+24:" #b "+25], -v[" #b "+26:" #b "+27]\n"     \
  "v_add_f64 v[" #b "+28:" #b "+29], v[" #b "+28:" #b "+29], -v[" #b "+30:" #b "+31]\n"     \
  "v_fma_f64 %[a0], v[" #b "+0:" #b "+1], v[" #b "+0:" #b "+1], %[a0]\n"                     \
  "v_fma_f64 %[a1], v[" #b "+4:" #b "+5], v[" #b "+4:" #b "+5], %[a1]\n"                     \
  "v_fma_f64 %[a2], v[" #b "+8:" #b "+9], v[" #b "+8:" #b "+9], %[a2]\n"                     \
  "v_fma_f64 %[a3], v[" #b "+12:" #b "+13], v[" #b "+12:" #b "+13], %[a3]\n"                 \
  "v_fma_f64 %[a0], v[" #b "+16:" #b "+17], v[" #b "+16:" #b "+17], %[a0]\n"                 \
  "v_fma_f64 %[a1], v[" #b "+20:" #b "+21], v[" #b "+20:" #b "+21], %[a1]\n"                 \
  "v_fma_f64 %[a2], v[" #b "+24:" #b "+25], v[" #b "+24:" #b "+25], %[a2]\n"                 \
  "v_fma_f64 %[a3], v[" #b "+28:" #b "+29], v[" #b "+28:" #b "+29], %[a3]\n"

#define LD8(b, off)                                                   \
  "ds_read_b128 v[" #b "+0:" #b "+3], %[addr] offset:" #off "+0\n"    \
  "ds_read_b128 v[" #b "+4:" #b "+7], %[addr] offset:" #off "+16\n"   \
  "ds_read_b128 v[" #b "+8:" #b "+11], %[addr] offset:" #off "+32\n"  \
  "ds_read_b128 v[" #b "+12:" #b "+15], %[addr] offset:" #off "+48\n" \
  "ds_read_b128 v[" #b "+16:" #b "+19], %[addr] offset:" #off "+64\n" \
  "ds_read_b128 v[" #b "+20:" #b "+23], %[addr] offset:" #off "+80\n" \
  "ds_read_b128 v[" #b "+24:" #b "+27], %[addr] offset:" #off "+96\n" \
  "ds_read_b128 v[" #b "+28:" #b "+31], %[addr] offset:" #off "+112\n"

#define CLOB_AB                                                                            \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76",     \
      "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", \
      "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101",      \
      "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",    \
      "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123",    \
      "v124", "v125", "v126", "v127"

// LDS loop over nb (even, >= 2) 8-row blocks at LDS byte address addr
__device__ __forceinline__ void loop_lds(unsigned addr, int nb, double b0, double b1,
                                         double& a0, double& a1, double& a2, double& a3) {
  int cnt = nb;
  asm volatile(
      LD8(64, 0)
      "L_lds_%=:\n"
      LD8(96, 128)
      "s_waitcnt lgkmcnt(8)\n"
      BLK(64)
      "v_add_u32 %[addr], 256, %[addr]\n"
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      LD8(64, 0)
      "s_waitcnt lgkmcnt(8)\n"
      BLK(96)
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc1 L_lds_%=\n"
      "s_waitcnt lgkmcnt(0)\n"
      : [addr] "+v"(addr), [cnt] "+s"(cnt), [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2),
        [a3] "+v"(a3)
      : [b0] "v"(b0), [b1] "v"(b1)
      : CLOB_AB, "scc", "memory");
}

// VALU only: the block math on whatever the registers hold (no loads)
__device__ __forceinline__ void loop_valu(int nb, double b0, double b1, double& a0, double& a1,
                                          double& a2, double& a3) {
  int cnt = nb;
  asm volatile(
      "L_valu_%=:\n"
      BLK(64)
      "s_sub_u32 %[cnt], %[cnt], 2\n"
      BLK(96)
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc1 L_valu_%=\n"
      : [cnt] "+s"(cnt), [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
      : [b0] "v"(b0), [b1] "v"(b1)
      : CLOB_AB, "scc");
}

// scalar loads: 8 rows = 128 B = two s_load_dwordx16 into s[64:95]; SGPR operands
#define SROW(k)                                                                                 \
  "v_fma_f64 v[64:65], s[" #k "*4+64:" #k "*4+65], %[b1], %[b0]\n"                            \
  "v_add_f64 v[64:65], v[64:65], -s[" #k "*4+66:" #k "*4+67]\n"                                \
  "v_fma_f64 %[a" #k "], v[64:65], v[64:65], %[a" #k "]\n"
#define SROW2(k, j)                                                                             \
  "v_fma_f64 v[" #j ":" #j "+1], s[" #k "*4+64:" #k "*4+65], %[b1], %[b0]\n"
__device__ __forceinline__ void loop_smem(const double* p, int nb, double b0, double b1,
                                          double& a0, double& a1, double& a2, double& a3) {
  int cnt = nb;
  unsigned long long base = (unsigned long long)p;
  asm volatile(
      "s_mov_b64 s[96:97], %[base]\n"
      "L_smem_%=:\n"
      "s_load_dwordx16 s[64:79], s[96:97], 0x0\n"
      "s_load_dwordx16 s[80:95], s[96:97], 0x40\n"
      "s_add_u32 s96, s96, 0x80\n"
      "s_addc_u32 s97, s97, 0\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_fma_f64 v[64:65], s[64:65], %[b1], %[b0]\n"
      "v_fma_f64 v[66:67], s[68:69], %[b1], %[b0]\n"
      "v_fma_f64 v[68:69], s[72:73], %[b1], %[b0]\n"
      "v_fma_f64 v[70:71], s[76:77], %[b1], %[b0]\n"
      "v_fma_f64 v[72:73], s[80:81], %[b1], %[b0]\n"
      "v_fma_f64 v[74:75], s[84:85], %[b1], %[b0]\n"
      "v_fma_f64 v[76:77], s[88:89], %[b1], %[b0]\n"
      "v_fma_f64 v[78:79], s[92:93], %[b1], %[b0]\n"
      "v_add_f64 v[64:65], v[64:65], -s[66:67]\n"
      "v_add_f64 v[66:67], v[66:67], -s[70:71]\n"
      "v_add_f64 v[68:69], v[68:69], -s[74:75]\n"
      "v_add_f64 v[70:71], v[70:71], -s[78:79]\n"
      "v_add_f64 v[72:73], v[72:73], -s[82:83]\n"
      "v_add_f64 v[74:75], v[74:75], -s[86:87]\n"
      "v_add_f64 v[76:77], v[76:77], -s[90:91]\n"
      "v_add_f64 v[78:79], v[78:79], -s[94:95]\n"
      "v_fma_f64 %[a0], v[64:65], v[64:65], %[a0]\n"
      "v_fma_f64 %[a1], v[66:67], v[66:67], %[a1]\n"
      "v_fma_f64 %[a2], v[68:69], v[68:69], %[a2]\n"
      "v_fma_f64 %[a3], v[70:71], v[70:71], %[a3]\n"
      "v_fma_f64 %[a0], v[72:73], v[72:73], %[a0]\n"
      "v_fma_f64 %[a1], v[74:75], v[74:75], %[a1]\n"
      "v_fma_f64 %[a2], v[76:77], v[76:77], %[a2]\n"
      "v_fma_f64 %[a3], v[78:79], v[78:79], %[a3]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_gt_i32 %[cnt], 0\n"
      "s_cbranch_scc1 L_smem_%=\n"
      : [base] "+s"(base), [cnt] "+s"(cnt), [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2),
        [a3] "+v"(a3)
      : [b0] "v"(b0), [b1] "v"(b1)
      : "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76",
        "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89",
        "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "v64", "v65", "v66", "v67", "v68", "v69", "v70",
        "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "scc", "memory");
}

template <int V>
__global__ void __launch_bounds__(1024) k_ll(const double* __restrict__ obs, int N, int npass,
                                             int nlik, double* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double* src = obs + (size_t)(blockIdx.x % 64) * N * 2;
  for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) lds[i] = src[i];
  __syncthreads();
  double b0 = 0.1 + 1e-3 * lane, b1 = 2.0 + 1e-4 * (lane & 7);
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  // wave w < nlik: rows [w * per, (w + 1) * per) in 16-row units
  const int per = ((N / nlik) / 16) * 16;
  const int nb = per / 8;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int ps = 0; ps < npass; ++ps) {
    if (w < nlik) {
      const int r0 = w * per;
      const int mode = V == 3 ? (w & 1) : V;
      if (mode == 0)
        loop_lds((unsigned)(size_t)(lds + 2 * r0), nb, b0, b1, a0, a1, a2, a3);
      else if (mode == 1)
        loop_smem(src + 2 * r0, nb, b0, b1, a0, a1, a2, a3);
      else
        loop_valu(nb, b0, b1, a0, a1, a2, a3);
    }
    __syncthreads();
    b0 += 1e-6;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = (a0 + a1) + (a2 + a3);
}

int main() {
  const int npass = 400;
  const int N = 1024;
  std::vector<double> h((size_t)64 * N * 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  double *obs, *out;
  unsigned long long* cyc;
  hipMalloc(&obs, h.size() * 8 + 4096);
  hipMemcpy(obs, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMalloc(&out, 256 * 1024 * 8);
  hipMalloc(&cyc, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[4] = {"lds", "smem", "valu", "mixed"};
  for (int W : {16, 13, 12, 8, 4}) {
    for (int V = 0; V < 4; ++V) {
      auto kern = V == 0 ? k_ll<0> : V == 1 ? k_ll<1> : V == 2 ? k_ll<2> : k_ll<3>;
      const size_t lds = (size_t)N * 16 + 512;
      hipLaunchKernelGGL(kern, dim3(256), dim3(1024), lds, 0, obs, N, 10, W, out, cyc);
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(256), dim3(1024), lds, 0, obs, N, npass, W, out, cyc);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      unsigned long long c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const int per = ((N / W) / 16) * 16;
      printf("{\"lik_waves\": %d, \"variant\": \"%s\", \"rows\": %d, \"cycles_per_pass\": %.0f, "
             "\"cycles_per_1000_rows\": %.0f, \"us_per_pass\": %.3f}\n",
             W, names[V], per * W, (double)c / npass, (double)c / npass * 1000.0 / (per * W),
             ms * 1e3 / npass);
    }
  }
  return 0;
}
