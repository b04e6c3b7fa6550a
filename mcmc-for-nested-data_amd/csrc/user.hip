// user.hip -- user-supplied device log-likelihoods (the reference's plug-in point,
// logLikelihoodFunction, posteriorSampling.py:61-102) compiled at run time with hiprtc.
//
// nmc_user_family_compile(source, n_fields, n_params, include_dir) registers
//   #define NMC_USER_NF / NMC_USER_P; #include "kernels.h"; <source>; #include "fam_user.h"
// under a family id >= NMC_LL_USER_BASE and compiles its group-LL kernel at once (source
// errors surface there).  Each other kernel -- the step kernel in the mode a run uses,
// the per-observation LL kernels -- is compiled with hiprtc for gfx950 the first time it
// is launched, with the library's own flags (-O3 -ffp-contract=off, no fast-math: the MH
// branches need IEEE NaN/inf), and loaded per device.  Every family op then launches the
// module's kernels through hipModuleLaunchKernel, with the same grids, LDS carve and
// residency rules as the built-in families (ctx.h nmc_run_launches).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "ctx.h"

namespace {

// kernel table entries, in name-expression order
// (nmc_k_run: mode m (0..4) with rows in LDS at UK_RUN0 + m, rows staged at UK_RUN0 + 5 + m;
// the half layout at UK_HALF)
enum { UK_RUN0 = 0, UK_NRUN = 5, UK_GROUP_LL = 10, UK_OBS_LL_ROWS = 11, UK_OBS_LL = 12,
       UK_GROUP_LL_RL = 13, UK_GROUP_FIN = 14, UK_HALF = 15, UK_N = 16 };
const char* const kNames[UK_N] = {
    "nmc_k_run<FamUser, 0, true>", "nmc_k_run<FamUser, 1, true>", "nmc_k_run<FamUser, 2, true>",
    "nmc_k_run<FamUser, 3, true>", "nmc_k_run<FamUser, 4, true>",
    "nmc_k_run<FamUser, 0, false>", "nmc_k_run<FamUser, 1, false>",
    "nmc_k_run<FamUser, 2, false>", "nmc_k_run<FamUser, 3, false>",
    "nmc_k_run<FamUser, 4, false>",
    "nmc_k_group_part<FamUser, false>", "nmc_k_obs_ll_rows<FamUser>",
    "nmc_k_obs_ll<FamUser>", "nmc_k_group_part<FamUser, true>", "nmc_k_group_fin<FamUser>",
    "nmc_k_run<FamUser, 6, true>"};
int run_index(const nmc_ctx* x, int mode) {
  if (mode == NMC_MODE_HALF) return UK_HALF;
  return UK_RUN0 + mode + (x->d.rows_lds ? 0 : UK_NRUN);
}

struct UserKernels {   // one device's modules, loaded on first use
  hipModule_t mod[UK_N] = {};
  hipFunction_t fn[UK_N] = {};
};

struct UserFamily {
  int nf = 0, np = 0;
  std::string src;                             // the full translation unit
  std::string inc;                             // -I<csrc>
  std::vector<char> code[UK_N];                // compiled on first use, per kernel
  std::string lowered[UK_N];
  std::map<int, UserKernels*> dev;             // per device
};

std::mutex g_mu;
std::vector<UserFamily*> g_fams;

struct FamUserArg { const double* k; };        // FamUser's only member

UserFamily* lookup(int family) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int i = family - NMC_LL_USER_BASE;
  return i >= 0 && i < (int)g_fams.size() ? g_fams[i] : nullptr;
}

// One kernel of the family, compiled alone: a user function with heavy math (lgamma,
// special functions) is inlined into every unrolled row loop, so each step-kernel mode
// costs seconds of compile time -- only the modes a run uses are built.
int compile_kernel(UserFamily* u, int idx) {
  if (!u->code[idx].empty()) return 0;
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, u->src.c_str(), "nestmc_user.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS)
    return nmc_fail(-2, "hiprtcCreateProgram failed");
  hiprtcAddNameExpression(prog, kNames[idx]);
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        u->inc.c_str()};
  const hiprtcResult r = hiprtcCompileProgram(prog, 5, opts);
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    return nmc_fail(-1, std::string("user family: compile failed: ") + hiprtcGetErrorString(r) +
                            "\n" + log);
  }
  const char* lo = nullptr;
  if (hiprtcGetLoweredName(prog, kNames[idx], &lo) != HIPRTC_SUCCESS || !lo) {
    hiprtcDestroyProgram(&prog);
    return nmc_fail(-2, std::string("user family: no lowered name for ") + kNames[idx]);
  }
  u->lowered[idx] = lo;
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  u->code[idx].swap(code);
  return 0;
}

// kernel idx of x's user family on x's device (compiled and loaded on first use)
int user_fn(nmc_ctx* x, int idx, hipFunction_t* f) {
  UserFamily* u = lookup(x->family);
  if (!u) return nmc_fail(-1, "unknown user family id");
  std::lock_guard<std::mutex> lk(g_mu);
  UserKernels*& k = u->dev[x->device];
  if (!k) k = new UserKernels();
  if (!k->fn[idx]) {
    if (int rc = compile_kernel(u, idx)) return rc;
    hipError_t e = hipModuleLoadData(&k->mod[idx], u->code[idx].data());
    if (e != hipSuccess)
      return nmc_fail(-2, std::string("user family: hipModuleLoadData: ") + hipGetErrorString(e));
    e = hipModuleGetFunction(&k->fn[idx], k->mod[idx], u->lowered[idx].c_str());
    if (e != hipSuccess) return nmc_fail(-2, "user family: kernel " + u->lowered[idx] + " missing");
  }
  *f = k->fn[idx];
  return 0;
}

int launch(nmc_ctx* x, hipFunction_t f, dim3 grid, dim3 block, size_t lds, void** args) {
  HIPCHK(hipModuleLaunchKernel(f, grid.x, grid.y, grid.z, block.x, block.y, block.z,
                               (unsigned)lds, x->stream, args, nullptr));
  return 0;
}

}  // namespace

extern "C" int nmc_user_family_compile(const char* source, int n_fields, int n_params,
                                       const char* include_dir, int* family_id) {
  *family_id = -1;
  if (!source || !include_dir) return nmc_fail(-1, "user family: source and include_dir needed");
  if (n_fields < 1 || n_fields > 64 || n_params < 1 || n_params > NMC_MAXP)
    return nmc_fail(-1, "user family: need 1 <= n_fields <= 64, 1 <= n_params <= 16");
  UserFamily* u = new UserFamily();
  u->nf = n_fields;
  u->np = n_params;
  // the library's own build-time kernel constants, so the JIT kernels index LDS and tiles
  // exactly as the host carve (nmc_lds / nmc_tiles) computed them
  const std::string defs = "#define NMC_NSLOT_N " + std::to_string((int)NMC_NSLOT) +
                           "\n#define NMC_HYPER_NS " + std::to_string((int)NMC_HYPER_NS) +
                           "\n#define NMC_LDS_ROW_DOUBLES " +
                           std::to_string((int)NMC_LDS_ROW_DOUBLES) +
                           "\n#define NMC_RUN_THREADS " + std::to_string((int)NMC_RUN_THREADS) +
                           "\n#define NMC_ZIN_BUILD " + std::to_string((int)NMC_ZIN_BUILD) +
                           "\n"
#ifdef NMC_STAMPS
                           "#define NMC_STAMPS 1\n"
#endif
      ;
  u->src = defs + "#define NMC_USER_NF " + std::to_string(n_fields) + "\n#define NMC_USER_P " +
           std::to_string(n_params) + "\n#include \"kernels.h\"\n#line 1 \"user\"\n" + source +
           "\n#include \"fam_user.h\"\n";
  u->inc = std::string("-I") + include_dir;
  // the cheapest kernel now: a source error is reported here, with the compiler log
  if (int rc = compile_kernel(u, UK_GROUP_LL)) {
    delete u;
    return rc;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_fams.push_back(u);
  *family_id = NMC_LL_USER_BASE + (int)g_fams.size() - 1;
  return 0;
}

extern "C" int nmc_user_family_shape(int family_id, int* n_fields, int* n_params) {
  UserFamily* u = lookup(family_id);
  if (!u) return nmc_fail(-1, "unknown user family id");
  *n_fields = u->nf;
  *n_params = u->np;
  return 0;
}

int nmc_user_attach(nmc_ctx* x, int family) {
  UserFamily* u = lookup(family);
  if (!u) return nmc_fail(-1, "unknown user family id (nmc_user_family_compile first)");
  if (u->nf != x->nf || u->np != x->P)
    return nmc_fail(-1, "user family compiled for other n_fields / n_params");
  x->user = u;
  return 0;
}

// The family ops of fam_ops.h nmc_fam_call, through the module's kernels.
int nmc_call_user(nmc_ctx* x, NmcCall& c) {
  if (!x->user) return nmc_fail(-1, "user family not attached");
  FamUserArg fam{x->user_k};
  hipFunction_t f = nullptr;
  const Dev& d0 = x->d;
  switch (c.op) {
    case NMC_OP_RUN: {
      const double* obs = d0.obs;
      int i0 = c.i0, i1 = c.i1, flags = c.flags;
      int rc = 0;
      const int e = nmc_run_launches(x, i0, i1, [&](int mode, const Dev& d, dim3 grid,
                                                   dim3 block, size_t lds) {
        if (rc) return;
        if (mode < 0 || (mode >= UK_NRUN && mode != NMC_MODE_HALF)) {
          rc = nmc_fail(-1, "user family: unknown step-kernel mode");
          return;
        }
        Dev dd = d;
        void* args[] = {&dd, &fam, (void*)&obs, &i0, &i1, &flags};
        hipFunction_t fr = nullptr;
        rc = user_fn(x, run_index(x, mode), &fr);
        if (!rc) rc = launch(x, fr, grid, block, lds, args);
      });
      return rc ? rc : e;
    }
    case NMC_OP_CAN_PERSIST: {
      if (const char* e = getenv("NMC_PERSIST")) {
        c.result = atoi(e) != 0;
        return 0;
      }
      int nb = 0;
      if (int rc = user_fn(x, run_index(x, nmc_persist_mode(x)), &f)) return rc;
      if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * x->d.W,
                                                            nmc_persist_lds(x)) != hipSuccess) {
        c.result = 0;
        return 0;
      }
      c.result = (int64_t)x->d.RB * x->d.G * x->d.S <= (int64_t)nmc_safe_blocks(x, nb) * x->ncu;
      return 0;
    }
    case NMC_OP_CAPACITY: {
      int nb = 0;
      if (int rc = user_fn(x, run_index(x, run_mode(x)), &f)) return rc;
      HIPCHK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f,
                                                               64 * x->d.W, run_lds_bytes(x)));
      c.result = nmc_safe_blocks(x, nb) * x->ncu;
      return 0;
    }
    case NMC_OP_GROUP_LL: {   // (fam_ops.h: member partials into c.aux, then the combine)
      Dev dd = d0;
      const double* obs = d0.obs;
      const double* in = c.in;
      double* aux = c.aux;
      double* out = c.out;
      void* a1[] = {&dd, &fam, (void*)&obs, (void*)&in, (void*)&aux};
      if (int rc = user_fn(x, d0.rows_lds ? UK_GROUP_LL_RL : UK_GROUP_LL, &f)) return rc;
      if (int rc = launch(x, f, dim3(d0.CB * d0.G * d0.S), dim3(64 * std::min(d0.W, 8)),
                          nmc_group_ll_lds(x), a1))
        return rc;
      const size_t n = (size_t)d0.G * d0.C;
      void* a2[] = {&dd, &fam, (void*)&in, (void*)&aux, (void*)&out};
      if (int rc = user_fn(x, UK_GROUP_FIN, &f)) return rc;
      return launch(x, f, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, a2);
    }
    case NMC_OP_OBS_LL_ROWS: {
      const int n = c.i1 - c.i0;
      if (n <= 0 || x->n_obs == 0) return 0;
      Dev dd = d0;
      const int* gidx = (const int*)x->gidx;
      int64_t n_obs = x->n_obs;
      int pc = x->pooling == NMC_POOL_PARTIAL ? 2 : 0, row0 = c.i0, nrows = n, c0 = c.c0;
      const int nc = c.nc > 0 ? c.nc : x->C;
      double* out = c.out;
      void* args[] = {&dd, &fam, (void*)&gidx, &n_obs, &pc, &row0, &nrows, &c0, &out};
      if (int rc = user_fn(x, UK_OBS_LL_ROWS, &f)) return rc;
      return launch(x, f,
                    dim3((unsigned)((x->n_obs + 255) / 256), (unsigned)nc, (unsigned)n),
                    dim3(256), 0, args);
    }
    case NMC_OP_OBS_LL: {
      Dev dd = d0;
      const double* in = c.in;
      double* out = c.out;
      int64_t n_obs = x->n_obs;
      void* args[] = {&dd, &fam, (void*)&in, &out, &n_obs};
      if (int rc = user_fn(x, UK_OBS_LL, &f)) return rc;
      return launch(x, f, dim3(x->d.CB * x->G), dim3(64), 0, args);
    }
  }
  return nmc_fail(-1, "unknown family op");
}
