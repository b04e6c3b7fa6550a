// fam_user.h -- a user-supplied log-likelihood as a device family, compiled at run time
// (hiprtc, user.hip).  The reference's plug-in point is an arbitrary Python callable
// logLikelihoodFunction(parameter[P][n]) -> ll[n] (posteriorSampling.py:61-102) that the
// sampler calls once per parameter step over every observation (:615-635); on the GPU
// the same contract is one observation at a time:
//
//   __device__ double nmc_user_loglik(const double* theta,   // [P] this chain's group values
//                                     const double* row,     // [NF] the observation's fields
//                                     const double* k);      // the model's constants
//
// defined by the user's source ahead of this header, with NMC_USER_NF / NMC_USER_P set.
// FamUser wraps it in the family interface of families.h: the group log-likelihood is the
// sum of the per-observation values in the kernels' fixed order, the same order as every
// built-in family, so a user functor that restates a built-in family's expression (e.g.
// FamLogistic's fma chain) reproduces it bit for bit.
#pragma once

struct FamUser {
  static constexpr int NFIELDS = NMC_USER_NF;
  static constexpr int MAXP = NMC_USER_P;
  static constexpr int NACC = 1;
  static constexpr bool ASM_ROWS = false;
  const double* k;   // device copy of the model constants (may be null)

  struct Reg { double t[MAXP]; };

  __device__ __forceinline__ Reg prepare(const double* th) const {
    Reg r;
#pragma unroll
    for (int j = 0; j < MAXP; ++j) r.t[j] = th[j];
    return r;
  }
  __device__ __forceinline__ void accum(const Reg& r, const double* __restrict__ row,
                                        double* acc) const {
    acc[0] += nmc_user_loglik(r.t, row, k);
  }
  template <int N>
  __device__ __forceinline__ void accumN(const Reg& r, const double* __restrict__ rows,
                                         double (&a)[4][NACC]) const {
#pragma unroll
    for (int i = 0; i < N; ++i) a[i & 3][0] += nmc_user_loglik(r.t, rows + i * NFIELDS, k);
  }
  __device__ __forceinline__ double finish(const Reg&, const double* acc, long n) const {
    return n == 0 ? 0.0 : acc[0];
  }
  __device__ __forceinline__ double gconst(long) const { return 0.0; }
  __device__ __forceinline__ void hold() {}   // (families.h FamLinreg::hold; no constants)
  __device__ __forceinline__ double finish_fast(const Reg& r, const double* acc, long n,
                                                double) const {
    return finish(r, acc, n);
  }
  __device__ __forceinline__ double obs_ll(const Reg& r, const double* __restrict__ row) const {
    return nmc_user_loglik(r.t, row, k);
  }
};
