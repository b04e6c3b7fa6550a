// varmath_check.hip -- accuracy of rng.h's nmc_log_unit and nmc_cos2pi (host build, no GPU):
// max and mean error in ulps against x86 long-double logl / cosl (64-bit significands) over
// 53-bit uniforms like the sampler's (and 1 - u, the Box-Muller radius argument), plus the
// library's own log / cos on the same inputs for comparison.
//   hipcc -O2 -std=c++17 -ffp-contract=off -I mcmc-for-nested-data_amd/csrc \
//     tools/varmath_check.hip -o /tmp/varmath_check && /tmp/varmath_check
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "rng.h"

static double ulp_err(double got, long double want) {
  if (want == 0.0L) return got == 0.0 ? 0.0 : 1e300;
  const double w = (double)want;
  const double u = nextafter(fabs(w), INFINITY) - fabs(w);
  return (double)fabsl(((long double)got - want) / (long double)u);
}

int main() {
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto next = [&]() {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return (double)(s >> 11) * (1.0 / 9007199254740992.0);
  };
  const long double tpl = 6.283185307179586476925286766559005768L;
  double mlog = 0, slog = 0, mlog_lib = 0, mcos = 0, scos = 0, mcos_lib = 0, mcos_abs = 0;
  const int N = 20000000;
  for (int i = 0; i < N; ++i) {
    double u = next();
    if (i < 64) u = (double)i / 64.0;          // the reduction's breakpoints
    const double x = 1.0 - u;                  // (0, 1]
    const double a = ulp_err(nmc_log_unit(x), logl((long double)x));
    const double b = ulp_err(log(x), logl((long double)x));
    const long double cw = cosl(tpl * (long double)u);
    const double c = ulp_err(nmc_cos2pi(u), cw);
    const double d = ulp_err(cos(6.283185307179586 * u), cw);
    const double ca = fabs((double)((long double)nmc_cos2pi(u) - cw));
    if (x != 1.0) { mlog = fmax(mlog, a); slog += a; mlog_lib = fmax(mlog_lib, b); }
    if (fabsl(cw) > 1e-3L) { mcos = fmax(mcos, c); scos += c; mcos_lib = fmax(mcos_lib, d); }
    mcos_abs = fmax(mcos_abs, ca);
  }
  printf("{\"samples\": %d, \"log_unit_max_ulp\": %.3f, \"log_unit_mean_ulp\": %.4f, "
         "\"libm_log_max_ulp\": %.3f, \"cos2pi_max_ulp\": %.3f, \"cos2pi_mean_ulp\": %.4f, "
         "\"libm_cos_of_rounded_2piu_max_ulp\": %.3f, \"cos2pi_max_abs_err\": %.3e, "
         "\"log0\": %g, \"log1\": %g, \"cos0\": %.17g, \"cos_quarter\": %.17g}\n",
         N, mlog, slog / N, mlog_lib, mcos, scos / N, mcos_lib, mcos_abs, nmc_log_unit(0.0),
         nmc_log_unit(1.0), nmc_cos2pi(0.0), nmc_cos2pi(0.25));
  return 0;
}
