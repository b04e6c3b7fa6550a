"""Device log-likelihood sources for the user-family tests (DeviceLikelihood)."""

import numpy
import scipy.special



def logistic_source(k):
    """FamLogistic's own expression (csrc/families.h) as a user function, rows
    [x_1..x_k, y], theta [b0, b1..bk]: eta = b0 + fma chain; ll = y eta - logaddexp(0, eta)
    (nmc_logaddexp0, the library's numpy.logaddexp restatement)."""
    return r"""
__device__ double nmc_user_loglik(const double* th, const double* row, const double* k) {
  double eta = th[0];
  for (int j = 0; j < %d; ++j) eta = fma(row[j], th[j + 1], eta);
  return row[%d] * eta - nmc_logaddexp0(eta);
}
""" % (k, k)


LOGISTIC4 = logistic_source(3)
LOGISTIC8 = logistic_source(7)

# A model no built-in family covers: Poisson regression with a log link and an exposure
# constant, rows [x, y, lgamma(y + 1)] (the data-only term precomputed per row), theta
# [a, b], k = {log exposure}:  ll = y eta - exp(eta) - lgamma(y + 1),  eta = a + b x + k[0]
POISSON = r"""
__device__ double nmc_user_loglik(const double* th, const double* row, const double* k) {
  const double eta = th[0] + th[1] * row[0] + k[0];
  return row[1] * eta - exp(eta) - row[2];
}
"""


def poisson_rows(x, y):
    return numpy.stack([x, y, scipy.special.gammaln(y + 1.0)], 1)


def poisson_host(x, y, log_exposure):
    """The same model in the reference's calling convention (parameter[P][n] -> ll[n])."""
    lgy = scipy.special.gammaln(y + 1.0)

    def f(parameter):
        eta = numpy.asarray(parameter[0]) + numpy.asarray(parameter[1]) * x + log_exposure
        return y * eta - numpy.exp(eta) - lgy
    return f


def poisson_data(G, N, seed=2):
    r = numpy.random.RandomState(seed)
    x = r.normal(size=G * N)
    a = r.normal(0.5, 0.3, size=G)
    b = r.normal(0.3, 0.2, size=G)
    g = numpy.repeat(numpy.arange(G), N)
    y = r.poisson(numpy.exp(a[g] + b[g] * x + 0.1)).astype(float)
    return x, y
