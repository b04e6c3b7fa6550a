"""User log-likelihood callbacks in the reference convention (parameter[P][n] -> ll[n]).

These are "user code" as the reference's examples write it; the golden fixtures
were captured by running the reference sampler on exactly these functions
(tests/golden/make_golden.py) and the oracle tests run the restatement on them.
"""

import numpy
import scipy.stats


def ll_regression3(parameter, X, y):
    """example/regression.py:53-67 (intercept, slope, noise sd)."""
    betaHat = numpy.vstack([parameter[0], parameter[1]]).T
    yHat = numpy.sum(X * betaHat, axis=1)
    noise = numpy.array(parameter[2])
    return scipy.stats.norm(loc=y, scale=noise).logpdf(yHat)


def ll_regression2(parameter, x, y):
    """cfg 3 model: y ~ N(b0 + b1 x, 1)."""
    yHat = numpy.array(parameter[0]) + numpy.array(parameter[1]) * x
    return scipy.stats.norm(loc=y, scale=1.0).logpdf(yHat)


def ll_logistic(parameter, X, y):
    """cfg 5 model: eta = X.theta, ll = y eta - logaddexp(0, eta)."""
    theta = numpy.vstack(parameter).T
    eta = numpy.sum(X * theta, axis=1)
    return y * eta - numpy.logaddexp(0.0, eta)


def ll_distribution(parameter, mu, sd, sizes):
    """example/distribution.py:18-24, vectorised with the same arithmetic:
    ll_i = sum_j norm(mu[j][g(i)], sd[j]).logpdf(parameter[j][i])."""
    g = numpy.repeat(numpy.arange(len(sizes)), sizes)
    out = 0
    for j in range(len(parameter)):
        out = out + scipy.stats.norm(loc=mu[j][g], scale=sd[j]).logpdf(
            numpy.asarray(parameter[j], float))
    return out
