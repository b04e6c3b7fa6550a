"""Seeded synthetic nested datasets for the benchmark configurations.

Every generator consumes a ``numpy.random.RandomState`` in a fixed, documented
order so that the same arrays can be rebuilt on any host (the GPU box never sees
the reference, so the fixtures and the bench regenerate data from these).

* ``example_regression``   -- ``example/regression.py:16-50`` (after
  ``numpy.random.seed(12345)``, ``:13``): X = [1, x], y = X.beta + N(0, 1).
* ``example_distribution`` -- ``example/distribution.py:28-37``: per parameter,
  group means mu_jg ~ N(0, 1) and a shared sd_j ~ Gamma(1).
* ``linreg``               -- SURVEY.md 8(d) cfg 3/4: RandomState(7),
  x ~ N(0,1), b0_g ~ N(0,1), b1_g ~ N(2,1), y = b0 + b1 x + N(0,1).
* ``logistic``             -- SURVEY.md 8(d) cfg 5: RandomState(1),
  X[:,0] = 1, X[:,1:] ~ N(0,1), theta_g ~ N(0, 0.5^2), y ~ Bernoulli(sigmoid).
"""

import numpy


def example_regression(n_groups, n_per_group, rs=None):
    """Restates ``generateData`` of ``example/regression.py:16-50``.

    ``rs`` defaults to ``RandomState(12345)`` which is the state the example
    module leaves behind at import (``example/regression.py:13``).
    Returns dict(group, X (n x 2 with the ones column), y) and the true betas.
    """
    if rs is None:
        rs = numpy.random.RandomState(12345)
    n = n_groups * n_per_group
    x = numpy.hstack([numpy.ones((n, 1)), rs.normal(size=(n, 1))])
    b0 = numpy.repeat(rs.normal(loc=0, scale=1, size=n_groups), n_per_group)
    b1 = numpy.repeat(rs.normal(loc=100, scale=100, size=n_groups), n_per_group)
    beta = numpy.vstack([b0, b1]).T
    y = numpy.sum(x * beta, axis=1) + rs.normal(size=n)
    group = numpy.repeat(numpy.arange(n_groups), n_per_group)
    return {"group": group, "X": x, "y": y}


def example_distribution(n_params, n_groups, rs=None):
    """Restates the parameter draws of ``example/distribution.py:28-37``.

    Returns (mu[P][G], sd[P]).  The example's per-response likelihood is
    sum_j norm(mu[j][g], sd[j]).logpdf(theta_j) (``:18-24``).
    """
    if rs is None:
        rs = numpy.random.RandomState(12345)
    mu = numpy.empty((n_params, n_groups))
    sd = numpy.empty(n_params)
    for j in range(n_params):
        mu[j] = rs.normal(loc=0, scale=1, size=n_groups)
        sd[j] = rs.gamma(1)
    return mu, sd


def linreg(n_groups, n_per_group, seed=7):
    """cfg 3/4 data: returns (x, y, b0, b1) with x, y of length G*N (group-major)."""
    rs = numpy.random.RandomState(seed)
    b0 = rs.normal(0.0, 1.0, n_groups)
    b1 = rs.normal(2.0, 1.0, n_groups)
    n = n_groups * n_per_group
    x = rs.normal(0.0, 1.0, n)
    g = numpy.repeat(numpy.arange(n_groups), n_per_group)
    y = b0[g] + b1[g] * x + rs.normal(0.0, 1.0, n)
    return x, y, b0, b1


def logistic(n_groups, n_per_group, n_coef=8, seed=1):
    """cfg 5 data: returns (X (n x K, X[:,0] = 1), y in {0,1}, theta[G][K])."""
    rs = numpy.random.RandomState(seed)
    theta = rs.normal(0.0, 0.5, (n_groups, n_coef))
    n = n_groups * n_per_group
    X = numpy.empty((n, n_coef))
    X[:, 0] = 1.0
    X[:, 1:] = rs.normal(0.0, 1.0, (n, n_coef - 1))
    g = numpy.repeat(numpy.arange(n_groups), n_per_group)
    eta = numpy.sum(X * theta[g], axis=1)
    p = 1.0 / (1.0 + numpy.exp(-eta))
    y = (rs.uniform(size=n) < p).astype(numpy.float64)
    return X, y, theta
