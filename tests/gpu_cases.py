"""Build device families / engines for the golden and synthetic parity cases."""

import numpy
import scipy.stats

from golden_cases import Case
from nestmc.families import GaussianMean, LinearRegression, Logistic


def family_for(case):
    a = case.arr
    n = case.name
    if n.startswith("regression"):
        return LinearRegression(a["X"], a["y"])
    if n.startswith("linreg"):
        return LinearRegression.simple(a["x"], a["y"], sigma=1.0)
    if n.startswith("distribution"):
        sizes = [case.n_per_group] * case.n_groups
        return GaussianMean.from_groups(a["mu"], a["sd"], sizes)
    if n.startswith("logistic"):
        return Logistic(a["X"], a["y"])
    raise KeyError(n)


def synthetic(kind, C, G, N, seed=3, ragged=False):
    """(family, sizes, priors, pooling, names) for GPU-vs-oracle Philox parity."""
    rs = numpy.random.RandomState(seed)
    if ragged:
        sizes = list(rs.randint(0, 2 * N, size=G))
        sizes[0] = max(sizes[0], 1)
    else:
        sizes = [N] * G
    n = int(sum(sizes))
    grp = numpy.repeat(numpy.arange(G), sizes)
    if kind == "linreg_partial":
        x = rs.normal(size=n)
        b0 = rs.normal(size=G)
        b1 = rs.normal(2, 1, size=G)
        y = b0[grp] + b1[grp] * x + rs.normal(size=n)
        return LinearRegression.simple(x, y, sigma=1.0), sizes, None, "partial", ("b0", "b1")
    if kind == "regression3_none":
        x = rs.normal(size=n)
        y = 1.0 + 3.0 * x + rs.normal(size=n) * 0.7
        priors = [scipy.stats.norm(0, 10), scipy.stats.norm(3, 10), scipy.stats.gamma(2)]
        fam = LinearRegression(numpy.vstack([numpy.ones(n), x]).T, y)
        return fam, sizes, priors, "none", ("b0", "b1", "sigma")
    if kind == "gauss_none":
        mu = rs.normal(size=(3, G))
        sd = rs.gamma(1, size=3) + 0.2
        fam = GaussianMean.from_groups(mu, sd, sizes)
        priors = [scipy.stats.norm(0, 1)] * 3
        return fam, sizes, priors, "none", ("a", "b", "c")
    if kind == "gauss1_partial":
        mu = rs.normal(size=(1, G))
        fam = GaussianMean.from_groups(mu, [0.8], sizes)
        return fam, sizes, None, "partial", ("a",)
    if kind == "logistic_partial":
        K = 4
        X = numpy.hstack([numpy.ones((n, 1)), rs.normal(size=(n, K - 1))])
        th = rs.normal(0, 0.5, size=(G, K))
        p = 1 / (1 + numpy.exp(-numpy.sum(X * th[grp], axis=1)))
        y = (rs.uniform(size=n) < p).astype(float)
        return Logistic(X, y), sizes, None, "partial", ("t0", "t1", "t2", "t3")
    if kind == "linreg_complete":
        x = rs.normal(size=n)
        y = 0.5 - 1.5 * x + rs.normal(size=n)
        priors = [scipy.stats.norm(0, 5), scipy.stats.norm(0, 5), scipy.stats.halfnorm(scale=3)]
        fam = LinearRegression(numpy.vstack([numpy.ones(n), x]).T, y)
        return fam, [n], priors, "complete", ("b0", "b1", "sigma")
    raise KeyError(kind)


def golden(name):
    return Case(name)
