"""Host-side chain initialisation, reproducing the reference's RNG consumption.

Chain c is seeded with ``RandomState(c)`` exactly like ``numpy.random.seed(chain)``
(posteriorSampling.py:225, :1015), so the start values equal the reference's:

* start point   MCMC._findStartingPoint (:1060-1095): uniform in the given range,
                else ``prior.rvs()``, until the pooled log-likelihood is finite
                (at most 1000 tries);
* optional MLE  MCMC._optimizeStartingPoint (:1107-1141): scipy Nelder-Mead on the
                pooled negative log-likelihood, same options and retry rule;
* none/complete StepMethod._setStartingPoint (:584-592): every group starts at the
                start point, logPrior = prior.logpdf, LL = NaN;
* partial       PartialPooling._initialiseParameters (:725-744) and
                _determineIndividualStartingPoint (:746-758), including the stale
                logPrior of re-drawn groups (:284-285).

This is one-off host work, not the sampling hot loop.
"""

import warnings
from concurrent.futures import ThreadPoolExecutor

import numpy
import scipy.optimize

from .families import GaussianMean  # noqa: F401  (documentation link)

LOG_C = 0.9189385332046727


class ChainInit:
    """Initial state of one chain (arrays [P, G], [G], [P])."""

    def __init__(self, value, log_prior, ll, mu=None, s2=None):
        self.value = value
        self.log_prior = log_prior
        self.ll = ll
        self.mu = mu
        self.s2 = s2


def _norm_logpdf(x, loc, scale):
    with numpy.errstate(divide="ignore", invalid="ignore"):
        y = (x - loc) / scale
        out = (-y ** 2 / 2.0 - LOG_C) - numpy.log(scale)
    if not scale > 0 or numpy.isnan(y):
        return numpy.nan
    return float(out)


def group_sums(ll, off):
    """Sequential per-group sums (the builtin ``sum`` of posteriorSampling.py:632)."""
    G = len(off) - 1
    out = numpy.zeros(G)
    for g in range(G):
        a, b = off[g], off[g + 1]
        if b > a:
            out[g] = numpy.cumsum(ll[a:b])[-1]
    return out


def host_group_ll(family, sizes, off):
    def f(theta_pg):
        param = [numpy.repeat(numpy.asarray(t, float), sizes) for t in theta_pg]
        return group_sums(numpy.asarray(family(param), dtype=numpy.float64), off)
    return f


def find_starting_point(family, n_total, names, rs, priors, ranges, mle):
    ranges = ranges or {}

    def objective(xx):
        return -1 * numpy.sum(family([numpy.full(n_total, float(v)) for v in xx]))

    ll = numpy.inf
    x = [0] * len(names)
    tries = 0
    while not numpy.isfinite(ll):
        for i, name in enumerate(names):
            if name in ranges:
                x[i] = rs.uniform(low=ranges[name][0], high=ranges[name][1])
            elif priors is not None:
                x[i] = priors[i].rvs(random_state=rs)
            else:
                raise ValueError(
                    "parameter %r needs a startingPointValueRange entry or a prior "
                    "(the reference fails here with numpy.random.norm, :1079)" % name)
        ll = objective(x)
        tries += 1
        if tries > 1000:
            raise RuntimeError("Failed to find a valid starting state: ll =", ll)
    start = list(x)
    if mle:
        n = 0
        while True:
            n += 1
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                res = scipy.optimize.minimize(objective, start, method="Nelder-Mead",
                                              options={"maxiter": None, "maxfev": None,
                                                       "xtol": 0.0001, "ftol": 0.0001})
            if numpy.isfinite(res.fun):
                start = res.x
                if res.success:
                    break
            else:
                # the reference calls _findStartingPoint() without arguments here
                # (:1131, a TypeError); restart the search instead.
                start = find_starting_point(family, n_total, names, rs, priors, ranges, False)
            if n > 10:
                start = res.x
                break
    return start


def init_chain(family, sizes, names, chain, pooling, priors, ranges, mle, group_ll=None):
    """Initial state of global chain ``chain`` (sizes already pooled for 'complete')."""
    sizes = numpy.asarray(sizes, dtype=numpy.int64)
    off = numpy.concatenate([[0], numpy.cumsum(sizes)])
    n_total = int(off[-1])
    rs = numpy.random.RandomState(chain)
    start = find_starting_point(family, n_total, names, rs, priors, ranges, mle)
    P, G = len(names), len(sizes)
    if pooling in ("none", "complete"):
        value = numpy.array([[float(start[p])] * G for p in range(P)])
        lp = numpy.array([[float(priors[p].logpdf(start[p]))] * G for p in range(P)])
        return ChainInit(value, lp, numpy.full(G, numpy.nan))
    if group_ll is None:
        group_ll = host_group_ll(family, sizes, off)
    mu = numpy.array([float(start[p]) for p in range(P)])
    s2 = numpy.array([numpy.sqrt(numpy.abs(start[p]) / 10.) for p in range(P)])
    sd = numpy.sqrt(s2)

    def draw(p):
        # scipy norm(mu, sd).rvs(): standard_normal * scale + loc; no draw if scale == 0
        if sd[p] == 0:
            return mu[p]
        return rs.standard_normal() * sd[p] + mu[p]

    value = numpy.empty((P, G))
    lp = numpy.empty((P, G))
    for p in range(P):
        for g in range(G):
            value[p, g] = draw(p)
            lp[p, g] = _norm_logpdf(value[p, g], mu[p], sd[p])
    LL = numpy.full(G, numpy.nan)
    ll = numpy.full(G, -numpy.inf)
    while not numpy.all(numpy.isfinite(ll)):
        ll = group_ll(value)
        for p in range(P):
            for g in range(G):
                if numpy.isfinite(ll[g]):
                    LL[g] = ll[g]
                else:
                    value[p, g] = draw(p)       # logPrior left stale (:284-285)
    return ChainInit(value, lp, LL, mu, s2)


def init_chains(family, sizes, names, chains, pooling, priors, ranges, mle, threads=1):
    """Stacked initial states for global chain ids ``chains``: dict of [C, ...] arrays."""
    chains = list(chains)

    def one(c):
        return init_chain(family, sizes, names, c, pooling, priors, ranges, mle)

    if threads > 1 and len(chains) > 1:
        with ThreadPoolExecutor(max_workers=threads) as ex:
            inits = list(ex.map(one, chains))
    else:
        inits = [one(c) for c in chains]
    out = dict(value=numpy.stack([i.value for i in inits]),
               log_prior=numpy.stack([i.log_prior for i in inits]),
               ll=numpy.stack([i.ll for i in inits]))
    if pooling == "partial":
        out["mu"] = numpy.stack([i.mu for i in inits])
        out["s2"] = numpy.stack([i.s2 for i in inits])
    else:
        out["mu"] = out["s2"] = None
    return out
