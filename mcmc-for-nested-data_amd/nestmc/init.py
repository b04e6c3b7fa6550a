"""Chain initialisation, reproducing the reference's RNG consumption, batched over chains.

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

Every chain draws from its own RandomState, so the chains can advance in lock step:
each round of the start-point search and of the partial init loop evaluates the
likelihoods of ALL chains in one batched call -- ``group_ll(theta[C, P, G]) -> [C, G]``,
the device's nmc_eval_group_ll -- and only the chains whose result
was not finite draw again, in the reference's order.  The draws and the decisions
taken on them are the reference's; only the finiteness tests and the stored group
log-likelihoods come from the device (its summation order; the first accepted step
replaces the latter anyway).  The MLE objective stays the exact numpy sum of the
family callable (:1102-1105): its value steers Nelder-Mead, so it keeps the
reference's rounding.  Without ``group_ll`` the host evaluates the family callable.
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


def _norm_logpdf_groups(x, loc, scale):
    """_norm_logpdf over one parameter's G values (elementwise the same IEEE operations;
    the one log is of the scalar scale, as in the scalar form)."""
    if not scale > 0:
        return numpy.full(x.shape, numpy.nan)
    with numpy.errstate(divide="ignore", invalid="ignore"):
        y = (x - loc) / scale
        out = (-y ** 2 / 2.0 - LOG_C) - numpy.log(scale)
    out[numpy.isnan(y)] = numpy.nan
    return out


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


def _draw_start(names, rs, priors, ranges):
    """One start candidate x[P] of MCMC._findStartingPoint (:1070-1079)."""
    x = [0] * len(names)
    for i, name in enumerate(names):
        if name in ranges:
            x[i] = rs.uniform(low=ranges[name][0], high=ranges[name][1])
        elif priors is not None:
            x[i] = priors[i].rvs(random_state=rs)
        else:
            raise ValueError(
                "parameter %r needs a startingPointValueRange entry or a prior "
                "(the reference fails here with numpy.random.norm, :1079)" % name)
    return x


def _host_batch_group_ll(family, sizes, off):
    one = host_group_ll(family, sizes, off)

    def f(theta):
        return numpy.stack([one(theta[c]) for c in range(theta.shape[0])])
    return f


def init_chains(family, sizes, names, chains, pooling, priors, ranges, mle, threads=1,
                group_ll=None):
    """Stacked initial states for global chain ids ``chains``: dict of [C, ...] arrays.

    group_ll: batched group log-likelihoods theta[C, P, G] -> [C, G] for exactly these
    chains (the device's Engine.eval_group_ll); None evaluates the family on the host.
    """
    chains = [int(c) for c in chains]
    C, P, G = len(chains), len(names), len(sizes)
    sizes = numpy.asarray(sizes, dtype=numpy.int64)
    off = numpy.concatenate([[0], numpy.cumsum(sizes)])
    n_total = int(off[-1])
    ranges = ranges or {}
    if group_ll is None:
        group_ll = _host_batch_group_ll(family, sizes, off)
    rss = [numpy.random.RandomState(c) for c in chains]

    # ---- start points (:1066-1089), every chain in lock step --------------------
    theta = numpy.zeros((C, P, G))
    x = [None] * C
    tries = [0] * C
    pending = list(range(C))
    for k in pending:
        x[k] = _draw_start(names, rss[k], priors, ranges)
    while pending:
        for k in pending:
            theta[k] = numpy.asarray(x[k], dtype=numpy.float64)[:, None]
        with numpy.errstate(over="ignore", invalid="ignore"):
            pooled = numpy.sum(group_ll(theta), axis=1)       # -objective(x), :1102-1105
        again = []
        for k in pending:
            tries[k] += 1
            if tries[k] > 1000:
                raise RuntimeError("Failed to find a valid starting state: ll =", -pooled[k])
            if not numpy.isfinite(pooled[k]):
                x[k] = _draw_start(names, rss[k], priors, ranges)
                again.append(k)
        pending = again
    if mle:   # :1107-1141 with the exact numpy objective, chains in parallel
        def opt(k):
            return _optimize_start(family, n_total, names, rss[k], priors, ranges, list(x[k]))
        if threads > 1 and C > 1:
            with ThreadPoolExecutor(max_workers=threads) as ex:
                x = list(ex.map(opt, range(C)))
        else:
            x = [opt(k) for k in range(C)]
    start = numpy.array([[float(v) for v in x[k]] for k in range(C)])   # [C, P]

    if pooling in ("none", "complete"):   # StepMethod._setStartingPoint (:584-592)
        value = numpy.repeat(start[:, :, None], G, axis=2)
        lp = numpy.empty((C, P, G))
        for p in range(P):
            lp[:, p, :] = numpy.asarray(priors[p].logpdf(start[:, p]), dtype=numpy.float64)[:, None]
        return dict(value=value, log_prior=lp, ll=numpy.full((C, G), numpy.nan), mu=None,
                    s2=None)

    # ---- partial (:725-758) ----------------------------------------------------
    mu = start.copy()
    s2 = numpy.sqrt(numpy.abs(start) / 10.)
    sd = numpy.sqrt(s2)
    value = numpy.empty((C, P, G))
    lp = numpy.empty((C, P, G))
    for k in range(C):
        rs = rss[k]
        for p in range(P):
            # scipy norm(mu, sd).rvs(): standard_normal * scale + loc; no draw if scale == 0
            if sd[k, p] == 0:
                value[k, p] = mu[k, p]
            else:
                value[k, p] = rs.standard_normal(G) * sd[k, p] + mu[k, p]
            lp[k, p] = _norm_logpdf_groups(value[k, p], mu[k, p], sd[k, p])
    LL = numpy.full((C, G), numpy.nan)
    pending = list(range(C))
    while pending:
        ll = group_ll(value)
        again = []
        for k in pending:
            fin = numpy.isfinite(ll[k])
            LL[k, fin] = ll[k, fin]
            if not fin.all():
                rs = rss[k]
                for p in range(P):        # _determineIndividualStartingPoint order
                    for g in numpy.flatnonzero(~fin):
                        # samplePriorAndSetValue: logPrior left stale (:284-285)
                        value[k, p, g] = (mu[k, p] if sd[k, p] == 0
                                          else rs.standard_normal() * sd[k, p] + mu[k, p])
                again.append(k)
        pending = again
    return dict(value=value, log_prior=lp, ll=LL, mu=mu, s2=s2)


def _optimize_start(family, n_total, names, rs, priors, ranges, start):
    """MCMC._optimizeStartingPoint (:1107-1141) from a found start point."""
    def objective(xx):
        return -1 * numpy.sum(family([numpy.full(n_total, float(v)) for v in xx]))

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
