"""CPU restatement of the reference MCMC hot path -- TEST INFRASTRUCTURE (oracle).

This is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  Parity is pinned: in
``rng="legacy"`` mode it reproduces the reference's ``sample.<chain>.csv`` byte
for byte (tests/test_oracle_golden.py against the fixtures captured by
tests/golden/make_golden.py from /root/reference).

What it restates (file:line into /root/reference/posteriorSampling.py):
  * schedule                  MCMC.__init__ :1018-1027, Sampler._loop :872-894
  * start point (+ MLE)       MCMC._findStartingPoint :1060-1095, _optimizeStartingPoint :1107-1141
  * pooling init              StepMethod._setStartingPoint :584-592,
                              PartialPooling._initialiseParameters :725-744,
                              _determineIndividualStartingPoint :746-758
  * per-obs expansion + sum   StepMethod._computeLogLikelihood :615-627,
                              _computeParameterLogLikelihood :629-635 (sequential sum)
  * proposal                  Parameter.propose :304-306
  * MH test (branch order)    Parameter.step :334-367, _accept/_reject :369-383,
                              group LL propagation :608-610
  * tuning                    Parameter.tune :385-437
  * hyper Gibbs update        HyperParameter.update :463-498, setPrior :273-282,
                              PartialPooling._stepHyperParameter :763-769
  * recording                 header/values :640-654, :771-787, Sampler._print* :898-936

Chains are vectorised: state arrays are [C, P, G].  The variates come from an
RNG object: ``LegacyRNG`` (numpy RandomState(chain), the reference's own stream,
one chain at a time), ``ReplayRNG`` (captured arrays) or ``PhiloxRNG`` (the
device's counter-based stream, oracle/philox.py).
"""

import math
import os
import warnings

import numpy
import scipy.optimize
import scipy.special
import scipy.stats

from . import philox as ph

LOG_C = 0.9189385332046727   # scipy.stats._continuous_distns._norm_pdf_logC


# ----------------------------------------------------------------------------
# schedule (posteriorSampling.py:1018-1027, :872-891)
# ----------------------------------------------------------------------------
def schedule(n_iter, n_samples):
    if n_iter < n_samples:
        raise ValueError("nIter cannot be less than nSamples")
    burn = n_iter // 2 if n_iter // 2 > n_samples else n_iter - n_samples
    thin = int(numpy.ceil((n_iter - burn) / n_samples))
    return burn, thin


def record_iterations(n_iter, burn, thin):
    return [i for i in range(n_iter) if i % thin == 0 and i >= burn]


# ----------------------------------------------------------------------------
# likelihood plumbing (posteriorSampling.py:554-555, :615-635)
# ----------------------------------------------------------------------------
class Nested:
    """Group structure + user LL callable in the reference convention."""

    def __init__(self, ll_function, sizes):
        self.f = ll_function
        self.sizes = numpy.asarray(sizes, dtype=numpy.int64)
        self.off = numpy.concatenate([[0], numpy.cumsum(self.sizes)])
        self.n_total = int(self.off[-1])

    @property
    def G(self):
        return len(self.sizes)

    def obs_ll(self, theta_pg):
        """Per-observation LL for one chain's values theta[P][G] (lists, as :619-625)."""
        param = [numpy.repeat(numpy.asarray(t, float), self.sizes).tolist() for t in theta_pg]
        ll = numpy.asarray(self.f(param), dtype=numpy.float64)
        assert ll.shape == (self.n_total,)
        return ll

    def group_ll(self, theta_pg):
        """Sequential (builtin-``sum``) per-group sums, posteriorSampling.py:631-633."""
        ll = self.obs_ll(theta_pg)
        out = numpy.zeros(self.G)
        for g in range(self.G):
            a, b = self.off[g], self.off[g + 1]
            if b > a:
                out[g] = numpy.cumsum(ll[a:b])[-1]
        return out


# ----------------------------------------------------------------------------
# tuning table (posteriorSampling.py:385-437), vectorised
# ----------------------------------------------------------------------------
def tune(scale, nacc, nrej):
    tot = nacc + nrej
    with numpy.errstate(invalid="ignore", divide="ignore"):
        rate = nacc / tot
    f = numpy.ones_like(scale)
    f = numpy.where(rate > 0.5, 1.1, f)
    f = numpy.where(rate > 0.75, 2.0, f)
    f = numpy.where(rate > 0.95, 10.0, f)
    f = numpy.where(rate < 0.2, 0.9, f)
    f = numpy.where(rate < 0.05, 0.5, f)
    f = numpy.where(rate < 0.001, 0.1, f)
    live = tot > 0
    new = numpy.where(live, scale * f, scale)
    new = numpy.where(new == 0.0, scale, new)
    return new, numpy.where(live, 0.0, nacc), numpy.where(live, 0.0, nrej)


# ----------------------------------------------------------------------------
# random streams
# ----------------------------------------------------------------------------
class LegacyRNG:
    """numpy legacy RandomState(chain): exactly the reference's consumption order."""

    def __init__(self, rs):
        self.rs = rs

    def proposal(self, it, p, value, sd):          # value, sd: [1, G]
        out = numpy.empty_like(value)
        for g in range(value.shape[1]):
            out[0, g] = self.rs.normal(value[0, g], sd[0, g])
        return out

    def accept_uniform(self, it, p, need):          # need: [1, G] bool
        u = numpy.full(need.shape, numpy.nan)
        for g in range(need.shape[1]):
            if need[0, g]:
                u[0, g] = self.rs.random_sample()
        return u

    def hyper_mean(self, it, p, mu_hat, sd):        # [1]
        return numpy.array([self.rs.normal(mu_hat[0], sd[0])])

    def hyper_s2(self, it, p, a, scale):            # scipy invgamma(a, scale).rvs()
        if scale[0] == 0:
            return numpy.array([0.0])
        u = self.rs.uniform()
        return numpy.array([(1.0 / scipy.special.gammainccinv(a, u)) * scale[0] + 0.0])


class ReplayRNG:
    """Variates captured from the reference (tests/golden/*.npz), for C chains."""

    def __init__(self, z, u, hz, hu):
        self.z, self.u, self.hz, self.hu = z, u, hz, hu   # [C, iter, P, G] / [C, iter, P]

    def proposal(self, it, p, value, sd):
        return value + sd * self.z[:, it, p, :]

    def accept_uniform(self, it, p, need):
        return numpy.where(need, self.u[:, it, p, :], numpy.nan)

    def hyper_mean(self, it, p, mu_hat, sd):
        return mu_hat + sd * self.hz[:, it, p]

    def hyper_s2(self, it, p, a, scale):
        u = self.hu[:, it, p]
        with numpy.errstate(divide="ignore"):
            s2 = (1.0 / scipy.special.gammainccinv(a, u)) * scale + 0.0
        return numpy.where(scale == 0, 0.0, s2)


class PhiloxRNG:
    """The device stream (oracle/philox.py), for chains chain_ids."""

    def __init__(self, chain_ids, seed):
        self.ch = numpy.asarray(chain_ids, dtype=numpy.int64)
        self.seed = seed

    def proposal(self, it, p, value, sd):
        G = value.shape[1]
        z = ph.normal(it, numpy.arange(G)[None, :], p, ph.PURPOSE_PROPOSAL,
                      self.ch[:, None], self.seed)
        return value + sd * z

    def accept_uniform(self, it, p, need):
        G = need.shape[1]
        u, _ = ph.uniforms(it, numpy.arange(G)[None, :], p, ph.PURPOSE_ACCEPT,
                           self.ch[:, None], self.seed)
        return u

    def hyper_mean(self, it, p, mu_hat, sd):
        z = ph.normal(it, 0, p, ph.PURPOSE_HYPER_NORMAL, self.ch, self.seed)
        return mu_hat + sd * z

    def hyper_s2(self, it, p, a, scale):
        x = ph.gamma_mt(a, it, p, self.ch, self.seed)
        return numpy.where(scale == 0, 0.0, (1.0 / x) * scale)


# ----------------------------------------------------------------------------
# chain state + the loop
# ----------------------------------------------------------------------------
class State:
    def __init__(self, value, log_prior, ll, mu=None, s2=None):
        self.value = numpy.array(value, float)          # [C, P, G]
        self.lp = numpy.array(log_prior, float)         # [C, P, G]
        self.ll = numpy.array(ll, float)                # [C, G]
        C, P, G = self.value.shape
        self.mu = None if mu is None else numpy.array(mu, float)     # [C, P]
        self.s2 = None if s2 is None else numpy.array(s2, float)
        self.scale = numpy.ones((C, P, G))
        self.nacc = numpy.zeros((C, P, G))
        self.nrej = numpy.zeros((C, P, G))
        self.total_acc = numpy.zeros((C, P, G), numpy.int64)


def norm_logpdf(x, loc, scale):
    """scipy.stats.norm(loc, scale).logpdf(x) (_distn_infrastructure logpdf + _norm_logpdf)."""
    with numpy.errstate(divide="ignore", invalid="ignore"):
        y = (x - loc) / scale
        out = (-y ** 2 / 2.0 - LOG_C) - numpy.log(scale)
    bad = ~(scale > 0) | numpy.isnan(y)
    out = numpy.where(bad, numpy.nan, out)
    return out


def pairwise_sum(a):
    """numpy's float64 add.reduce order (verified equal to numpy.sum)."""
    n = len(a)
    if n < 8:
        r = 0.0
        for x in a:
            r += x
        return r
    if n <= 128:
        r = [a[j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise_sum(a[:n2]) + pairwise_sum(a[n2:])


def run(nested, state, pooling, priors, n_iter, burn, thin, rng, *,
        tune_interval=100, iter_begin=0, trace=None, record=None):
    """Sampler._loop restated for C chains in lockstep.

    ``priors``: list of scipy frozen distributions (none/complete pooling).
    ``trace``:  optional dict collecting acc/llprop/lpprop/u per (iter, p).
    ``record``: optional list receiving (iteration, rows[C][cols]) at record iterations.
    """
    st = state
    C, P, G = st.value.shape
    partial = pooling == "partial"
    for i in range(iter_begin, n_iter):
        do_tune = bool(i) and i < burn and i % tune_interval == 0
        for p in range(P):
            prop = rng.proposal(i, p, st.value[:, p, :], 1.0 * st.scale[:, p, :])
            llp = numpy.empty((C, G))
            for c in range(C):
                th = st.value[c].copy()
                th[p] = prop[c]
                llp[c] = nested.group_ll(th)
            if partial:
                lpp = norm_logpdf(prop, st.mu[:, p, None], numpy.sqrt(st.s2[:, p, None]))
            else:
                lpp = numpy.asarray(priors[p].logpdf(prop), float)
            with numpy.errstate(invalid="ignore"):
                postp = lpp + llp
                post = st.lp[:, p, :] + st.ll
                diff = postp - post
            b1 = ~numpy.isfinite(post) & numpy.isfinite(postp)
            b2 = ~b1 & ~numpy.isfinite(llp)
            b3 = ~b1 & ~b2 & ~numpy.isfinite(diff)
            b4 = ~b1 & ~b2 & ~b3
            u = rng.accept_uniform(i, p, b4)
            with numpy.errstate(divide="ignore", invalid="ignore"):
                acc = b1 | (b4 & (numpy.log(u) < diff))
            st.value[:, p, :] = numpy.where(acc, prop, st.value[:, p, :])
            st.lp[:, p, :] = numpy.where(acc, lpp, st.lp[:, p, :])
            st.ll = numpy.where(acc, llp, st.ll)
            st.nacc[:, p, :] += acc
            st.nrej[:, p, :] += ~acc
            st.total_acc[:, p, :] += acc
            if trace is not None:
                trace.setdefault("acc", []).append(acc.copy())
                trace.setdefault("llp", []).append(llp)
                trace.setdefault("lpp", []).append(lpp)
                trace.setdefault("margin", []).append(
                    numpy.where(b4, numpy.abs(numpy.log(numpy.where(b4, u, 1.0)) - diff),
                                numpy.inf))
            if do_tune:
                st.scale[:, p, :], st.nacc[:, p, :], st.nrej[:, p, :] = tune(
                    st.scale[:, p, :], st.nacc[:, p, :], st.nrej[:, p, :])
            if partial:
                x = st.value[:, p, :]
                mu_hat = numpy.array([pairwise_sum(x[c]) / G for c in range(C)])
                mu = rng.hyper_mean(i, p, mu_hat, numpy.sqrt(st.s2[:, p] / G))
                hat = numpy.array([pairwise_sum((x[c] - mu[c]) ** 2) for c in range(C)]) / (G - 1)
                a = (G - 1) / 2.
                s2 = rng.hyper_s2(i, p, a, a * hat)
                st.mu[:, p] = mu
                st.s2[:, p] = s2
                st.lp[:, p, :] = norm_logpdf(x, mu[:, None], numpy.sqrt(s2)[:, None])
        if record is not None and i >= burn and i % thin == 0:
            record.append((i, row_values(st, partial)))
    return st


def row_values(st, partial):
    """StepMethod.values / PartialPooling.values (posteriorSampling.py:648-654, :780-787)."""
    C, P, G = st.value.shape
    cols = []
    for p in range(P):
        if partial:
            cols.append(st.mu[:, p:p + 1])
            cols.append(st.s2[:, p:p + 1])
        cols.append(st.value[:, p, :])
    return numpy.concatenate(cols, axis=1)


def header(names, G, partial):
    h = []
    for n in names:
        if partial:
            h += ["%s_mu" % n, "%s_sigma2" % n]
        h += ["%s[%.3i]" % (n, g) for g in range(G)]
    return h


# ----------------------------------------------------------------------------
# chain initialisation (posteriorSampling.py:1060-1141, :584-592, :725-758)
# ----------------------------------------------------------------------------
def find_starting_point(nested, names, rs, priors, ranges, mle):
    ranges = ranges or {}
    ll = numpy.inf
    x = [0] * len(names)
    counter = 0
    n = nested.n_total

    def objective(xx):
        return -1 * numpy.sum(nested.f([[v for _ in range(n)] for v in xx]))

    while not numpy.isfinite(ll):
        for i, name in enumerate(names):
            if name in ranges:
                x[i] = rs.uniform(low=ranges[name][0], high=ranges[name][1])
            elif priors is not None:
                x[i] = priors[i].rvs(random_state=rs)
            else:
                raise AttributeError("module 'numpy.random' has no attribute 'norm'")
        ll = objective(x)
        counter += 1
        if counter > 1000:
            raise RuntimeError("Failed to find a valid starting state")
    start = x
    if mle:
        n_try = 0
        while True:
            n_try += 1
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
                raise TypeError("reference bug: _findStartingPoint() called without args")
            if n_try > 10:
                start = res.x
                break
    return start


def init_chain(nested, names, chain, pooling, priors, ranges, mle):
    """Returns (State for one chain [1,P,G], RandomState positioned after init)."""
    rs = numpy.random.RandomState(chain)
    start = find_starting_point(nested, names, rs, priors, ranges, mle)
    P = len(names)
    G = nested.G
    if pooling in ("none", "complete"):
        value = numpy.array([[start[p]] * G for p in range(P)], float)
        lp = numpy.array([[float(priors[p].logpdf(start[p]))] * G for p in range(P)])
        st = State(value[None], lp[None], numpy.full((1, G), numpy.nan))
        return st, rs
    mu = numpy.array([start[p] for p in range(P)], float)
    s2 = numpy.array([numpy.sqrt(numpy.abs(start[p]) / 10.) for p in range(P)])
    value = numpy.empty((P, G))
    lp = numpy.empty((P, G))

    def draw(p):
        sd = numpy.sqrt(s2[p])
        if sd == 0:
            return mu[p]
        return rs.standard_normal() * sd + mu[p]

    for p in range(P):
        for g in range(G):
            value[p, g] = draw(p)
            lp[p, g] = norm_logpdf(value[p, g], mu[p], numpy.sqrt(s2[p]))
    ll = numpy.full(G, -numpy.inf)
    LL = numpy.full(G, numpy.nan)
    while not numpy.all(numpy.isfinite(ll)):
        ll = nested.group_ll(value)
        for p in range(P):
            for g in range(G):
                if numpy.isfinite(ll[g]):
                    LL[g] = ll[g]
                else:
                    value[p, g] = draw(p)      # logPrior deliberately left stale (:284-285)
    st = State(value[None], lp[None], LL[None], mu[None], s2[None])
    return st, rs


# ----------------------------------------------------------------------------
# end-to-end: reference-identical CSV output (legacy RNG)
# ----------------------------------------------------------------------------
def sample_posterior_legacy(n_chains, n_iter, n_samples, names, n_groups, sizes,
                            pooling, ll_function, out_dir, priors=None, mle=False,
                            ranges=None):
    """Writes sample/sample.<chain>.csv exactly as the reference (no logs, no LL file)."""
    if isinstance(sizes, int):
        sizes = [sizes] * n_groups
    if pooling == "complete":
        sizes = [int(sum(sizes))]
    nested = Nested(ll_function, sizes)
    burn, thin = schedule(n_iter, n_samples)
    os.makedirs(os.path.join(out_dir, "sample"), exist_ok=True)
    partial = pooling == "partial"
    for chain in range(n_chains):
        st, rs = init_chain(nested, names, chain, pooling, priors, ranges, mle)
        rows = []
        run(nested, st, pooling, priors, n_iter, burn, thin, LegacyRNG(rs), record=rows)
        path = os.path.join(out_dir, "sample", "sample.%i.csv" % chain)
        with open(path, "w") as h:
            h.write("index,chain," + ",".join(header(names, nested.G, partial)) + "\n")
            for i, vals in rows:
                h.write("%i,%i," % (i, chain) + ",".join(["%f" % v for v in vals[0]]) + "\n")
    return burn, thin
