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


def partial_state(fam, sizes, C, P, seed=11, spread=1.0):
    """A random partial-pooling start ([C] chains) and the oracle's Nested for it."""
    from oracle import restatement as rs
    r = numpy.random.RandomState(seed)
    nested = rs.Nested(fam, sizes)
    G = len(sizes)
    mu = r.normal(0, 0.5, size=(C, P)) + numpy.arange(P) * (1.0 if P <= 2 else 0.0)
    s2 = r.uniform(0.2, 1.0, size=(C, P)) * spread
    value = mu[:, :, None] + numpy.sqrt(s2)[:, :, None] * r.normal(size=(C, P, G))
    lp = rs.norm_logpdf(value, mu[:, :, None], numpy.sqrt(s2)[:, :, None])
    ll = numpy.array([nested.group_ll(value[c]) for c in range(C)])
    return rs.State(value, lp, ll, mu, s2), nested


def run_engine(fam, sizes, st, sel, chain_base, n_iter, seed, pooling="partial", priors=None,
               env=None, burn=None, thin=1, tune_interval=5, launch_iters=0, calls=None,
               resident=False):
    """Run the HIP engine on chains ``sel`` of state ``st``; returns
    (accept flags [C, iter, P, G], proposal LLs, recorded rows [C, rows, cols], launch config).
    calls: the engine calls in order, ("run" | "prefill", i0, i1), ("synchronize", 0, 0),
    ("sleep", ms, 0) or ("get_state", 0, 0) (default: one run).  resident: nmc_set_resident
    (launch config: "resident" stats, "state" the final get_state, "accept" the counts)."""
    import os
    from nestmc.engine import Engine
    old = {}
    for k, v in (env or {}).items():
        old[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        eng = Engine(fam, sizes, len(sel), pooling, priors, seed=seed, chain_base=chain_base)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    mu = None if st.mu is None else st.mu[sel]
    s2 = None if st.s2 is None else st.s2[sel]
    eng.set_state(st.value[sel], st.lp[sel], st.ll[sel], mu, s2)
    eng.set_schedule(n_iter, n_iter // 2 if burn is None else burn, thin,
                     tune_interval=tune_interval)
    eng.set_trace(True)
    if launch_iters:
        eng.set_launch_iters(launch_iters)
    if resident:
        eng.set_resident(True)
    for op, a, b in calls or [("run", 0, n_iter)]:
        if op == "synchronize":
            eng.synchronize()
        elif op == "sleep":
            import time
            time.sleep(a / 1e3)
        elif op == "get_state":
            eng.get_state()
        else:
            getattr(eng, op)(a, b)
    eng.synchronize()
    res = eng.resident_stats()
    acc, llp = eng.trace(n_iter)
    rows = eng.samples()
    cfg = eng.launch_config()
    cfg["gibbs_fallbacks"] = eng.gibbs_fallbacks()
    cfg["prefill"] = eng.prefill_stats()
    cfg["resident"] = res
    cfg["state"] = eng.get_state()
    cfg["accept"] = eng.accept_counts()
    eng.close()
    return acc, llp, rows, cfg


def run_oracle(nested, st, sel, chain_ids, n_iter, seed, pooling="partial", priors=None,
               burn=None, thin=1, tune_interval=5):
    """The numpy oracle on the same Philox stream for chains ``sel`` (global ids chain_ids)."""
    from oracle import restatement as rs
    C = len(sel)
    o = rs.State(st.value[sel].copy(), st.lp[sel].copy(), st.ll[sel].copy(),
                 None if st.mu is None else st.mu[sel].copy(),
                 None if st.s2 is None else st.s2[sel].copy())
    P, G = o.value.shape[1], o.value.shape[2]
    trace, rec = {}, []
    rs.run(nested, o, pooling, priors, n_iter, n_iter // 2 if burn is None else burn, thin,
           rs.PhiloxRNG(numpy.asarray(chain_ids), seed), tune_interval=tune_interval,
           trace=trace, record=rec)
    acc = numpy.stack(trace["acc"], 1).reshape(C, n_iter, P, G)
    llp = numpy.stack(trace["llp"], 1).reshape(C, n_iter, P, G)
    margin = numpy.min(numpy.stack(trace["margin"]))
    rows = numpy.stack([r for _, r in rec], 1)
    return acc, llp, rows, margin
