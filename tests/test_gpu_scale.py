"""GPU properties at the benchmark's full size and across shardings.

* shard invariance: chains keyed by global id, so two engines holding halves of
  the chains (chain_base = 0 / C/2, as two ranks would) reproduce the one-engine
  run bit for bit -- the multi-GPU correctness argument, on one device;
* cfg 3 at full size (256 chains x 64 groups x 1000 obs, partial pooling): the
  persistent launch (register Gibbs hand-off, paired-chain row loop), the one-chain
  broadcast row loop and the launch-per-iteration fallback are bit-identical (the likelihood partition and every summation order
  are launch-mode independent), and the first chains match the numpy oracle on the
  same Philox stream (flags exact, values within 1e-9).
"""

import os

import numpy
import pytest

from gpu_cases import synthetic
from nestmc import data
from nestmc.engine import Engine
from nestmc.families import LinearRegression
from oracle import restatement as rs

pytestmark = pytest.mark.gpu


def _state(fam, sizes, C, P, seed=11):
    r = numpy.random.RandomState(seed)
    nested = rs.Nested(fam, sizes)
    G = len(sizes)
    mu = r.normal(0, 0.5, size=(C, P)) + numpy.arange(P)
    s2 = r.uniform(0.2, 1.0, size=(C, P))
    value = mu[:, :, None] + numpy.sqrt(s2)[:, :, None] * r.normal(size=(C, P, G))
    lp = rs.norm_logpdf(value, mu[:, :, None], numpy.sqrt(s2)[:, :, None])
    ll = numpy.array([nested.group_ll(value[c]) for c in range(C)])
    return rs.State(value, lp, ll, mu, s2), nested


def _run(fam, sizes, st, sel, chain_base, n_iter, seed, env=None, launch_iters=0):
    old = {}
    for k, v in (env or {}).items():
        old[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        eng = Engine(fam, sizes, len(sel), "partial", seed=seed, chain_base=chain_base)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    eng.set_state(st.value[sel], st.lp[sel], st.ll[sel], st.mu[sel], st.s2[sel])
    eng.set_schedule(n_iter, n_iter // 2, 1, tune_interval=5)
    eng.set_trace(True)
    if launch_iters:
        eng.set_launch_iters(launch_iters)
    eng.run(0, n_iter)
    acc, llp = eng.trace(n_iter)
    rows = eng.samples()
    cfg = eng.launch_config()
    eng.close()
    return acc, llp, rows, cfg


def test_shard_invariance(gpu_lib):
    fam, sizes, _, _, _ = synthetic("linreg_partial", 192, 16, 100)
    C, P, n_iter, seed = 192, fam.n_params, 16, 404
    st, _ = _state(fam, sizes, C, P)
    whole = _run(fam, sizes, st, numpy.arange(C), 0, n_iter, seed)
    lo = _run(fam, sizes, st, numpy.arange(0, 96), 0, n_iter, seed)
    hi = _run(fam, sizes, st, numpy.arange(96, 192), 96, n_iter, seed)
    for k in range(3):   # acc, llp, rows: chain axis first
        merged = numpy.concatenate([lo[k], hi[k]], axis=0)
        assert numpy.array_equal(merged, whole[k], equal_nan=True), k


def test_cfg3_full_size_launch_modes_and_oracle(gpu_lib):
    C, G, N, n_iter, seed = 256, 64, 1000, 12, 7
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, nested = _state(fam, sizes, C, 2)
    sel = numpy.arange(C)
    pers = _run(fam, sizes, st, sel, 0, n_iter, seed)
    assert pers[3]["persistent"], pers[3]
    launch = _run(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_PERSIST": "0"})
    assert not launch[3]["persistent"]
    bcast = _run(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_ROWS": "bcast"})
    assert bcast[3]["persistent"], bcast[3]
    # persistent launches of 5, 5 and 2 iterations: each launch's closing Gibbs tasks (one
    # per closing workgroup, in parallel) and the publish counters carried over
    multi = _run(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=5)
    assert multi[3]["mode"] == "NMC_MODE_SYNC_REG", multi[3]
    assert pers[3]["kernel"].startswith("nmc_k_run<"), pers[3]
    for other in (launch, bcast, multi):
        for k in range(3):
            assert numpy.array_equal(pers[k], other[k], equal_nan=True), k
    acc = pers[0]
    assert 0.05 < acc.mean() < 0.95

    # the first chains against the oracle on the same stream
    n = 3
    o = rs.State(st.value[:n].copy(), st.lp[:n].copy(), st.ll[:n].copy(), st.mu[:n].copy(),
                 st.s2[:n].copy())
    trace, rec = {}, []
    rs.run(nested, o, "partial", None, n_iter, n_iter // 2, 1,
           rs.PhiloxRNG(numpy.arange(n), seed), tune_interval=5, trace=trace, record=rec)
    oacc = numpy.stack(trace["acc"], 1).reshape(n, n_iter, 2, G)
    dev = acc[:n].astype(bool)
    assert numpy.array_equal(dev, oacc)
    orows = numpy.stack([r for _, r in rec], 1)
    drows = pers[2][:n]
    assert numpy.allclose(drows, orows, rtol=1e-9, atol=1e-9)
