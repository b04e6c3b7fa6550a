"""GPU: the resident step launch (nmc_set_resident) changes no bit.

One launch serves consecutive nmc_run calls: a call continuing where the last one ended is
handed to the running launch (kernels.h res_gate) instead of a new launch, and every other
entry point parks it.  Each call is closed as a launch ends, so every call plan below --
synchronized calls, calls queued without a synchronize, an idle gap longer than the
launch's own park, a state read (park) in the middle, explicit prefills, a call that does
not continue the last -- must give the accept flags, proposal log-likelihoods, recorded rows,
final state and accept counts of separate launches bit for bit, and the Philox run must
still match the oracle.  The cfg-3 and cfg-2 geometries (every CU holding one workgroup of
the launch) run at full size.
"""

import numpy
import pytest

from gpu_cases import partial_state, run_engine, run_oracle, synthetic

pytestmark = pytest.mark.gpu

S, G0 = "synchronize", ("synchronize", 0, 0)
PLANS = {
    "synced": [("run", 0, 3), G0, ("run", 3, 6), G0, ("run", 6, 7), G0, ("run", 7, 12)],
    "queued": [("run", 0, 2), ("run", 2, 5), ("run", 5, 9), ("run", 9, 12)],
    "idle_park": [("run", 0, 4), G0, ("sleep", 40, 0), ("run", 4, 8), G0, ("run", 8, 12)],
    "state_read": [("run", 0, 4), ("get_state", 0, 0), ("run", 4, 8), ("run", 8, 12)],
    "prefill": [("run", 0, 3), ("prefill", 3, 9), ("run", 3, 9), ("run", 9, 12)],
}


def _same(a, b, what, partial=True):
    for k in range(3):
        assert numpy.array_equal(a[k], b[k], equal_nan=True), (what, k)
    # (the hyper-parameters exist under partial pooling only)
    for k in ("value", "log_prior", "ll", "scale") + (("mu", "s2") if partial else ()):
        assert numpy.array_equal(a[3]["state"][k], b[3]["state"][k], equal_nan=True), (what, k)
    assert numpy.array_equal(a[3]["accept"], b[3]["accept"]), what


def _case(kind, C, G, N):
    fam, sizes, priors, _, _ = synthetic(kind, C, G, N)
    if kind == "linreg_partial":
        st, nested = partial_state(fam, sizes, C, fam.n_params)
        pooling = "partial"
    elif kind == "gauss_none":   # (as test_gpu_configs.test_cfg2_full_size_half_layout)
        from oracle import restatement as rs
        pooling = "none"
        r = numpy.random.RandomState(4)
        nested = rs.Nested(fam, sizes)
        value = numpy.repeat((r.normal(0, 0.3, size=(C, 3)))[:, :, None], G, axis=2)
        lp = numpy.stack([numpy.asarray(priors[p].logpdf(value[:, p, :])) for p in range(3)], 1)
        st = rs.State(value, lp, numpy.full((C, G), numpy.nan))
    else:
        from test_gpu_parity import _synthetic_state
        pooling = "none"
        st, nested = _synthetic_state(fam, sizes, priors, pooling, C, fam.n_params, G)
    return fam, sizes, priors, st, nested, pooling


@pytest.mark.parametrize("kind", ["linreg_partial", "regression3_none"])
def test_resident_plans_bit_identical(gpu_lib, kind, monkeypatch):
    monkeypatch.setenv("NMC_RESIDENT_IDLE_US", "5000")
    C, G, N, n_iter, seed = 130, 6, 40, 12, 31
    fam, sizes, priors, st, nested, pooling = _case(kind, C, G, N)
    sel = numpy.arange(C)
    kw = dict(pooling=pooling, priors=priors)
    base = run_engine(fam, sizes, st, sel, 0, n_iter, seed, calls=PLANS["synced"], **kw)
    assert base[3]["resident"]["launches"] == 0
    for name, plan in PLANS.items():
        got = run_engine(fam, sizes, st, sel, 0, n_iter, seed, calls=plan, resident=True, **kw)
        r = got[3]["resident"]
        assert r["enabled"], (name, r)
        assert r["launches"] >= 1 and r["calls"] >= 1, (name, r)
        _same(got, base, name, pooling == "partial")
    # one call per launch when each call does not continue the last (a park between)
    got = run_engine(fam, sizes, st, sel, 0, n_iter, seed, resident=True,
                     calls=[("run", 0, 6), ("get_state", 0, 0), ("run", 6, 12)], **kw)
    assert got[3]["resident"]["launches"] == 2 and got[3]["resident"]["calls"] == 0
    _same(got, base, "parked", pooling == "partial")
    oacc, ollp, orows, margin = run_oracle(nested, st, sel, sel, n_iter, seed, pooling=pooling,
                                           priors=priors)
    assert numpy.array_equal(base[0].astype(bool), oacc), margin
    assert numpy.allclose(base[2], orows, rtol=1e-9, atol=1e-9, equal_nan=True)


@pytest.mark.parametrize("kind,C,G,N", [("linreg_partial", 256, 64, 1000),
                                        ("gauss_none", 256, 32, 500)])
def test_resident_full_size_bit_identical(gpu_lib, kind, C, G, N):
    """cfg-3 / cfg-2 geometry: the launch holds every CU; five calls of four iterations."""
    n_iter, seed = 20, 7
    fam, sizes, priors, st, _, pooling = _case(kind, C, G, N)
    sel = numpy.arange(C)
    plan = [("run", 4 * k, 4 * k + 4) for k in range(5)]
    plan = [p for k in plan for p in (k, G0)]
    base = run_engine(fam, sizes, st, sel, 0, n_iter, seed, calls=plan, pooling=pooling,
                      priors=priors)
    got = run_engine(fam, sizes, st, sel, 0, n_iter, seed, calls=plan, pooling=pooling,
                     priors=priors, resident=True)
    r = got[3]["resident"]
    assert r["launches"] == 1 and r["calls"] == 4, (r, got[3]["mode"], got[3]["prefill"])
    _same(got, base, kind, pooling == "partial")
