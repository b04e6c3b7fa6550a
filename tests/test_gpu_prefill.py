"""GPU: nmc_run's pipelined variate fill (nmc_prefill) changes no bit.

The variates of a chunk are drawn on a second stream beside the previous chunk's step
launch (within a call, and the same length again for the next call), or by an explicit
nmc_prefill.  A chunk that starts where the pending prefill starts takes its iterations
(a longer chunk fills the rest), any other chunk fills its own.  Every call plan below must
give the accept flags, proposal log-likelihoods and recorded rows of the unpipelined run
(NMC_PREFILL=0) bit for bit, and the replayed reference variates must still reproduce the
reference's flags and rows through chunked, pipelined launches.
"""

import numpy
import pytest

from golden_cases import Case
from gpu_cases import family_for, partial_state, run_engine, run_oracle, synthetic
from nestmc.engine import Engine
from oracle import restatement as rs

pytestmark = pytest.mark.gpu

# (run | prefill, i0, i1): prefix takes, a longer chunk than the prefill, a prefill that no
# chunk starts at, an explicit prefill replaced by nmc_run's own
PLANS = {
    "one_call_chunks": [("run", 0, 12)],
    "calls": [("run", 0, 2), ("run", 2, 5), ("run", 5, 6), ("prefill", 8, 11), ("run", 6, 12)],
    "explicit": [("run", 0, 1), ("prefill", 1, 7), ("run", 1, 4), ("prefill", 4, 5),
                 ("run", 4, 9), ("run", 9, 12)],
}


def _same(a, b):
    for k in range(3):
        assert numpy.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("pooling", ["partial", "none"])
def test_prefill_plans_bit_identical(gpu_lib, pooling):
    kind = "linreg_partial" if pooling == "partial" else "regression3_none"
    C, G, N, n_iter, seed = 130, 6, 40, 12, 23
    fam, sizes, priors, _, _ = synthetic(kind, C, G, N)
    if pooling == "partial":
        st, nested = partial_state(fam, sizes, C, fam.n_params)
    else:
        from test_gpu_parity import _synthetic_state
        st, nested = _synthetic_state(fam, sizes, priors, pooling, C, fam.n_params, G)
    sel = numpy.arange(C)
    kw = dict(pooling=pooling, priors=priors, launch_iters=3)
    base = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_PREFILL": "0"}, **kw)
    assert base[3]["prefill"] == {"issued": 0, "used": 0}
    for name, plan in PLANS.items():
        got = run_engine(fam, sizes, st, sel, 0, n_iter, seed, calls=plan, **kw)
        _same(got, base)
        assert got[3]["prefill"]["used"] > 0, (name, got[3]["prefill"])
    # the pipelined run against the oracle itself
    oacc, ollp, orows, margin = run_oracle(nested, st, sel, sel, n_iter, seed, pooling=pooling,
                                           priors=priors)
    assert numpy.array_equal(base[0].astype(bool), oacc), margin
    assert numpy.allclose(base[2], orows, rtol=1e-9, atol=1e-9, equal_nan=True)


def test_prefill_counts_one_call_chunks(gpu_lib):
    """Four chunks of 3 in one call: the last three come from prefills drawn beside the
    chunk before them; the call ends at the schedule's end, so nothing is drawn after it."""
    C, G, N, n_iter, seed = 64, 5, 30, 12, 5
    fam, sizes = synthetic("linreg_partial", C, G, N)[:2]
    st, _ = partial_state(fam, sizes, C, fam.n_params)
    got = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, launch_iters=3)
    assert got[3]["prefill"] == {"issued": 9, "used": 9}, got[3]["prefill"]


@pytest.mark.parametrize("name", ["linreg_partial"])
def test_prefill_replay_chunks_match_reference(gpu_lib, name):
    """The reference's own variates, replayed through launches of 2 iterations whose
    variates are drawn beside the launch before: the reference's flags and rows."""
    c = Case(name)
    a = c.arr
    fam = family_for(c)
    eng = Engine(fam, c.sizes, c.n_chains, c.pooling, c.priors, rng="replay")
    eng.set_state(a["init_value"], a["init_lp"], a["init_ll"][:, 0, :],
                  a.get("init_mu"), a.get("init_s2"))
    eng.set_replay(a["z"], a["u"], a["hz"], a["hu"])
    burn, thin = rs.schedule(c.n_iter, c.n_samples)
    eng.set_schedule(c.n_iter, burn, thin)
    eng.set_trace(True)
    eng.set_launch_iters(2)
    half = c.n_iter // 2
    eng.run(0, half)
    eng.run(half, c.n_iter)
    acc, llp = eng.trace(c.n_iter)
    assert numpy.array_equal(acc.astype(numpy.int8), a["acc"])
    assert numpy.allclose(llp, a["ll"], rtol=1e-9, atol=1e-9, equal_nan=True)
    assert numpy.allclose(eng.samples(), a["rows"], rtol=1e-9, atol=1e-9, equal_nan=True)
    assert eng.prefill_stats()["used"] > 0
    eng.close()
