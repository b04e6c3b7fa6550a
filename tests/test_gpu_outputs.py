"""Per-observation log-likelihood output on the GPU (saveLogLikelihood, the
reference's default: posteriorSampling.py:28-35, :890-891, :907-909, :656-659).

The device re-evaluates StepMethod.logLikelihood at every recorded row of its sample
store; each row must equal the reference callable evaluated at the recorded values
(oracle/restatement.Nested.obs_ll, the :619-625 expansion of theta[P][G] to
observations) for every pooling, and the streamed CSV writer must produce exactly the
"%f" rows of those values.  Tolerance: 1e-12 relative (the device evaluates the
reference's own per-observation formula; only libm rounding may differ).
"""

import os

import numpy
import pytest
import scipy.stats

from gpu_cases import synthetic
from nestmc.engine import Engine
from oracle import restatement as rs

pytestmark = pytest.mark.gpu


def _state(fam, sizes, C, P, pooling, seed=5):
    r = numpy.random.RandomState(seed)
    G = len(sizes)
    value = r.normal(size=(C, P, G)) * 0.3
    if fam.family == "linreg" and P == 3:
        value[:, 2] = 1.0 + numpy.abs(value[:, 2])     # sigma > 0
    lp = numpy.zeros((C, P, G))
    nested = rs.Nested(fam, sizes)
    ll = numpy.array([nested.group_ll(value[c]) for c in range(C)])
    mu = numpy.zeros((C, P)) if pooling == "partial" else None
    s2 = numpy.full((C, P), 0.5) if pooling == "partial" else None
    return value, lp, ll, mu, s2, nested


@pytest.mark.parametrize("kind,C,G,N", [("linreg_partial", 70, 5, 30),
                                        ("gauss_none", 65, 4, 25),
                                        ("linreg_complete", 3, 1, 200)])
def test_obs_ll_rows_match_reference_callable(gpu_lib, kind, C, G, N, tmp_path):
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N)
    P = fam.n_params
    value, lp, ll, mu, s2, nested = _state(fam, sizes, C, P, pooling)
    eng = Engine(fam, sizes, C, pooling, priors, seed=3)
    eng.set_state(value, lp, ll, mu, s2)
    n_iter = 60
    eng.set_schedule(n_iter, 20, 4)
    eng.run(0, n_iter)
    eng.synchronize()
    rows = eng.samples()                       # [C, rows, cols]
    got = eng.obs_ll_rows()                    # [C, rows, n_obs]
    assert got.shape == (C, eng.n_rows, int(sum(sizes)))
    Gs = len(sizes)
    pc = 2 if pooling == "partial" else 0
    for c in (0, 1, C - 1):
        for r in (0, eng.n_rows // 2, eng.n_rows - 1):
            theta = numpy.stack([rows[c, r, q * (Gs + pc) + pc:(q + 1) * (Gs + pc)]
                                 for q in range(P)])
            want = nested.obs_ll(theta)
            assert numpy.allclose(got[c, r], want, rtol=1e-12, atol=1e-12), (kind, c, r)
    # the streamed files: one "%f" row per recorded row, chain ids as given
    ids = list(range(100, 100 + C))
    eng.write_ll_csvs(str(tmp_path), ids, threads=4)
    for c in (0, C - 1):
        lines = open(os.path.join(str(tmp_path), "logLikelihood.%d.csv" % ids[c])).read().splitlines()
        assert len(lines) == eng.n_rows
        for r in (0, eng.n_rows - 1):
            assert lines[r] == ",".join("%f" % v for v in got[c, r]), (c, r)
    eng.close()


def test_obs_ll_rows_at_final_state_equal_eval_obs_ll(gpu_lib):
    """The last recorded row is the final state when the last iteration is recorded:
    the sample-store evaluation and the current-state evaluation agree bit for bit."""
    fam, sizes, priors, pooling, names = synthetic("linreg_partial", 130, 6, 40)
    value, lp, ll, mu, s2, _ = _state(fam, sizes, 130, 2, pooling)
    eng = Engine(fam, sizes, 130, pooling, priors, seed=9)
    eng.set_state(value, lp, ll, mu, s2)
    eng.set_schedule(41, 1, 2)                 # rows at 2, 4, ..., 40 (the last iteration)
    eng.run(0, 41)
    eng.synchronize()
    a = eng.obs_ll_rows(eng.n_rows - 1, 1)[:, 0]
    b = eng.eval_obs_ll()
    assert numpy.array_equal(a, b)
    eng.close()


def test_ll_csvs_chain_batched_branch_byte_identical(gpu_lib, tmp_path, monkeypatch):
    """nmc_write_ll_csvs's second branch (one row of every chain over the batch budget:
    one row of a sub-range of the chains per batch, per-chain 'w' / 'a' opens) writes the
    one-batch run's files byte for byte.  NMC_LL_BATCH_BYTES shrinks the 256 MiB budget to
    three chains' rows, so 70 chains take 24 chain blocks x every recorded row."""
    fam, sizes, priors, pooling, names = synthetic("linreg_partial", 70, 5, 30)
    value, lp, ll, mu, s2, _ = _state(fam, sizes, 70, 2, pooling)
    eng = Engine(fam, sizes, 70, pooling, priors, seed=4)
    eng.set_state(value, lp, ll, mu, s2)
    eng.set_schedule(50, 20, 3)
    eng.run(0, 50)
    eng.synchronize()
    ids = list(range(7, 77))
    one, many = tmp_path / "one", tmp_path / "many"
    one.mkdir()
    many.mkdir()
    monkeypatch.delenv("NMC_LL_BATCH_BYTES", raising=False)
    eng.write_ll_csvs(str(one) + "/", ids, threads=4)
    monkeypatch.setenv("NMC_LL_BATCH_BYTES", str(3 * int(sum(sizes)) * 8))
    eng.write_ll_csvs(str(many) + "/", ids, threads=3)
    monkeypatch.delenv("NMC_LL_BATCH_BYTES")
    for c in ids:
        a = (one / ("logLikelihood.%d.csv" % c)).read_bytes()
        b = (many / ("logLikelihood.%d.csv" % c)).read_bytes()
        assert a == b and a.count(b"\n") == eng.n_rows, c
    eng.close()
