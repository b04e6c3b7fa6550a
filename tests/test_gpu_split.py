"""GPU: row-split none/complete pooling (reference CompletePooling
posteriorSampling.py:662-685 -- every observation in ONE group, so one (chain, group)
is a single workgroup's worth of chains over the whole dataset).

Groups much larger than one workgroup's 64 KiB LDS row area are shared by S member
workgroups (kernels.h nmc_split_exchange): each owns a contiguous row chunk, the
members exchange their partial sums every step and all make the same decision.

* complete pooling at n_total = 120 000 rows and none pooling with four 20 000-row
  groups against the numpy oracle on the same Philox stream (flags exact, proposal LLs
  within 1e-9 relative, recorded rows within 1e-9);
* the split's order depends on (rows, fields, groups) only: two engines
  holding halves of the chains, and chain blocks launched one per resident batch,
  reproduce the one-engine run bit for bit.
"""

import numpy
import pytest

from gpu_cases import run_engine, run_oracle, synthetic
from test_gpu_parity import _synthetic_state, close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,C,G,N,n_iter", [
    ("linreg_complete", 70, 1, 120000, 16),
    ("regression3_none", 65, 4, 20000, 12),
])
def test_split_matches_oracle(gpu_lib, kind, C, G, N, n_iter):
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N)
    P = fam.n_params
    st, nested = _synthetic_state(fam, sizes, priors, pooling, C, P, len(sizes))
    seed = 4242
    acc, llp, rows, cfg = run_engine(fam, sizes, st, numpy.arange(C), 11, n_iter, seed,
                                     pooling=pooling, priors=priors, tune_interval=5)
    assert cfg["split_members"] > 1, cfg
    n = 3
    oacc, ollp, orows, margin = run_oracle(nested, st, numpy.arange(n), numpy.arange(n) + 11,
                                           n_iter, seed, pooling=pooling, priors=priors,
                                           tune_interval=5)
    bad = numpy.argwhere(acc[:n].astype(bool) != oacc)
    assert bad.size == 0, "flag mismatch at %s (min decision margin %g)" % (bad[:5], margin)
    assert close(llp[:n], ollp, rtol=1e-10)
    assert close(rows[:n], orows)
    assert acc.mean() > 0.02


def test_split_shard_and_batch_invariance(gpu_lib):
    fam, sizes, priors, pooling, names = synthetic("linreg_complete", 130, 1, 30000)
    C, P = 130, fam.n_params
    st, _ = _synthetic_state(fam, sizes, priors, pooling, C, P, 1)
    args = dict(pooling=pooling, priors=priors, tune_interval=5)
    whole = run_engine(fam, sizes, st, numpy.arange(C), 0, 10, 99, **args)
    assert whole[3]["split_members"] > 1, whole[3]
    lo = run_engine(fam, sizes, st, numpy.arange(0, 64), 0, 10, 99, **args)
    hi = run_engine(fam, sizes, st, numpy.arange(64, C), 64, 10, 99, **args)
    batched = run_engine(fam, sizes, st, numpy.arange(C), 0, 10, 99,
                         env={"NMC_SPLIT_BATCH": "1"}, **args)
    assert batched[3]["chain_blocks_per_launch"] == 1, batched[3]
    for k in range(3):
        merged = numpy.concatenate([lo[k], hi[k]], axis=0)
        assert numpy.array_equal(merged, whole[k], equal_nan=True), k
        assert numpy.array_equal(batched[k], whole[k], equal_nan=True), k


def test_split_ragged_and_empty_groups(gpu_lib):
    """Members whose chunk of a small group is empty, and an empty group, under the split
    (S fixed by the largest group): against the oracle."""
    import scipy.stats
    from nestmc.families import LinearRegression
    r = numpy.random.RandomState(8)
    sizes = [30000, 5, 0, 17000]
    n = sum(sizes)
    x = r.normal(size=n)
    y = 1.0 + 3.0 * x + r.normal(size=n) * 0.7
    fam = LinearRegression(numpy.vstack([numpy.ones(n), x]).T, y)
    priors = [scipy.stats.norm(0, 10), scipy.stats.norm(3, 10), scipy.stats.gamma(2)]
    C, P = 66, 3
    st, nested = _synthetic_state(fam, sizes, priors, "none", C, P, len(sizes))
    acc, llp, rows, cfg = run_engine(fam, sizes, st, numpy.arange(C), 0, 12, 21, pooling="none",
                                     priors=priors, tune_interval=5)
    assert cfg["split_members"] > 5, cfg
    oacc, ollp, orows, margin = run_oracle(nested, st, numpy.arange(3), numpy.arange(3), 12, 21,
                                           pooling="none", priors=priors, tune_interval=5)
    assert numpy.array_equal(acc[:3].astype(bool), oacc), margin
    assert close(llp[:3], ollp, rtol=1e-10)
    assert close(rows[:3], orows)
