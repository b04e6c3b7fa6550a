"""nmc_k_duo (csrc/duo.h): the barrier-free partial-pooling step kernel, two half blocks of
32 chains per workgroup stepping on their own, quad row layout.

Every sum is bit-identical to nmc_k_run's (same tiles, same residue accumulators, same
order), so the two kernels must agree bit for bit -- accept flags, proposal LLs, recorded
rows -- on the same inputs; and both agree with the numpy oracle on the Philox stream
(flags exact, values within 1e-9).  Cases: cfg 3 at full size (several launches per run),
ragged groups with empty ones and a chain count that leaves a half block empty, P = 1 (no
intercept) and P = 3 (sigma sampled: NaN likelihoods when a proposal is negative).
"""

import numpy
import pytest

from gpu_cases import partial_state, run_engine, run_oracle
from nestmc import data
from nestmc.families import LinearRegression

pytestmark = pytest.mark.gpu
DUO = {"NMC_DUO": "1"}   # (opt-in: measured slower than nmc_k_run, profiles/r05_duo)


def _same(a, b):
    for k in range(3):
        assert numpy.array_equal(a[k], b[k], equal_nan=True), k


def _oracle_check(dev, nested, st, n, n_iter, seed, tune_interval=5):
    acc, llp, rows, _ = run_oracle(nested, st, numpy.arange(n), numpy.arange(n), n_iter, seed,
                                   tune_interval=tune_interval)
    assert numpy.array_equal(dev[0][:n].astype(bool), acc)
    assert numpy.allclose(dev[1][:n], llp, rtol=1e-9, atol=1e-9, equal_nan=True)
    assert numpy.allclose(dev[2][:n], rows, rtol=1e-9, atol=1e-9, equal_nan=True)


def test_duo_cfg3_full_size_matches_run_and_oracle(gpu_lib):
    C, G, N, n_iter, seed = 256, 64, 1000, 12, 7
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, nested = partial_state(fam, sizes, C, 2)
    sel = numpy.arange(C)
    duo = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env=DUO)
    assert duo[3]["kernel"] == "nmc_k_duo<FamLinreg<2>>", duo[3]
    assert duo[3]["mode"] == "NMC_MODE_DUO" and duo[3]["persistent"], duo[3]
    run = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_DUO": "0"})
    assert run[3]["kernel"].startswith("nmc_k_run<"), run[3]
    _same(duo, run)
    # launches of 5, 5 and 2 iterations: closing Gibbs tasks and counters carried over
    multi = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env=DUO, launch_iters=5)
    _same(duo, multi)
    # six waves (two likelihood waves)
    six = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env=dict(DUO, NMC_DUO_WAVES="6"))
    assert six[3]["waves_per_group"] == 6, six[3]
    _same(duo, six)
    assert 0.05 < duo[0].mean() < 0.95
    _oracle_check(duo, nested, st, 3, n_iter, seed)


@pytest.mark.parametrize("C", [80, 17])
def test_duo_ragged_groups_partial_blocks(gpu_lib, C):
    """Ragged groups (some empty), G = 37 (the Gibbs sum's 8-block tail), chain counts that
    leave half blocks partly or wholly empty (80 = 64 + 16; 17)."""
    r = numpy.random.RandomState(5)
    G = 37
    sizes = [int(v) for v in r.randint(0, 300, size=G)]
    sizes[3], sizes[7], sizes[11], sizes[20] = 0, 5, 16, 1000   # empty, tail only, one block
    n = sum(sizes)
    grp = numpy.repeat(numpy.arange(G), sizes)
    x = r.normal(size=n)
    y = r.normal(size=G)[grp] + r.normal(2, 1, size=G)[grp] * x + r.normal(size=n)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    P, n_iter, seed = fam.n_params, 14, 91
    st, nested = partial_state(fam, sizes, C, P, seed=4)
    sel = numpy.arange(C)
    duo = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env=DUO, launch_iters=6)
    assert duo[3]["mode"] == "NMC_MODE_DUO", duo[3]
    run = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_DUO": "0"}, launch_iters=6)
    _same(duo, run)
    _oracle_check(duo, nested, st, 4, n_iter, seed)
    # the last chains (the second chain block's half) against the oracle too
    lo = C - 2
    acc, llp, rows, _ = run_oracle(nested, st, numpy.arange(lo, C), numpy.arange(lo, C),
                                   n_iter, seed)
    assert numpy.array_equal(duo[0][lo:].astype(bool), acc)
    assert numpy.allclose(duo[2][lo:], rows, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("kind", ["P1", "P3"])
def test_duo_parameter_counts(gpu_lib, kind):
    """P = 1 (slope only: every step proposes the parameter the last one decided) and P = 3
    (sigma sampled under partial pooling: negative proposals give NaN likelihoods, the
    reference's non-finite branches)."""
    r = numpy.random.RandomState(12)
    G, N, C, n_iter, seed = 24, 90, 96, 16, 33
    sizes = [N] * G
    x = r.normal(size=G * N)
    grp = numpy.repeat(numpy.arange(G), N)
    y = 0.3 + (1.5 + 0.3 * r.normal(size=G))[grp] * x + r.normal(size=G * N) * 0.8
    if kind == "P1":
        fam = LinearRegression(x[:, None], y, sigma=0.8)
    else:
        fam = LinearRegression(numpy.vstack([numpy.ones_like(x), x]).T, y)
    P = fam.n_params
    assert P == (1 if kind == "P1" else 3)
    st, nested = partial_state(fam, sizes, C, P, seed=6, spread=0.5)
    if kind == "P3":   # sigma around 0.8, a few chains near 0
        st.value[:, 2, :] = numpy.abs(st.value[:, 2, :]) * 0.5 + 0.3
        st.mu[:, 2] = 0.8
        st.ll[:] = numpy.array([nested.group_ll(st.value[c]) for c in range(C)])
    sel = numpy.arange(C)
    duo = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env=DUO)
    assert duo[3]["mode"] == "NMC_MODE_DUO", duo[3]
    run = run_engine(fam, sizes, st, sel, 0, n_iter, seed, env={"NMC_DUO": "0"})
    _same(duo, run)
    _oracle_check(duo, nested, st, 3, n_iter, seed)
