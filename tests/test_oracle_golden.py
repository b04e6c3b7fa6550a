"""Pin the oracle: the numpy restatement against fixtures captured from the reference.

* legacy-RNG mode must reproduce the reference's sample.<chain>.csv byte for byte
  (the reference's own numpy MT19937 stream, init, MLE and tuning included);
* replay mode (variates captured from the reference) must reproduce every accept
  flag and the full-precision recorded rows;
* scipy known answers and the Philox KATs hold.
"""

import filecmp
import os

import numpy
import pytest
import scipy.special

from golden_cases import CASES, GOLDEN, Case
from oracle import philox as ph
from oracle import restatement as rs


@pytest.mark.parametrize("name", CASES)
def test_legacy_byte_exact(name, tmp_path):
    c = Case(name)
    if name == "regression_complete":
        pytest.importorskip("scipy.optimize")
    rs.sample_posterior_legacy(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups,
                               c.n_per_group, c.pooling, c.ll, str(tmp_path),
                               priors=c.priors, mle=c.mle, ranges=c.ranges)
    for ch in range(c.n_chains):
        mine = os.path.join(str(tmp_path), "sample", "sample.%i.csv" % ch)
        assert filecmp.cmp(mine, c.csv_path(ch), shallow=False), (name, ch)


@pytest.mark.parametrize("name", [n for n in CASES if n != "regression_complete"])
def test_replay_flags_and_rows(name):
    c = Case(name)
    a = c.arr
    nested = rs.Nested(c.ll, c.sizes)
    partial = c.pooling == "partial"
    st = rs.State(a["init_value"], a["init_lp"], a["init_ll"][:, 0, :],
                  a.get("init_mu"), a.get("init_s2"))
    burn, thin = rs.schedule(c.n_iter, c.n_samples)
    rows, trace = [], {}
    rng = rs.ReplayRNG(a["z"], a["u"], a["hz"], a["hu"])
    rs.run(nested, st, c.pooling, c.priors, c.n_iter, burn, thin, rng, record=rows,
           trace=trace)
    acc = numpy.stack(trace["acc"], axis=1).reshape(a["acc"].shape)
    assert numpy.array_equal(acc.astype(numpy.int8), a["acc"])
    llp = numpy.stack(trace["llp"], axis=1).reshape(a["ll"].shape)
    assert numpy.array_equal(llp, a["ll"], equal_nan=True)
    got = numpy.stack([r for _, r in rows], axis=1)
    assert got.shape == a["rows"].shape
    assert numpy.array_equal(got, a["rows"], equal_nan=True)
    assert [i for i, _ in rows] == list(a["row_index"])
    del partial


def test_init_state_matches_reference():
    for name in CASES:
        c = Case(name)
        nested = rs.Nested(c.ll, c.sizes)
        for ch in range(c.n_chains):
            st, _ = rs.init_chain(nested, c.names, ch, c.pooling, c.priors, c.ranges, c.mle)
            assert numpy.array_equal(st.value[0], c.arr["init_value"][ch])
            assert numpy.array_equal(st.lp[0], c.arr["init_lp"][ch], equal_nan=True)
            assert numpy.array_equal(st.ll[0], c.arr["init_ll"][ch][0], equal_nan=True)


def test_known_answers():
    k = numpy.load(os.path.join(GOLDEN, "known_answers.npz"))
    x = k["x"]
    for (loc, scale), want in zip(k["norm_params"], k["norm_logpdf"]):
        with numpy.errstate(all="ignore"):
            got = rs.norm_logpdf(x, loc, scale)
        assert numpy.array_equal(got, want, equal_nan=True), (loc, scale)
    got = scipy.special.gammainccinv(k["igamci_a"][:, None], k["igamci_q"][None, :])
    assert numpy.array_equal(got, k["igamci"])
    for n_iter, n_samples, burn, thin, n_rows in k["schedule"]:
        assert rs.schedule(n_iter, n_samples) == (burn, thin)
        assert len(rs.record_iterations(n_iter, burn, thin)) == n_rows


def test_philox_kat():
    """Random123 known-answer vectors for philox4x32-10."""
    kat = [((0, 0, 0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 6, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for inp, out in kat:
        assert tuple(int(v) for v in ph.philox4x32_10(*inp)) == out


def test_pairwise_sum_is_numpy_sum():
    r = numpy.random.RandomState(3)
    for n in list(range(1, 140)) + [255, 256, 257, 1000, 1031]:
        a = r.standard_normal(n) * 10 ** r.uniform(-3, 3, n)
        assert rs.pairwise_sum(a) == numpy.sum(a)


def test_philox_gamma_distribution():
    """The Marsaglia-Tsang hyper draw is Gamma(a): KS test against scipy."""
    import scipy.stats
    for a in (0.5, 3.5, 31.5):
        x = ph.gamma_mt(a, 5, 1, numpy.arange(20000), 1234)
        assert scipy.stats.kstest(x, scipy.stats.gamma(a).cdf).pvalue > 1e-3
