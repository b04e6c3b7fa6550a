"""GPU parity: the HIP path (through the C-ABI) against the reference and the oracle.

* replay: the reference's own variates (captured in tests/golden) drive the device;
  every accept flag must equal the reference's, the proposal group log-likelihoods
  must match within 1e-9 relative and the recorded rows within 1e-9.
* philox: device vs the numpy oracle on the same counter-based stream at sizes the
  oracle finishes in seconds (several chain blocks, ragged groups, NaN branches).
* known answers: device priors / gammainccinv / RNG transforms vs scipy and the oracle.
"""

import numpy
import pytest
import scipy.special
import scipy.stats

from golden_cases import CASES, Case
from gpu_cases import family_for, synthetic
from nestmc import priors as npriors
from nestmc.engine import Engine
from oracle import philox as ph
from oracle import restatement as rs

pytestmark = pytest.mark.gpu

RTOL = 1e-9   # log-densities / values: north_star asks <= 1e-6 relative


def close(a, b, rtol=RTOL, atol=1e-9):
    return numpy.allclose(a, b, rtol=rtol, atol=atol, equal_nan=True)


@pytest.mark.parametrize("name", CASES)
def test_replay_matches_reference(gpu_lib, name):
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
    eng.run(0, c.n_iter)
    acc, llp = eng.trace(c.n_iter)
    assert numpy.array_equal(acc.astype(numpy.int8), a["acc"]), \
        "accept flags differ at %s" % (numpy.argwhere(acc.astype(numpy.int8) != a["acc"])[:5],)
    assert close(llp, a["ll"]), numpy.nanmax(numpy.abs(llp - a["ll"]) / (1 + numpy.abs(a["ll"])))
    rows = eng.samples()
    assert rows.shape == a["rows"].shape
    assert close(rows, a["rows"])
    eng.close()


def _synthetic_state(fam, sizes, priors, pooling, C, P, G, seed=5):
    r = numpy.random.RandomState(seed)
    nested = rs.Nested(fam, sizes)
    if pooling == "partial":
        mu = r.normal(0, 0.5, size=(C, P))
        s2 = r.uniform(0.2, 1.0, size=(C, P))
        value = mu[:, :, None] + numpy.sqrt(s2)[:, :, None] * r.normal(size=(C, P, G))
        lp = rs.norm_logpdf(value, mu[:, :, None], numpy.sqrt(s2)[:, :, None])
        ll = numpy.array([nested.group_ll(value[c]) for c in range(C)])
        return rs.State(value, lp, ll, mu, s2), nested
    start = numpy.array([float(d.mean()) for d in priors])
    start = start + r.normal(0, 0.1, size=(C, P))
    value = numpy.repeat(start[:, :, None], G, axis=2)
    lp = numpy.stack([numpy.asarray(priors[p].logpdf(value[:, p, :])) for p in range(P)], 1)
    return rs.State(value, lp, numpy.full((C, G), numpy.nan)), nested


@pytest.mark.parametrize("kind,C,G,N,ragged,n_iter", [
    ("linreg_partial", 70, 9, 40, True, 120),
    ("logistic_partial", 66, 5, 30, False, 60),
    ("regression3_none", 65, 4, 25, False, 150),
    ("gauss_none", 64, 6, 20, True, 80),
    ("linreg_complete", 3, 1, 300, False, 250),
    # persistent launch, Gibbs update by auxiliary waves from LDS (W = 5, NAUX = 2)
    ("linreg_partial", 64, 64, 256, False, 24),
    # persistent launch, Gibbs update by auxiliary waves, ragged rows
    ("logistic_partial", 96, 24, 200, True, 16),
    # one parameter: the auxiliary update and the decision share a step
    ("gauss1_partial", 64, 40, 256, False, 30),
])
def test_philox_matches_oracle(gpu_lib, kind, C, G, N, ragged, n_iter):
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N, ragged=ragged)
    P = fam.n_params
    G = len(sizes)
    st, nested = _synthetic_state(fam, sizes, priors, pooling, C, P, G)
    seed = 20241015
    eng = Engine(fam, sizes, C, pooling, priors, seed=seed, chain_base=7)
    eng.set_state(st.value, st.lp, st.ll, st.mu, st.s2)
    burn, thin = n_iter // 2, 2
    eng.set_schedule(n_iter, burn, thin, tune_interval=20)
    eng.set_trace(True)
    eng.run(0, n_iter)
    acc, llp = eng.trace(n_iter)
    rows = eng.samples()
    eng.close()

    trace, rec = {}, []
    rs.run(nested, st, pooling, priors, n_iter, burn, thin,
           rs.PhiloxRNG(numpy.arange(C) + 7, seed), tune_interval=20, trace=trace, record=rec)
    oacc = numpy.stack(trace["acc"], 1).reshape(C, n_iter, P, G)
    ollp = numpy.stack(trace["llp"], 1).reshape(C, n_iter, P, G)
    margin = numpy.min(numpy.stack(trace["margin"]))
    bad = numpy.argwhere(acc.astype(bool) != oacc)
    assert bad.size == 0, "flag mismatch at %s (min decision margin %g)" % (bad[:5], margin)
    assert close(llp, ollp, rtol=1e-10)
    orows = numpy.stack([r for _, r in rec], 1)
    assert close(rows, orows, rtol=1e-9)
    # the chain must actually move
    assert acc.mean() > 0.02


def test_rng_matches_oracle(gpu_lib):
    import ctypes
    n = 4096
    r = numpy.random.RandomState(1)
    ctr = numpy.stack([r.randint(0, 5000, n), r.randint(0, 300, n), r.randint(0, 16, n),
                       r.randint(0, 4, n), r.randint(0, 100000, n)], 1).astype(numpy.uint32)
    out = numpy.empty((n, 4))
    seed, a = 99, 31.5
    rc = gpu_lib.nmc_debug_rng(ctr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, seed, a,
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    assert rc == 0
    ua, ub = ph.uniforms(ctr[:, 0], ctr[:, 1], ctr[:, 2], ctr[:, 3], ctr[:, 4], seed)
    assert numpy.array_equal(out[:, 1], ua) and numpy.array_equal(out[:, 2], ub)
    z = ph.box_muller(ua, ub)
    assert numpy.allclose(out[:, 0], z, rtol=1e-14, atol=1e-15)
    g = numpy.array([ph.gamma_mt(a, int(ctr[i, 0]), int(ctr[i, 2]), numpy.array([ctr[i, 4]]),
                                 seed)[0] for i in range(256)])
    assert numpy.allclose(out[:256, 3], g, rtol=1e-13)


def test_priors_match_scipy(gpu_lib):
    import ctypes
    x = numpy.array([-5.0, -1.0, -1e-12, 0.0, 1e-12, 0.3, 1.0, 2.5, 9.0, 120.0, numpy.inf,
                     -numpy.inf, numpy.nan])
    dists = [scipy.stats.norm(0, 10), scipy.stats.norm(100, 10), scipy.stats.gamma(10),
             scipy.stats.gamma(0.5, loc=-1, scale=2), scipy.stats.gamma(1.0),
             scipy.stats.uniform(-1, 3), scipy.stats.expon(scale=2), scipy.stats.halfnorm(scale=3),
             scipy.stats.cauchy(1, 2), scipy.stats.laplace(0, 1.5), scipy.stats.lognorm(0.7),
             scipy.stats.invgamma(3.0, scale=2)]
    for d in dists:
        fam, prm = npriors.encode(d)
        prm = numpy.array(prm)
        out = numpy.empty_like(x)
        rc = gpu_lib.nmc_debug_prior_logpdf(fam, prm.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                            x.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                            len(x), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        assert rc == 0
        with numpy.errstate(all="ignore"):
            want = d.logpdf(x)
        fin = numpy.isfinite(want)
        assert numpy.array_equal(numpy.isnan(out), numpy.isnan(want)), (d.dist.name, out, want)
        assert numpy.array_equal(out[~fin & ~numpy.isnan(want)], want[~fin & ~numpy.isnan(want)])
        assert numpy.allclose(out[fin], want[fin], rtol=1e-13, atol=1e-13), (d.dist.name, out, want)


def test_igamci_matches_scipy(gpu_lib):
    import ctypes
    a = numpy.repeat([0.5, 1.5, 3.5, 15.5, 31.5, 63.5, 127.5, 511.5], 12)
    q = numpy.tile([1e-12, 1e-6, 1e-3, 0.05, 0.25, 0.5, 0.6, 0.75, 0.95, 0.999, 1 - 1e-9, 0.123456], 8)
    lga = scipy.special.gammaln(a)
    out = numpy.empty_like(a)
    P = lambda v: v.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    assert gpu_lib.nmc_debug_igamci(P(a), P(q), P(lga), len(a), P(out)) == 0
    want = scipy.special.gammainccinv(a, q)
    assert numpy.allclose(out, want, rtol=1e-12, atol=0), numpy.max(numpy.abs(out / want - 1))


def test_eval_group_ll_matches_oracle(gpu_lib):
    fam, sizes, priors, pooling, names = synthetic("logistic_partial", 70, 7, 33, ragged=True)
    C, P, G = 70, fam.n_params, len(sizes)
    theta = numpy.random.RandomState(2).normal(0, 0.4, size=(C, P, G))
    eng = Engine(fam, sizes, C, pooling)
    got = eng.eval_group_ll(theta)
    nested = rs.Nested(fam, sizes)
    want = numpy.array([nested.group_ll(theta[c]) for c in range(C)])
    assert numpy.allclose(got, want, rtol=1e-11)
    eng.close()


@pytest.mark.parametrize("kind,C,G,N,ragged,n_iter", [
    ("linreg_partial", 70, 9, 40, True, 40),        # asm row loop, ragged, odd chain count
    ("logistic_partial", 66, 5, 30, False, 30),     # generic loop, 4 fields (R = 2)
    ("regression3_none", 65, 4, 25, False, 40),     # asm loop, sigma sampled, no pooling
    ("gauss_none", 64, 6, 20, True, 30),            # generic loop, 3 fields
    ("linreg_partial", 64, 64, 256, False, 12),     # register Gibbs hand-off, G = 64
    ("linreg_partial", 130, 100, 48, True, 12),     # LDS Gibbs payload, 64 < G <= 128
    ("logistic_partial", 96, 24, 200, True, 10),    # tails in every group
])
def test_paired_rows_bit_identical(gpu_lib, kind, C, G, N, ragged, n_iter):
    """The paired-chain row loop (each lane evaluates its row pair half for its own chain
    and for lane ^ 32's, kernels.h nmc_ll_rows_lds<Fam, true>) and, for {x, y} rows, the
    quad-chain loop (each lane evaluates rows 4m+q for the four chains of its quarter
    position, nmc_ll_rows_lds_quad; the default) reproduce the one-chain broadcast loop bit
    for bit: flags, proposal LLs and recorded rows; so does the 64-chain layout where none
    pooling runs the half layout."""
    from gpu_cases import run_engine
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N, ragged=ragged)
    P = fam.n_params
    st, _ = _synthetic_state(fam, sizes, priors, pooling, C, P, len(sizes))
    runs = {}
    envs = {"paired": {"NMC_ROWS": "paired"}, "bcast": {"NMC_ROWS": "bcast"},
            "pair": {"NMC_ROWS": "pair"},     # the paired loop where the quad loop is default
            # none pooling on few workgroups runs the half layout (32 chains per workgroup,
            # lane pairs on the two row parities); this keeps 64 chains per workgroup
            "full": {"NMC_HALF": "0"}}
    for name, env in envs.items():
        runs[name] = run_engine(fam, sizes, st, numpy.arange(C), 5, n_iter, 777, pooling=pooling,
                                priors=priors, env=env, tune_interval=7)
    if pooling != "partial":
        assert runs["paired"][3]["mode"] == "NMC_MODE_HALF", runs["paired"][3]
        assert runs["full"][3]["mode"] == "NMC_MODE_NOPOOL", runs["full"][3]
    assert runs["paired"][3]["kernel"].startswith("nmc_k_run<"), runs["paired"][3]
    assert runs["paired"][3]["zin"] == 0, runs["paired"][3]
    for k in range(3):
        assert numpy.array_equal(runs["paired"][k], runs["bcast"][k], equal_nan=True), k
        assert numpy.array_equal(runs["paired"][k], runs["full"][k], equal_nan=True), k
        assert numpy.array_equal(runs["paired"][k], runs["pair"][k], equal_nan=True), k
    assert runs["paired"][0].mean() > 0.02
