"""CPU-only checks of the host side: the C-ABI library loads and exports every
declared symbol (no device calls), family callbacks equal the reference-style
callbacks bit for bit, priors encode, data generators reproduce the fixtures."""

import os
import re

import numpy
import pytest
import scipy.stats

from golden_cases import Case
from nestmc import _lib, data, priors
from nestmc.families import GaussianMean, LinearRegression, Logistic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "nestmc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nmc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, "no ctypes signature for %s" % s
    assert _lib.version().startswith("nestmc")


def test_device_count_without_gpu_is_safe():
    n = _lib.device_count()
    assert n >= 0


def test_families_bit_identical_to_reference_callbacks():
    from callbacks import ll_distribution, ll_logistic, ll_regression2, ll_regression3
    r = numpy.random.RandomState(0)
    c = Case("regression_none")
    fam = LinearRegression(c.arr["X"], c.arr["y"])
    par = [r.normal(size=240), r.normal(100, 10, size=240), r.uniform(-0.5, 3, size=240)]
    assert numpy.array_equal(fam(par), ll_regression3(par, c.arr["X"], c.arr["y"]), equal_nan=True)
    c = Case("linreg_partial")
    fam = LinearRegression.simple(c.arr["x"], c.arr["y"], sigma=1.0)
    par = [r.normal(size=400), r.normal(size=400)]
    assert numpy.array_equal(fam(par), ll_regression2(par, c.arr["x"], c.arr["y"]))
    c = Case("logistic_partial")
    fam = Logistic(c.arr["X"], c.arr["y"])
    par = [r.normal(size=200) for _ in range(4)]
    assert numpy.array_equal(fam(par), ll_logistic(par, c.arr["X"], c.arr["y"]))
    c = Case("distribution_none")
    sizes = [20] * 4
    fam = GaussianMean.from_groups(c.arr["mu"], c.arr["sd"], sizes)
    par = [r.normal(size=80) for _ in range(3)]
    assert numpy.array_equal(fam(par), ll_distribution(par, c.arr["mu"], c.arr["sd"], sizes))


def test_family_layout():
    x = numpy.arange(6.0)
    y = 2 * x
    f = LinearRegression.simple(x, y, sigma=1.0)
    assert f.n_fields == 2 and f.n_params == 2 and f.intercept
    assert numpy.array_equal(f.obs(), numpy.stack([x, y], 1))
    f3 = LinearRegression(numpy.stack([numpy.ones(6), x], 1), y)
    assert f3.n_params == 3 and f3.consts()[:3] == [1.0, 1.0, 0.0]
    g = Logistic(numpy.stack([numpy.ones(6), x, x ** 2], 1), (x > 2).astype(float))
    assert g.n_params == 3 and g.n_fields == 3


def test_data_generators_reproduce_fixtures():
    c = Case("regression_complete")
    d = data.example_regression(8, 100)
    assert numpy.array_equal(d["X"], c.arr["X"]) and numpy.array_equal(d["y"], c.arr["y"])
    c = Case("linreg_partial")
    x, y, _, _ = data.linreg(8, 50)
    assert numpy.array_equal(x, c.arr["x"]) and numpy.array_equal(y, c.arr["y"])
    c = Case("distribution_none")
    mu, sd = data.example_distribution(3, 4)
    assert numpy.array_equal(mu, c.arr["mu"]) and numpy.array_equal(sd, c.arr["sd"])
    c = Case("logistic_partial")
    X, yl, _ = data.logistic(5, 40, n_coef=4)
    assert numpy.array_equal(X, c.arr["X"]) and numpy.array_equal(yl, c.arr["y"])


def test_prior_encoding():
    fam, prm = priors.encode(scipy.stats.gamma(10))
    assert fam == _lib.PRIOR["gamma"] and prm[2] == 10 and prm[1] == 1.0
    fam, prm = priors.encode(scipy.stats.norm(loc=100, scale=10))
    assert prm[:2] == [100.0, 10.0] and prm[4] == numpy.log(10.0)
    with pytest.raises(ValueError):
        priors.encode(scipy.stats.beta(2, 3))


@pytest.mark.parametrize("name", ["regression_complete", "regression_none", "regression3_partial",
                                  "linreg_partial", "linreg_ragged_partial", "distribution_none",
                                  "distribution_partial", "logistic_partial"])
def test_batched_init_matches_reference_order(name):
    """nestmc.init.init_chains advances every chain's RandomState in lock step (one
    batched likelihood call per round); the start points, MLE starts, values, log
    priors (stale ones included, :284-285) and hyper starts must equal the oracle's
    one-chain-at-a-time restatement of :1060-1141 / :725-758 exactly."""
    from gpu_cases import family_for
    from nestmc.init import init_chains
    from oracle import restatement as rs
    c = Case(name)
    st = init_chains(family_for(c), c.sizes, c.names, range(c.n_chains), c.pooling, c.priors,
                     c.ranges, c.mle)
    nested = rs.Nested(c.ll, c.sizes)
    for ch in range(c.n_chains):
        o, _ = rs.init_chain(nested, c.names, ch, c.pooling, c.priors, c.ranges, c.mle)
        assert numpy.array_equal(st["value"][ch], o.value[0])
        assert numpy.array_equal(st["log_prior"][ch], o.lp[0], equal_nan=True)
        assert numpy.allclose(st["ll"][ch], o.ll[0], equal_nan=True, rtol=1e-12, atol=0)
        if c.pooling == "partial":
            assert numpy.array_equal(st["mu"][ch], o.mu[0])
            assert numpy.array_equal(st["s2"][ch], o.s2[0])


def test_user_family_compiles_without_gpu():
    """hiprtc compiles a user log-likelihood for gfx950 on the host (no device needed);
    a broken source surfaces the compiler log; the host callable is optional."""
    import user_models
    from nestmc import _lib
    from nestmc.families import DeviceLikelihood
    fam = DeviceLikelihood(numpy.zeros((10, 3)), user_models.POISSON, 2, consts=[0.1])
    fid = fam.family_id()
    assert fid >= 100
    assert fam.family_id() == fid            # cached per process
    lib = _lib.load()
    import ctypes
    nf, npar = ctypes.c_int(), ctypes.c_int()
    assert lib.nmc_user_family_shape(fid, ctypes.byref(nf), ctypes.byref(npar)) == 0
    assert (nf.value, npar.value) == (3, 2)
    bad = DeviceLikelihood(numpy.zeros((10, 2)), "__device__ double nmc_user_loglik("
                           "const double* t, const double* r, const double* k) { return q; }", 2)
    with pytest.raises(_lib.NestmcError, match="q"):
        bad.family_id()
    with pytest.raises(TypeError):
        fam([numpy.zeros(10), numpy.zeros(10)])
