"""Device-batched chain initialisation (posteriorSampling.py:1060-1095
start-point search, :746-758 partial init loop): every chain's likelihoods of a round
are one nmc_eval_group_ll call on the GPU, the draws stay in each chain's
RandomState(chain) order.  Checked against the oracle's one-chain restatement
(values, log priors, hyper starts exact; group LLs within 1e-12 relative -- the device's
summation order), and timed at the cfg-4 shard size (1024 chains x 256 groups x 2000
observations): under one second.
"""

import time

import numpy
import pytest

from golden_cases import Case
from gpu_cases import family_for
from nestmc import data
from nestmc.engine import Engine
from nestmc.families import LinearRegression
from nestmc.init import init_chains
from oracle import restatement as rs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["regression3_partial", "linreg_ragged_partial",
                                  "logistic_partial", "regression_none"])
def test_device_init_matches_reference_order(gpu_lib, name):
    c = Case(name)
    fam = family_for(c)
    eng = Engine(fam, c.sizes, c.n_chains, c.pooling, c.priors)
    st = init_chains(fam, c.sizes, c.names, range(c.n_chains), c.pooling, c.priors, c.ranges,
                     c.mle, group_ll=eng.eval_group_ll)
    eng.close()
    nested = rs.Nested(c.ll, c.sizes)
    for ch in range(c.n_chains):
        o, _ = rs.init_chain(nested, c.names, ch, c.pooling, c.priors, c.ranges, c.mle)
        assert numpy.array_equal(st["value"][ch], o.value[0])
        assert numpy.array_equal(st["log_prior"][ch], o.lp[0], equal_nan=True)
        assert numpy.allclose(st["ll"][ch], o.ll[0], equal_nan=True, rtol=1e-12, atol=1e-9)
        if c.pooling == "partial":
            assert numpy.array_equal(st["mu"][ch], o.mu[0])
            assert numpy.array_equal(st["s2"][ch], o.s2[0])


def test_device_init_cfg4_shard_under_a_second(gpu_lib):
    G, N, C = 256, 2000, 1024
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    eng = Engine(fam, sizes, C, "partial")
    ranges = {"b0": [-1, 1], "b1": [0, 3]}
    init_chains(fam, sizes, ("b0", "b1"), range(4), "partial", None, ranges, False,
                group_ll=lambda th: eng.eval_group_ll(numpy.resize(th, (C, 2, G)))[:4])  # warm
    t0 = time.perf_counter()
    st = init_chains(fam, sizes, ("b0", "b1"), range(C), "partial", None, ranges, False,
                     group_ll=eng.eval_group_ll)
    dt = time.perf_counter() - t0
    eng.close()
    print("cfg-4 shard init: %.3f s for %d chains" % (dt, C))
    assert numpy.isfinite(st["ll"]).all()
    assert dt < 1.0, dt
