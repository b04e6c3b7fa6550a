"""GPU: user-supplied device log-likelihoods (north_star "user log-likelihood", cfg 5
"user-supplied"; the reference's plug-in point logLikelihoodFunction,
posteriorSampling.py:61-102), compiled at run time with hiprtc (csrc/user.hip).

* a logistic model written as a user function with FamLogistic's own expression runs
  bit-identical to the built-in Logistic family (partial pooling, register Gibbs
  hand-off; no pooling), including the per-observation LL rows of saveLogLikelihood;
* a model no built-in family covers (Poisson regression with an exposure constant)
  matches the numpy oracle driving the same model's host callable on the same Philox
  stream (flags exact, LLs and rows within 1e-9 relative), partial and no pooling;
* the drop-in API: samplePosterior with a DeviceLikelihood writes the same sample CSVs
  as with the built-in family.
"""

import os

import numpy
import pytest
import scipy.stats

import user_models
from gpu_cases import run_engine, run_oracle, synthetic
from nestmc.families import DeviceLikelihood
from test_gpu_parity import _synthetic_state, close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pooling,C,G,N,n_iter", [
    ("partial", 66, 5, 30, 30),
    ("partial", 64, 24, 200, 12),
    ("none", 70, 6, 40, 25),
])
def test_user_logistic_bit_identical_to_builtin(gpu_lib, pooling, C, G, N, n_iter):
    fam, sizes, _, _, _ = synthetic("logistic_partial", C, G, N)
    assert fam.n_fields == 4 and fam.n_params == 4
    user = DeviceLikelihood(fam.obs(), user_models.LOGISTIC4, 4, host_function=fam)
    priors = None if pooling == "partial" else [scipy.stats.norm(0, 1)] * 4
    st, _ = _synthetic_state(fam, sizes, priors, pooling, C, 4, len(sizes))
    a = run_engine(fam, sizes, st, numpy.arange(C), 3, n_iter, 31, pooling=pooling,
                   priors=priors, tune_interval=7)
    b = run_engine(user, sizes, st, numpy.arange(C), 3, n_iter, 31, pooling=pooling,
                   priors=priors, tune_interval=7)
    for k in range(3):
        assert numpy.array_equal(a[k], b[k], equal_nan=True), k
    assert a[0].mean() > 0.02


@pytest.mark.parametrize("pooling,C,G,N,n_iter", [
    ("partial", 70, 8, 50, 30),
    ("none", 65, 5, 60, 30),
])
def test_user_poisson_matches_oracle(gpu_lib, pooling, C, G, N, n_iter):
    x, y = user_models.poisson_data(G, N)
    le = 0.1
    fam = DeviceLikelihood(user_models.poisson_rows(x, y), user_models.POISSON, 2, consts=[le],
                           host_function=user_models.poisson_host(x, y, le))
    sizes = [N] * G
    priors = None if pooling == "partial" else [scipy.stats.norm(0, 2)] * 2
    st, nested = _synthetic_state(fam, sizes, priors, pooling, C, 2, G)
    seed = 555
    acc, llp, rows, cfg = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed,
                                     pooling=pooling, priors=priors, tune_interval=5)
    n = 3
    oacc, ollp, orows, margin = run_oracle(nested, st, numpy.arange(n), numpy.arange(n), n_iter,
                                           seed, pooling=pooling, priors=priors, tune_interval=5)
    bad = numpy.argwhere(acc[:n].astype(bool) != oacc)
    assert bad.size == 0, "flag mismatch at %s (min decision margin %g)" % (bad[:5], margin)
    assert close(llp[:n], ollp, rtol=1e-10)
    assert close(rows[:n], orows)
    assert acc.mean() > 0.02


@pytest.mark.parametrize("G,S", [(64, 4), (128, 2)])
def test_cfg5_user_logistic8_staged_rows(gpu_lib, G, S):
    """BASELINE cfg 5 as stated: a USER-supplied 8-parameter logistic, 5000 rows per group,
    partial pooling, at group counts where each row-split member's chunk (G = 64: S = 4
    members of 1250 rows; G = 128, the cfg-5 shard: S = 2 of 2500 rows; 64 B per row)
    exceeds the LDS row area, so the staged-row instances nmc_k_run<FamUser, m, false>
    run (a row split is always persistent: its members exchange every step).  Bit-identical
    to the built-in Logistic on every chain; chains 0 and 63 against the oracle."""
    from gpu_cases import partial_state
    from nestmc import data
    from nestmc.families import Logistic
    N, n_iter, seed, C = 5000, 4, 5, 64
    X, yl, _ = data.logistic(G, N, n_coef=8, seed=1)
    fam = Logistic(X, yl)
    assert fam.n_params == 8 and fam.n_fields == 8
    user = DeviceLikelihood(fam.obs(), user_models.LOGISTIC8, 8, host_function=fam)
    sizes = [N] * G
    st, nested = partial_state(fam, sizes, C, 8, spread=0.1)
    a = run_engine(fam, sizes, st, numpy.arange(C), 100, n_iter, seed, tune_interval=2)
    b = run_engine(user, sizes, st, numpy.arange(C), 100, n_iter, seed, tune_interval=2)
    cfg = b[3]
    assert cfg["split_members"] == S and cfg["persistent"], cfg
    assert cfg["kernel"].startswith("nmc_k_run<FamUser, NMC_MODE_SYNC"), cfg
    assert cfg["kernel"].endswith(", false>"), cfg   # rows staged from global memory
    for k in range(3):
        assert numpy.array_equal(a[k], b[k], equal_nan=True), k
    sel = numpy.array([0, 63])
    oacc, ollp, orows, margin = run_oracle(nested, st, sel, sel + 100, n_iter, seed,
                                           tune_interval=2)
    bad = numpy.argwhere(b[0][sel].astype(bool) != oacc)
    assert bad.size == 0, "flag mismatch at %s (min margin %g)" % (bad[:5], margin)
    assert close(b[1][sel], ollp, rtol=1e-10)
    assert close(b[2][sel], orows)
    assert b[0].mean() > 0.02


def test_user_family_through_sample_posterior(gpu_lib, tmp_path):
    import posteriorSampling
    fam, sizes, _, _, _ = synthetic("logistic_partial", 4, 6, 25)
    user = DeviceLikelihood(fam.obs(), user_models.LOGISTIC4, 4, host_function=fam)
    names = ("t0", "t1", "t2", "t3")
    ranges = dict((k, [-0.5, 0.5]) for k in names)
    out = {}
    for tag, f in (("builtin", fam), ("user", user)):
        d = str(tmp_path / tag)
        posteriorSampling.samplePosterior(4, 60, 20, names, 6, 25, "partial", f, d,
                                          saveLogLikelihood=True,
                                          startingPointValueRange=ranges, displayProgress=False)
        out[tag] = d
    files = sorted(os.listdir(os.path.join(out["builtin"], "sample")))
    assert sum(f.startswith("sample.") for f in files) == 4
    for fn in files:
        a = open(os.path.join(out["builtin"], "sample", fn)).read()
        b = open(os.path.join(out["user"], "sample", fn)).read()
        if fn.startswith("sample."):
            assert a == b, fn
        else:   # per-observation LL rows: the user function's fma chain vs the reference's
                # numpy row sum in the built-in obs_ll -- equal to rounding
            va = numpy.array([[float(v) for v in ln.split(",")] for ln in a.split()])
            vb = numpy.array([[float(v) for v in ln.split(",")] for ln in b.split()])
            assert va.shape == vb.shape and numpy.allclose(va, vb, atol=2e-6), fn
