"""GPU parity on the geometry of BASELINE configs 4 and 5 and the kernel branches
they take (SURVEY 8(d) cfg 4/5), against the numpy oracle on the same Philox stream.

* cfg-4 shard geometry: G = 129 / 256 groups of 2000 rows -> more than one numpy
  pairwise leaf in the Gibbs update (posteriorSampling.py:481-498), persistent
  (one chain block, 256 workgroups) and launch-per-iteration (two chain blocks);
  all chains must agree bit for bit across launch modes and chain-block counts.
* cfg-5 shape: 8-parameter logistic, 5000 rows per group (rows exceed the 64 KiB
  LDS tile -> rows streamed from global memory, :615-635), P > 2 closing update.
* odd chain counts in the payload-in-LDS Gibbs mode (register fallback).
* launch-per-iteration grids larger than one residency wave.
* one-rank RCCL gather of the sample store.
Tolerances: accept flags bit-exact; values and proposal LLs within 1e-9 relative.
"""

import ctypes

import numpy
import pytest

from gpu_cases import partial_state, run_engine, run_oracle
from nestmc import data
from nestmc.families import LinearRegression, Logistic

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-9):
    return numpy.allclose(a, b, rtol=rtol, atol=1e-9, equal_nan=True)


def _check_vs_oracle(dev, nested, st, sel, chain_ids, n_iter, seed, **kw):
    acc, llp, rows, _ = dev
    oacc, ollp, orows, margin = run_oracle(nested, st, sel, chain_ids, n_iter, seed, **kw)
    bad = numpy.argwhere(acc[sel].astype(bool) != oacc)
    assert bad.size == 0, "flag mismatch at %s (min margin %g)" % (bad[:5], margin)
    assert _close(llp[sel], ollp, rtol=1e-10)
    assert _close(rows[sel], orows)


def test_cfg4_sweep_resident_batches_of_chain_blocks(gpu_lib):
    """Three chain blocks of the cfg-4 geometry (192 chains x 256 groups x 2000 rows): the
    sweep with its Gibbs kernel fits two chain blocks at a time, so each launch runs the
    chain blocks in resident batches (2 + 1) -- bit for bit nmc_k_run's single grid,
    across three launches (counters carried over)."""
    G, N, n_iter, seed, C = 256, 2000, 6, 41, 192
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, _ = partial_state(fam, sizes, C, 2)
    sel = numpy.arange(C)
    bat = run_engine(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=2)
    cfg = bat[3]
    assert cfg["kernel"].startswith("nmc_k_sweep<") and cfg["mode"] == "NMC_MODE_SYNC_OWN", cfg
    assert cfg["chain_blocks"] == 3 and cfg["chain_blocks_per_launch"] < 3, cfg
    ref = run_engine(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=2,
                     env={"NMC_SWEEP": "0"})
    assert ref[3]["kernel"].startswith("nmc_k_run<"), ref[3]
    for k in range(3):
        assert numpy.array_equal(bat[k], ref[k], equal_nan=True), k


def test_cfg4_gsep_serialized_kernels_fall_back(gpu_lib):
    """The cfg-4 shard (128 chains x 256 groups x 2000 rows) on its default path -- nmc_k_sweep
    SYNC_OWN beside its Gibbs kernel nmc_k_sweep_gibbs on a second stream -- when the two
    kernels do NOT run at the same time (as under a profiler's PMC pass): both on one stream,
    the Gibbs kernel first (it gives up after the patience and leaves) or second (it finds the
    launch taken over and leaves).  Every launch completes, the likelihood workgroups update
    the Gibbs tasks themselves, and flags, proposal LLs and recorded rows (hyper-parameters
    included) are bit for bit nmc_k_run's, over launches of 2, 2 and 1 iterations (the last
    one too short for any task to fall due inside its loop)."""
    G, N, n_iter, seed, C = 256, 2000, 5, 43, 128
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, _ = partial_state(fam, sizes, C, 2)
    sel = numpy.arange(C)
    ref = run_engine(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=2,
                     env={"NMC_SWEEP": "0"})
    assert ref[3]["kernel"].startswith("nmc_k_run<"), ref[3]
    sep = run_engine(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=2)
    assert sep[3]["kernel"].startswith("nmc_k_sweep<") and sep[3]["mode"] == "NMC_MODE_SYNC_OWN"
    assert sep[3]["gibbs_fallbacks"] == 0, sep[3]   # (the two kernels met)
    runs = {"sep": sep}
    for order in ("1", "2"):
        runs[order] = run_engine(fam, sizes, st, sel, 0, n_iter, seed, launch_iters=2,
                                 env={"NMC_GSEP_SERIAL": order, "NMC_GSEP_PATIENCE_US": "500"})
        # every (launch, chain block) fell back: 3 launches x 2 chain blocks
        assert runs[order][3]["gibbs_fallbacks"] == 6, (order, runs[order][3])
    for name, r in runs.items():
        for k in range(3):
            assert numpy.array_equal(r[k], ref[k], equal_nan=True), (name, k)


@pytest.mark.parametrize("G", [129, 256])
def test_cfg4_geometry_multileaf_gibbs(gpu_lib, G):
    N, n_iter, seed = 2000, 8, 31
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    C = 128
    st, nested = partial_state(fam, sizes, C, 2)
    # one chain block: G workgroups + P Gibbs workgroups, co-resident -> persistent
    # (nmc_k_sweep SYNC_OWN: each task computed once per chain block by its Gibbs
    # workgroup, multi-leaf plan, read by every likelihood workgroup)
    one = run_engine(fam, sizes, st, numpy.arange(64), 0, n_iter, seed)
    assert one[3]["persistent"], one[3]
    assert one[3]["kernel"].startswith("nmc_k_sweep<"), one[3]
    assert one[3]["mode"] == "NMC_MODE_SYNC_OWN", one[3]
    # nmc_k_run's all-wave update (every workgroup streams the G values after barrier A)
    syn = run_engine(fam, sizes, st, numpy.arange(64), 0, n_iter, seed, env={"NMC_SWEEP": "0"})
    assert syn[3]["mode"] == "NMC_MODE_SYNC", syn[3]
    # the sweep drawing every variate inside the kernel (NMC_ZIN=1: three queue jobs per
    # step and the Gibbs workgroups' own draws, no fill launch) on four waves
    zin = run_engine(fam, sizes, st, numpy.arange(64), 0, n_iter, seed,
                     env={"NMC_ZIN": "1", "NMC_SWEEP_WAVES": "4"})
    assert zin[3]["kernel"].startswith("nmc_k_sweep<") and zin[3]["zin"] == 1, zin[3]
    assert one[3]["zin"] == 0, one[3]
    # the same chains in a two-block launch (two 4-wave workgroups per CU, persistent) and
    # forced launch per iteration
    two = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, env={"NMC_SWEEP": "0"})
    lau = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, env={"NMC_PERSIST": "0"})
    assert not lau[3]["persistent"]
    # the sweep kernel's Gibbs workgroups over launches of 3, 3 and 2 iterations (one chain
    # block: two need more workgroups than fit with the Gibbs workgroups' LDS carve)
    swl = run_engine(fam, sizes, st, numpy.arange(64), 0, n_iter, seed, launch_iters=3)
    assert swl[3]["kernel"].startswith("nmc_k_sweep<"), swl[3]
    # two chain blocks on the sweep (the default for G > 128): at G = 256 the Gibbs
    # workgroups run as their own kernel on a second stream (Dev.gsep), co-resident with the
    # 512 likelihood workgroups
    sep = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed)
    if G == 256:
        assert sep[3]["kernel"].startswith("nmc_k_sweep<"), sep[3]
        assert sep[3]["mode"] == "NMC_MODE_SYNC_OWN", sep[3]
    for k in range(3):
        assert numpy.array_equal(two[k], sep[k], equal_nan=True), k
        assert numpy.array_equal(one[k], two[k][:64], equal_nan=True), k
        assert numpy.array_equal(one[k], zin[k], equal_nan=True), k
        assert numpy.array_equal(one[k], syn[k], equal_nan=True), k
        assert numpy.array_equal(one[k], swl[k], equal_nan=True), k
        assert numpy.array_equal(two[k], lau[k], equal_nan=True), k
    assert 0.05 < lau[0].mean() < 0.95
    # chains 0, 1 and 127 against the oracle
    sel = numpy.array([0, 1, 127])
    _check_vs_oracle(lau, nested, st, sel, sel, n_iter, seed)


def test_cfg5_logistic_p8_rows_beyond_lds(gpu_lib):
    G, N, n_iter, seed = 6, 5000, 5, 5
    X, yl, _ = data.logistic(G, N, n_coef=8, seed=1)
    fam = Logistic(X, yl)
    assert fam.n_params == 8 and fam.n_fields == 8 and N * 8 * 8 > 64 * 1024
    sizes = [N] * G
    C = 64
    st, nested = partial_state(fam, sizes, C, 8, spread=0.1)
    dev = run_engine(fam, sizes, st, numpy.arange(C), 100, n_iter, seed, tune_interval=2)
    # (S = 5 members of 1000 rows: a row split always runs persistent -- its members
    # exchange every step -- so there is no launch-per-iteration form to compare with)
    assert dev[3]["persistent"] and dev[3]["split_members"] == 5, dev[3]
    sel = numpy.array([0, 63])
    _check_vs_oracle(dev, nested, st, sel, sel + 100, n_iter, seed, tune_interval=2)
    assert dev[0].mean() > 0.02


def test_staged_rows_unsplit_launch_modes(gpu_lib):
    """Rows beyond LDS WITHOUT a row split (130 groups of 1700 5-field rows: 66 KiB per
    group, S = 1; G > 128: the multi-leaf Gibbs update): the staged-row step kernel
    persistent and launched per iteration must agree bit for bit; chains 0 and 63
    against the oracle."""
    G, N, n_iter, seed = 130, 1700, 5, 9
    X, yl, _ = data.logistic(G, N, n_coef=5, seed=4)
    fam = Logistic(X, yl)
    assert fam.n_fields == 5 and fam.n_params == 5
    sizes = [N] * G
    C = 64
    st, nested = partial_state(fam, sizes, C, 5, spread=0.1)
    dev = run_engine(fam, sizes, st, numpy.arange(C), 7, n_iter, seed, tune_interval=2)
    assert dev[3]["split_members"] == 1 and dev[3]["persistent"], dev[3]
    assert dev[3]["kernel"].endswith(", false>"), dev[3]
    lau = run_engine(fam, sizes, st, numpy.arange(C), 7, n_iter, seed, tune_interval=2,
                     env={"NMC_PERSIST": "0"})
    assert not lau[3]["persistent"], lau[3]
    for k in range(3):
        assert numpy.array_equal(dev[k], lau[k], equal_nan=True), k
    sel = numpy.array([0, 63])
    _check_vs_oracle(dev, nested, st, sel, sel + 7, n_iter, seed, tune_interval=2)
    assert dev[0].mean() > 0.02


@pytest.mark.parametrize("C", [65, 63])
def test_odd_chain_count_payload_in_lds(gpu_lib, C):
    G, N, n_iter, seed = 40, 256, 10, 77
    x, y, _, _ = data.linreg(G, N, seed=3)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, nested = partial_state(fam, sizes, C, 2)
    dev = run_engine(fam, sizes, st, numpy.arange(C), 9, n_iter, seed)
    assert dev[3]["persistent"] and dev[3]["waves_per_group"] >= 4
    sel = numpy.arange(C)
    _check_vs_oracle(dev, nested, st, sel, sel + 9, n_iter, seed)


def test_launch_mode_grid_beyond_residency(gpu_lib):
    """4096 chains x 64 groups launched per iteration (4096 workgroups, more than the
    chip holds at once): every chain block must read the hyper-parameters of the
    previous iteration, whatever dispatch wave its workgroups land in."""
    G, N, n_iter, seed = 64, 64, 8, 12
    x, y, _, _ = data.linreg(G, N, seed=5)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    C = 4096
    st, nested = partial_state(fam, sizes, C, 2)
    big = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, env={"NMC_PERSIST": "0"})
    assert not big[3]["persistent"]
    for lo in (0, C - 64):
        sel = numpy.arange(lo, lo + 64)
        small = run_engine(fam, sizes, st, sel, lo, n_iter, seed)
        for k in range(3):
            assert numpy.array_equal(big[k][sel], small[k], equal_nan=True), (lo, k)
    sel = numpy.array([0, 2047, 4095])
    _check_vs_oracle(big, nested, st, sel, sel, n_iter, seed)


def test_rccl_gather_one_rank(gpu_lib):
    from nestmc import parallel
    from nestmc.engine import Engine
    G, N, C, n_iter = 8, 50, 70, 12
    x, y, _, _ = data.linreg(G, N, seed=2)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    st, _ = partial_state(fam, sizes, C, 2)
    eng = Engine(fam, sizes, C, "partial", seed=3)
    eng.set_state(st.value, st.lp, st.ll, st.mu, st.s2)
    eng.set_schedule(n_iter, 4, 2)
    eng.run(0, n_iter)
    want = eng.samples_raw()
    comm = parallel.rccl_comm(None, 1, 0, 0)
    try:
        assert parallel.comm_size(comm) == (1, 0)
        got = parallel.gather_samples(eng, comm, root=0)
    finally:
        parallel.rccl_destroy(comm)
    eng.close()
    assert got.shape == (1,) + want.shape
    assert numpy.array_equal(got[0], want)
    # a root buffer that is too small is refused, not overrun
    from nestmc import _lib
    comm = parallel.rccl_comm(None, 1, 0, 0)
    try:
        eng = Engine(fam, sizes, C, "partial", seed=3)
        eng.set_state(st.value, st.lp, st.ll, st.mu, st.s2)
        eng.set_schedule(n_iter, 4, 2)
        small = numpy.empty(10)
        rc = _lib.load().nmc_gather_samples(eng.h, comm, 0,
                                            small.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                            small.size)
        assert rc != 0
        eng.close()
    finally:
        parallel.rccl_destroy(comm)


def test_cfg2_full_size_half_layout(gpu_lib):
    """cfg 2 (example/distribution.py:18-24 at 256 chains x 32 groups x 500 obs, no
    pooling): the 64-chain grid is 128 workgroups on 256 CUs, so the step kernel runs the
    half layout (32 chains per workgroup, NMC_MODE_HALF); flags, proposal LLs and recorded
    rows are bit-identical to the 64-chain layout, and chains 0, 1 and 255 match the oracle."""
    from gpu_cases import synthetic
    C, G, N, n_iter, seed = 256, 32, 500, 6, 13
    fam, sizes, priors, pooling, _ = synthetic("gauss_none", C, G, N)
    r = numpy.random.RandomState(4)
    from oracle import restatement as rs
    nested = rs.Nested(fam, sizes)
    value = numpy.repeat((r.normal(0, 0.3, size=(C, 3)))[:, :, None], G, axis=2)
    lp = numpy.stack([numpy.asarray(priors[p].logpdf(value[:, p, :])) for p in range(3)], 1)
    st = rs.State(value, lp, numpy.full((C, G), numpy.nan))
    half = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, pooling=pooling,
                      priors=priors)
    full = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, pooling=pooling,
                      priors=priors, env={"NMC_HALF": "0"})
    assert half[3]["mode"] == "NMC_MODE_HALF" and half[3]["chains_per_block"] == 32, half[3]
    assert full[3]["mode"] == "NMC_MODE_NOPOOL", full[3]
    # the balanced tiles (500 rows: 80-row tiles for the 7 likelihood waves) come from the
    # rows alone -- a launch with a different wave count sums the same tiles
    w4 = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed, pooling=pooling,
                    priors=priors, env={"NMC_WAVES": "4"})
    for k in range(3):
        assert numpy.array_equal(half[k], full[k], equal_nan=True), k
        assert numpy.array_equal(half[k], w4[k], equal_nan=True), k
    assert 0.05 < half[0].mean() < 0.95
    sel = numpy.array([0, 1, 255])
    _check_vs_oracle(half, nested, st, sel, sel, n_iter, seed, pooling=pooling, priors=priors)
