"""CPU: the spawn and shard plumbing of samplePosterior(process_per_device=True)
(nestmc.ranks; the reference's process fan-out, posteriorSampling.py:182-201, at the GPU
level).  A dry run starts the ranks for real -- child processes with the torchrun-style
environment -- and each reports its shard and exits before any HIP call; the GPU form is
tests/test_gpu_multi.py::test_process_per_device_one_rank_byte_identical."""

import pickle

import numpy
import pytest

from nestmc import _lib, data, ranks
from nestmc.families import LinearRegression
from nestmc.parallel import padded_shard


def _kw(n_chains):
    x, y, _, _ = data.linreg(4, 10, seed=1)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    return dict(nChains=n_chains, nIter=10, nSamples=5, parameterName=("b0", "b1"), nGroups=4,
                nResponsesPerGroup=10, pooling="partial", logLikelihoodFunction=fam,
                outputDirectory="/nonexistent", displayProgress=False)


@pytest.mark.parametrize("n_chains,world", [(70, 3), (8, 8), (5, 4), (1, 2)])
def test_dry_run_ranks_and_shards(n_chains, world):
    devs = list(range(world))[::-1]   # rank r -> devices[r], whatever the ids
    out = ranks.run_per_device(_kw(n_chains), devs, dry_run=True, timeout=120)
    assert [o["rank"] for o in out] == list(range(world))
    assert all(o["world"] == world for o in out)
    assert [o["device"] for o in out] == devs
    assert len({o["bootstrap_port"] for o in out}) == 1
    assert not any(o["libnestmc_mapped"] for o in out)     # no HIP before the real run
    # equal-size contiguous stores (the RCCL gather), the real chains tiling [0, n) once
    per = {o["chains"] for o in out}
    assert len(per) == 1
    covered = []
    for o in out:
        assert o["chain_base"] == o["rank"] * o["chains"]
        covered += list(range(o["chain_base"], o["chain_base"] + o["real"]))
        assert (o["chain_base"], o["chains"], o["real"]) == padded_shard(n_chains, world,
                                                                        o["rank"])
    assert covered == list(range(n_chains))


def test_failed_rank_fails_the_run():
    kw = _kw(10)
    del kw["nChains"]            # every rank raises before it reports
    with pytest.raises(_lib.NestmcError, match="ranks failed"):
        ranks.run_per_device(kw, [0, 1], dry_run=True, timeout=120)


def test_call_pickles_for_the_ranks():
    kw = _kw(3)
    back = pickle.loads(pickle.dumps(kw))
    fam, fam2 = kw["logLikelihoodFunction"], back["logLikelihoodFunction"]
    th = numpy.array([[0.1] * 40, [0.5] * 40])
    assert numpy.array_equal(fam(th), fam2(th))


def test_interrupted_parent_leaves_no_rank(monkeypatch):
    """Ctrl-C (any exception) in the parent's wait kills every rank before it propagates."""
    import os
    import signal
    monkeypatch.setenv(ranks._DRY_HOLD_S, "60")      # the dry-run ranks sleep a minute

    def _interrupt(signum, frame):
        raise KeyboardInterrupt
    old = signal.signal(signal.SIGALRM, _interrupt)
    try:
        signal.setitimer(signal.ITIMER_REAL, 1.5)
        with pytest.raises(KeyboardInterrupt):
            ranks.run_per_device(_kw(4), [0, 1], dry_run=True, timeout=120)
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)
        signal.signal(signal.SIGALRM, old)
    assert len(ranks.last_pids) == 2
    for pid in ranks.last_pids:     # killed and reaped: no such process any more
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_main_script_callable_refused_before_spawn():
    """A host_function defined in the caller's script cannot be unpickled by the ranks: the
    parent refuses it with a clear error instead of N rank tracebacks."""
    from nestmc.families import DeviceLikelihood

    def computeLogLikelihood(parameter):
        return numpy.zeros(parameter.shape[1])
    computeLogLikelihood.__module__ = "__main__"     # as if defined in the user's script
    kw = _kw(4)
    kw["logLikelihoodFunction"] = DeviceLikelihood(
        numpy.zeros((40, 2)), "__device__ double nmc_user_loglik(const double* t, "
        "const double* r, const double* k) { return 0.0; }", 2,
        host_function=computeLogLikelihood)
    del ranks.last_pids[:]
    with pytest.raises(ValueError, match="__main__"):
        ranks.run_per_device(kw, [0, 1], dry_run=True, timeout=120)
    assert ranks.last_pids == []     # nothing was started


def test_bench_spawn_waits_for_every_rank():
    """bench.py's rank spawn polls every rank and stops the rest on the first failure
    (nestmc.ranks.wait_all)."""
    import subprocess
    import sys
    import time
    ok = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"],
                          start_new_session=True)
    bad = subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(3)"],
                           start_new_session=True)
    t0 = time.time()
    assert ranks.wait_all([ok, bad], timeout=100) == [(1, 3)]
    assert time.time() - t0 < 30
    assert ok.returncode is not None      # killed and reaped


def test_process_per_device_refuses_chain_subsets():
    from nestmc.sampler import sample_posterior
    kw = _kw(4)
    with pytest.raises(ValueError, match="process_per_device"):
        sample_posterior(**dict(kw, outputDirectory=None), write_files=False,
                         process_per_device=True, chains=[0, 1])
