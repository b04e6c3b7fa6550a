"""GPU: the product's multi-engine path -- samplePosterior sharding chains over several
engines (the rebuild's replacement of the reference's process fan-out,
posteriorSampling.py:182-201) -- run for real on one device.

* devices=[0, 0]: two engines on the same GPU, each holding a contiguous block of the
  chains (nestmc.parallel.shard), initialised and driven by the same host flow as one
  engine per GPU; the CSVs (samples and per-observation log-likelihoods) must be byte-
  identical to devices=[0];
* chains=: two calls holding the two halves of the chains (what two ranks of a job
  launched by torchrun do) write, between them, the files of the one-call run byte for
  byte;
* on a golden case with the reference's own variates replayed, devices=[0, 0] still
  writes the reference's bytes.
"""

import filecmp
import os

import numpy
import pytest

from golden_cases import Case
from gpu_cases import family_for, synthetic
from nestmc.sampler import sample_posterior

pytestmark = pytest.mark.gpu


def _files(d):
    return sorted(f for f in os.listdir(os.path.join(d, "sample")))


def _same_tree(a, b, names):
    for fn in names:
        pa, pb = os.path.join(a, "sample", fn), os.path.join(b, "sample", fn)
        assert filecmp.cmp(pa, pb, shallow=False), fn


@pytest.mark.parametrize("kind", ["linreg_partial", "regression3_none"])
def test_devices_and_chain_halves_byte_identical(gpu_lib, tmp_path, kind):
    C, G, N = 70, 6, 40
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N)
    ranges = {n: [-0.5, 0.5] for n in names if n != "sigma"}
    if "sigma" in names:
        ranges["sigma"] = [0.5, 1.5]
    kw = dict(saveLogLikelihood=True, priorDistribution=priors,
              startingPointValueRange=ranges, displayProgress=False, seed=17)
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, one, devices=[0], **kw)
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, two, devices=[0, 0], **kw)
    files = _files(one)
    assert sum(f.startswith("sample.") for f in files) == C
    assert sum(f.startswith("logLikelihood.") for f in files) == C
    assert _files(two) == files
    _same_tree(one, two, files)
    # two "ranks": halves of the chains, each in its own call and output directory
    h0, h1 = str(tmp_path / "h0"), str(tmp_path / "h1")
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, h0, chains=range(0, 33), **kw)
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, h1, chains=range(33, C), **kw)
    for c in range(C):
        h = h0 if c < 33 else h1
        for fn in ("sample.%d.csv" % c, "logLikelihood.%d.csv" % c):
            assert filecmp.cmp(os.path.join(one, "sample", fn), os.path.join(h, "sample", fn),
                               shallow=False), fn
    # the returned arrays of a two-engine run are the one-engine arrays
    r1 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, None, devices=[0],
                          write_files=False, return_samples=True,
                          **dict(kw, saveLogLikelihood=False))
    r2 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, None, devices=[0, 0],
                          write_files=False, return_samples=True,
                          **dict(kw, saveLogLikelihood=False))
    assert numpy.array_equal(r1["rows"], r2["rows"], equal_nan=True)
    assert numpy.array_equal(r1["accepted"], r2["accepted"])


@pytest.mark.parametrize("name", ["linreg_partial", "regression_none"])
def test_devices_replay_writes_reference_csvs(gpu_lib, tmp_path, name):
    c = Case(name)
    a = c.arr
    out = str(tmp_path) + "/"
    sample_posterior(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups, c.n_per_group,
                     c.pooling, family_for(c), out, saveLogLikelihood=False,
                     priorDistribution=c.priors, startWithMLE=c.mle,
                     startingPointValueRange=c.ranges, displayProgress=False,
                     devices=[0] * c.n_chains,
                     rng="replay", replay={k: a[k] for k in ("z", "u", "hz", "hu")})
    for ch in range(c.n_chains):
        mine = os.path.join(out, "sample", "sample.%i.csv" % ch)
        assert filecmp.cmp(mine, c.csv_path(ch), shallow=False), (name, ch)


def test_process_per_device_one_rank_byte_identical(gpu_lib, tmp_path):
    """samplePosterior(process_per_device=True): this process starts one rank per device
    (nestmc.ranks) before touching the GPU; the rank samples its chains, gathers its sample
    store to rank 0 with ncclGather and writes every file -- byte for byte the in-process
    path's files (samples, per-observation LLs) and the same returned arrays."""
    C, G, N = 70, 6, 40
    fam, sizes, priors, pooling, names = synthetic("linreg_partial", C, G, N)
    kw = dict(saveLogLikelihood=True, priorDistribution=priors,
              startingPointValueRange={n: [-0.5, 0.5] for n in names}, displayProgress=False,
              seed=23)
    one, ppd = str(tmp_path / "one"), str(tmp_path / "ppd")
    r1 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, one, devices=[0],
                          return_samples=True, **kw)
    r2 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, ppd, devices=[0],
                          return_samples=True, process_per_device=True, **kw)
    files = _files(one)
    assert sum(f.startswith("sample.") for f in files) == C
    assert _files(ppd) == files
    _same_tree(one, ppd, files)
    assert sorted(os.listdir(os.path.join(ppd, "log"))) == \
        sorted(os.listdir(os.path.join(one, "log")))
    assert numpy.array_equal(r1["rows"], r2["rows"], equal_nan=True)
    assert numpy.array_equal(r1["accepted"], r2["accepted"])
    assert r1["row_index"] == r2["row_index"]


# ---- two processes (host-group ranks), each driving its own engine on the GPU ----------
def _npy(*arrays):
    import io
    f = io.BytesIO()
    numpy.savez(f, *arrays)
    return f.getvalue()


def _unnpy(blob):
    import io
    z = numpy.load(io.BytesIO(blob), allow_pickle=False)
    return [z["arr_%d" % i] for i in range(len(z.files))]


def _host_engine_worker(rank, world, port, q):
    """Rank `rank`: its contiguous shard of the chains (nestmc.parallel.shard), run by an
    engine with chain_base = the shard's first global id; the recorded rows travel to
    rank 0 over the product's host group (nestmc.parallel.HostGroup, bench.py's bootstrap),
    and bench.py's max-over-ranks timing reduction runs too."""
    from nestmc import parallel
    from gpu_cases import partial_state, run_engine, synthetic
    try:
        hg = parallel.HostGroup(world, rank, addr="127.0.0.1", port=port, timeout=120)
        C, G, N, n_iter, seed = 70, 5, 30, 24, 19
        fam, sizes, _, _, _ = synthetic("linreg_partial", C, G, N)
        st, _ = partial_state(fam, sizes, C, 2)
        start, count = parallel.shard(C, world, rank)
        sel = numpy.arange(start, start + count)
        acc, _, rows, _ = run_engine(fam, sizes, st, sel, start, n_iter, seed)
        t = parallel.max_over_ranks(1.0 + rank, hg)
        parts = hg.gather(_npy(numpy.array([start, count]), acc, rows))
        if rank == 0:
            out = [tuple([int(v) for v in a[0]]) + tuple(a[1:]) for a in map(_unnpy, parts)]
            whole = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, seed)
            q.put(("ok", t, out, whole[0], whole[2]))
        hg.barrier()
        hg.close()
    except Exception as e:   # reported to the parent
        q.put(("error", repr(e), None, None, None))


def test_two_host_ranks_engines_reproduce_one_engine(gpu_lib):
    """The N > 1 path with the engine on every rank: two processes, one host
    group (stdlib TCP), each samples its chain shard on the device; the shards are the
    one-engine run bit for bit (every variate keyed by global chain id)."""
    import socket
    import multiprocessing as mp
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_host_engine_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    status, t, shards, acc1, rows1 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", t
    assert t == float(world)
    assert [sh[0] for sh in shards] == [0, 35] and [sh[1] for sh in shards] == [35, 35]
    assert numpy.array_equal(numpy.concatenate([sh[2] for sh in shards], 0), acc1)
    assert numpy.array_equal(numpy.concatenate([sh[3] for sh in shards], 0), rows1,
                             equal_nan=True)
