"""N > 1 path on the CPU: two gloo ranks, chains sharded by global id.

The multi-GPU design (nestmc/parallel.py, DESIGN.md "Multi-GPU") shards chains
across ranks with no collective in the sampling loop: every variate is keyed by the
GLOBAL chain id, so rank r's chains must reproduce the same chains of a one-rank
run.  Here each rank runs its shard through the oracle's Philox stream (the same
stream the device consumes) and the shards travel to rank 0 over gloo, which checks
them against a single-process run of all chains; max_over_ranks (bench.py's timing
reduction) and the padded-shard assembly used by the RCCL gather are checked too.
"""

import os
import socket

import numpy
import pytest

WORLD = 2
C, G, N, P, N_ITER, SEED = 7, 4, 15, 2, 12, 31


def _problem():
    from nestmc.families import LinearRegression
    from oracle import restatement as rs
    r = numpy.random.RandomState(3)
    x = r.normal(size=G * N)
    y = 0.5 + 1.5 * x + r.normal(size=G * N)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    nested = rs.Nested(fam, [N] * G)
    mu = numpy.tile([0.0, 1.5], (C, 1))
    s2 = numpy.full((C, P), 0.5)
    value = mu[:, :, None] + 0.4 * r.normal(size=(C, P, G))
    lp = rs.norm_logpdf(value, mu[:, :, None], numpy.sqrt(s2)[:, :, None])
    ll = numpy.array([nested.group_ll(value[c]) for c in range(C)])
    return nested, value, lp, ll, mu, s2


def _run_chains(ids):
    """Oracle run of global chains ``ids`` -> recorded rows [len(ids), rows, cols]."""
    from oracle import restatement as rs
    nested, value, lp, ll, mu, s2 = _problem()
    sel = numpy.asarray(ids)
    st = rs.State(value[sel].copy(), lp[sel].copy(), ll[sel].copy(), mu[sel].copy(),
                  s2[sel].copy())
    rec = []
    rs.run(nested, st, "partial", None, N_ITER, N_ITER // 2, 2, rs.PhiloxRNG(sel, SEED),
           record=rec)
    return numpy.stack([row for _, row in rec], 1)


def _worker(rank, port, q):
    """gloo ranks: the oracle shards gathered over torch.distributed (test harness)."""
    import torch.distributed as dist
    from nestmc import parallel
    try:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                                world_size=WORLD, rank=rank)
        start, count = parallel.shard(C, WORLD, rank)
        rows = _run_chains(range(start, start + count))
        t = [None] * WORLD
        dist.all_gather_object(t, 1.0 + rank)
        out = [None] * WORLD
        dist.all_gather_object(out, (start, count, rows))
        if rank == 0:
            q.put(("ok", max(t), out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # reported to the parent
        q.put(("error", repr(e), None))


def _host_worker(rank, port, q):
    """The product's bootstrap (nestmc.parallel.HostGroup, stdlib TCP, no PyTorch): the
    max-over-ranks timing, the 128-byte id broadcast, barrier and the shards' rows."""
    import sys
    from nestmc import parallel
    try:
        hg = parallel.HostGroup(WORLD, rank, addr="127.0.0.1", port=port, timeout=60)
        start, count = parallel.shard(C, WORLD, rank)
        rows = _run_chains(range(start, start + count))
        t = parallel.max_over_ranks(1.0 + rank, hg)
        idb = hg.broadcast(bytes(range(128)) if rank == 0 else None, src=0)
        hg.barrier()
        last = hg.broadcast(b"from-1" if rank == 1 else None, src=1)
        parts = hg.all_gather(numpy.ascontiguousarray(rows).tobytes())
        if rank == 0:
            q.put(("ok", (t, idb, last, [len(p) for p in parts], "torch" in sys.modules),
                   (start, count, parts)))
        hg.barrier()
        hg.close()
    except Exception as e:   # reported to the parent
        q.put(("error", repr(e), None))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_shards_reproduce_single_rank_run():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    status, t, shards = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", t
    assert t == float(WORLD)                       # max over ranks
    assert [s[0] for s in shards] == [0, 4] and [s[1] for s in shards] == [4, 3]
    merged = numpy.concatenate([s[2] for s in shards], 0)
    whole = _run_chains(range(C))
    assert numpy.array_equal(merged, whole)        # bit-identical: keyed by global id


def test_padded_shards_and_assembly():
    from nestmc import parallel
    shards = [parallel.padded_shard(10, 4, r) for r in range(4)]
    assert shards == [(0, 3, 3), (3, 3, 3), (6, 3, 3), (9, 3, 1)]
    rows, cols = 2, 5
    gathered = numpy.zeros((4, rows, cols, 3))
    for r, (start, per, real) in enumerate(shards):
        for k in range(per):
            gathered[r, :, :, k] = start + k if k < real else -1
    full = parallel.assemble(gathered, [s[2] for s in shards])
    assert full.shape == (rows, cols, 10)
    assert numpy.array_equal(full[0, 0], numpy.arange(10))
    # balanced split covers every chain once
    parts = [parallel.shard(13, 3, r) for r in range(3)]
    assert sum(c for _, c in parts) == 13 and parts[0] == (0, 5) and parts[2] == (9, 4)


def test_host_group_bootstrap_two_processes():
    """nestmc.parallel.HostGroup (what bench.py and the RCCL bootstrap use): two spawned
    processes, no PyTorch imported, the shard rows merged on rank 0 equal one run."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    status, info, payload = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", info
    t, idb, last, sizes, torch_loaded = info
    assert t == float(WORLD) and idb == bytes(range(128)) and last == b"from-1"
    assert not torch_loaded                         # the bootstrap needs no PyTorch
    whole = _run_chains(range(C))
    got = [numpy.frombuffer(b, dtype=numpy.float64) for b in payload[2]]
    assert numpy.array_equal(numpy.concatenate(got), numpy.concatenate(
        [whole[:4].ravel(), whole[4:].ravel()]))
