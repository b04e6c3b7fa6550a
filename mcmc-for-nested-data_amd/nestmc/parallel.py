"""Multi-GPU: chains sharded across ranks, one RCCL gather at the end.

Replaces the reference's process-per-chain fan-out (posteriorSampling.py:182-201).
Chains are independent and every random draw is keyed by the GLOBAL chain id
(Philox key, csrc/rng.h), so a chain's trajectory does not depend on how many GPUs
run or which one runs it.  Groups are never split (the partial-pooling Gibbs update
reduces over a chain's groups every parameter step).  There is no collective in
the sampling loop; after it, ``gather_samples`` moves every rank's sample store to
the root with one ncclGather over xGMI.

The RCCL unique id is bootstrapped through a host process group (torch.distributed
gloo in bench.py / tests): plumbing only, the data path is RCCL.
"""

import ctypes

import numpy

from . import _lib
from ._lib import check, dptr


def shard(n_chains, world, rank):
    """Balanced contiguous split: (first global chain id, count) of ``rank``."""
    base, extra = divmod(n_chains, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def padded_shard(n_chains, world, rank):
    """Equal-size shards (RCCL gather needs equal counts): (start, count, n_real)."""
    per = -(-n_chains // world)
    start = rank * per
    real = max(0, min(per, n_chains - start))
    return start, per, real


def max_over_ranks(value, pg=None):
    if pg is None:
        return value
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def rccl_comm(pg, world, rank, device):
    """Create an RCCL communicator; the 128-byte id travels over the host group."""
    lib = _lib.load()
    idb = (ctypes.c_ubyte * 128)()
    if rank == 0:
        check(lib.nmc_comm_unique_id(idb))
    obj = [bytes(idb) if rank == 0 else None]
    if pg is not None and world > 1:
        pg.broadcast_object_list(obj, src=0)
    idb = (ctypes.c_ubyte * 128).from_buffer_copy(obj[0])
    comm = ctypes.c_void_p()
    check(lib.nmc_comm_init(ctypes.byref(comm), idb, world, rank, device))
    return comm


def rccl_destroy(comm):
    _lib.load().nmc_comm_destroy(comm)


def comm_size(comm):
    """(nranks, rank) of an RCCL communicator."""
    n, r = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().nmc_comm_size(comm, ctypes.byref(n), ctypes.byref(r)))
    return n.value, r.value


def gather_samples(engine, comm, root=0):
    """ncclGather of every rank's [rows][cols][C_local] store.

    The root gets [rank][rows][cols][C_local]; the other ranks get None (and
    allocate nothing).  Every rank must hold the same C_local (padded_shard).
    """
    world, rank = comm_size(comm)
    if rank == root:
        out = numpy.empty((world, engine.n_rows, engine.cols, engine.C))
        check(_lib.load().nmc_gather_samples(engine.h, comm, root, dptr(out), out.size))
        return out
    check(_lib.load().nmc_gather_samples(engine.h, comm, root, None, 0))
    return None


def assemble(gathered, n_real):
    """[rank][rows][cols][C_local] -> [rows][cols][C_total] dropping padding chains."""
    parts = [gathered[r][:, :, :n_real[r]] for r in range(len(n_real))]
    return numpy.concatenate(parts, axis=2)
