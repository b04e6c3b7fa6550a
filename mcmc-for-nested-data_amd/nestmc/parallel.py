"""Multi-GPU: chains sharded across ranks, one RCCL gather at the end.

Replaces the reference's process-per-chain fan-out (posteriorSampling.py:182-201).
Chains are independent and every random draw is keyed by the GLOBAL chain id
(Philox key, csrc/rng.h), so a chain's trajectory does not depend on how many GPUs
run or which one runs it.  Groups are never split (the partial-pooling Gibbs update
reduces over a chain's groups every parameter step).  There is no collective in
the sampling loop; after it, ``gather_samples`` moves every rank's sample store to
the root with one ncclGather over xGMI.

The RCCL unique id (128 bytes), the barrier and the max-over-ranks timing travel over
``HostGroup``: a stdlib TCP star through rank 0, rendezvous at MASTER_ADDR and
MASTER_PORT + 1 (torchrun's own store holds MASTER_PORT; NMC_BOOTSTRAP_PORT overrides).
torchrun stays usable as the launcher; nothing here imports PyTorch.  Plumbing only: the
data path is RCCL.
"""

import ctypes
import os
import socket
import struct
import time

import numpy

from . import _lib
from ._lib import check, dptr


class HostGroup:
    """Rank-0-centred TCP process group for the host-side bootstrap (no PyTorch).

    ``broadcast(data, src=0)``, ``gather(data)`` (root 0), ``all_gather(data)``,
    ``barrier()`` and ``max_float(v)`` move ``bytes`` between the ranks; every rank must
    call the same sequence.  Rank 0 listens on ``addr:port``; the others connect (retrying
    until ``connect_timeout`` seconds) and announce their rank.  Every collective then waits
    up to ``timeout`` seconds for its peers (default 1800 s, gloo's default, or
    NMC_HOSTGROUP_TIMEOUT): a rank may reach a barrier minutes after the others (chain
    init, hiprtc compilation of a user family).
    """

    def __init__(self, world, rank, addr=None, port=None, timeout=None, connect_timeout=120.0):
        if timeout is None:
            timeout = float(os.environ.get("NMC_HOSTGROUP_TIMEOUT", "1800"))
        self.world, self.rank = int(world), int(rank)
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            if os.environ.get("NMC_BOOTSTRAP_PORT"):
                port = int(os.environ["NMC_BOOTSTRAP_PORT"])
            else:
                port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        self.peers = {}          # rank 0: rank -> socket
        self.sock = None         # other ranks: the connection to rank 0
        if self.world == 1:
            return
        deadline = time.time() + connect_timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(max(1.0, deadline - time.time()))
            try:
                while len(self.peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(timeout)
                    r = struct.unpack("<i", self._recv_exact(conn, 4))[0]
                    if not 0 < r < self.world or r in self.peers:
                        raise RuntimeError("HostGroup: bad rank %d announced" % r)
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise RuntimeError("HostGroup: rank 0 at %s:%d unreachable" % (addr, port))
                    time.sleep(0.05)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.settimeout(timeout)
            c.sendall(struct.pack("<i", self.rank))
            self.sock = c

    @staticmethod
    def _recv_exact(s, n):
        buf = bytearray()
        while len(buf) < n:
            chunk = s.recv(n - len(buf))
            if not chunk:
                raise RuntimeError("HostGroup: peer closed the connection")
            buf += chunk
        return bytes(buf)

    def _send(self, s, data):
        s.sendall(struct.pack("<q", len(data)) + data)

    def _recv(self, s):
        n = struct.unpack("<q", self._recv_exact(s, 8))[0]
        return self._recv_exact(s, n)

    def gather(self, data):
        """Rank 0 gets [bytes of rank 0, 1, ...]; the others get None."""
        if self.world == 1:
            return [data]
        if self.rank == 0:
            return [data] + [self._recv(self.peers[r]) for r in range(1, self.world)]
        self._send(self.sock, data)
        return None

    def broadcast(self, data=None, src=0):
        """Rank ``src``'s bytes on every rank (through rank 0)."""
        if self.world == 1:
            return data
        if src != 0:
            parts = self.gather(data if self.rank == src else b"")
            data = parts[src] if self.rank == 0 else None
        if self.rank == 0:
            for r in range(1, self.world):
                self._send(self.peers[r], data)
            return data
        return self._recv(self.sock)

    def all_gather(self, data):
        parts = self.gather(data)
        blob = b"" if parts is None else b"".join(struct.pack("<q", len(p)) + p for p in parts)
        blob = self.broadcast(blob)
        out, i = [], 0
        while i < len(blob):
            n = struct.unpack("<q", blob[i:i + 8])[0]
            out.append(blob[i + 8:i + 8 + n])
            i += 8 + n
        return out

    def barrier(self):
        self.all_gather(b"")

    def max_float(self, value):
        vals = self.all_gather(struct.pack("<d", float(value)))
        return max(struct.unpack("<d", v)[0] for v in vals)

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None


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


def max_over_ranks(value, hg=None):
    """The maximum of ``value`` over the ranks of host group ``hg`` (None: one rank)."""
    if hg is None:
        return value
    return hg.max_float(value)


def rccl_comm(hg, world, rank, device):
    """Create an RCCL communicator; the 128-byte id travels over host group ``hg``."""
    lib = _lib.load()
    idb = (ctypes.c_ubyte * 128)()
    if rank == 0:
        check(lib.nmc_comm_unique_id(idb))
    blob = bytes(idb) if rank == 0 else None
    if hg is not None and world > 1:
        blob = hg.broadcast(blob, src=0)
    idb = (ctypes.c_ubyte * 128).from_buffer_copy(blob)
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
