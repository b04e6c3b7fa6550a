"""One process per GPU for samplePosterior(..., process_per_device=True).

The reference fans chains out over a process pool (posteriorSampling.py:182-201) and each
process writes its chains' files (:1048-1049).  Here the unit is a GPU: the calling process
starts one rank per device as a child process -- before it makes any HIP call itself -- with
the torchrun-style environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR and the host
bootstrap port NMC_BOOTSTRAP_PORT).  Rank r runs its contiguous block of chains
(parallel.padded_shard) on devices[r]; after the loop the ranks meet in a HostGroup and ONE
ncclGather (RCCL over xGMI) brings every sample store to rank 0, which writes every
sample.<chain>.csv; each rank writes its own chains' logLikelihood.<chain>.csv.  Rank 0
hands samplePosterior's return value back through a file.  A rank that fails ends the run:
the others are stopped and the caller gets the error.

    python -m nestmc.ranks SPEC      (a rank; SPEC is the parent's pickled call)
"""

import json
import os
import pickle
import shutil
import socket
import subprocess
import sys
import tempfile
import time
import types

from . import _lib


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stop(procs):
    """Kill every child still running (each leads its own session: its whole process group)
    and reap it."""
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, 9)
            except OSError:
                pass
            p.wait()


def wait_all(procs, timeout=None):
    """Wait for every rank.  Returns None when all exited 0, else the failures -- [(rank,
    exit code)] or "timeout" -- after killing the ranks still running (they would wait on the
    failed one in the host group's collectives).  Any exception in the caller's wait
    (KeyboardInterrupt included) kills every rank before it propagates: no rank outlives
    the call, none keeps writing into the output directory."""
    deadline = None if timeout is None else time.time() + timeout
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad or (deadline is not None and time.time() > deadline):
                _stop(procs)
                return bad or "timeout"
            if all(c == 0 for c in codes):
                return None
            time.sleep(0.02)
    except BaseException:
        _stop(procs)
        raise


class _SpecPickler(pickle.Pickler):
    """Pickles the call for the ranks, refusing what a rank cannot unpickle: a function or
    class defined in the caller's script (module __main__ -- e.g. a DeviceLikelihood's
    host_function = functools.partial(computeLogLikelihood, ...) from the reference
    examples).  A rank is a fresh interpreter running nestmc.ranks, so such names do not
    exist there; without this check every rank would die on the unpickle and the caller see
    only their exit codes."""

    def reducer_override(self, obj):
        if isinstance(obj, (type, types.FunctionType, types.BuiltinFunctionType)) and \
                getattr(obj, "__module__", None) == "__main__":
            raise ValueError(
                "process_per_device: %r is defined in the calling script (module __main__) "
                "and cannot be loaded by the ranks, which are separate processes; define it "
                "in an importable module (or drop DeviceLikelihood's host_function when "
                "startWithMLE is False: the sampler never calls it then)"
                % getattr(obj, "__qualname__", obj))
        return NotImplemented


# (tests) dry-run ranks sleep this long before reporting, so a test can interrupt the parent
# while they run
_DRY_HOLD_S = "NMC_RANKS_DRY_HOLD_S"
last_pids = []      # (tests) the ranks of the latest run_per_device call


def run_per_device(kwargs, devices, dry_run=False, timeout=None):
    """Start len(devices) ranks of sample_posterior(**kwargs), wait for all of them and
    return rank 0's result (dry_run: every rank reports its shard and exits before any HIP
    call -- the list of those reports)."""
    n = len(devices)
    if n < 1:
        raise ValueError("process_per_device needs at least one device")
    tmp = tempfile.mkdtemp(prefix="nmc_ranks_")
    try:
        spec = os.path.join(tmp, "spec.pkl")
        with open(spec, "wb") as f:
            _SpecPickler(f).dump({"kwargs": kwargs, "devices": list(devices), "dir": tmp,
                                  "dry_run": bool(dry_run)})
        port = _free_port()
        pkg_parent = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        pp = os.environ.get("PYTHONPATH")
        procs = []
        del last_pids[:]
        try:
            for r in range(n):
                env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                           LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                           NMC_BOOTSTRAP_PORT=str(port),
                           PYTHONPATH=pkg_parent + (os.pathsep + pp if pp else ""))
                env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
                procs.append(subprocess.Popen([sys.executable, "-m", "nestmc.ranks", spec],
                                              env=env, start_new_session=True))
                last_pids.append(procs[-1].pid)
        except BaseException:
            _stop(procs)
            raise
        failed = wait_all(procs, timeout)
        if failed is not None:
            raise _lib.NestmcError("samplePosterior ranks failed (rank, exit code): %s" % (failed,))
        if dry_run:
            out = []
            for r in range(n):
                with open(os.path.join(tmp, "dry.%d.json" % r)) as f:
                    out.append(json.load(f))
            return out
        res = os.path.join(tmp, "result.pkl")
        if os.path.exists(res):
            with open(res, "rb") as f:     # (written by our own rank 0 just now)
                return pickle.load(f)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main(spec_path):
    with open(spec_path, "rb") as f:        # (the parent's own pickle of this call)
        spec = pickle.load(f)
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    kw, devices = spec["kwargs"], spec["devices"]
    if spec["dry_run"]:
        from .parallel import padded_shard
        time.sleep(float(os.environ.get(_DRY_HOLD_S, "0") or 0))
        s0, per, real = padded_shard(kw["nChains"], world, rank)
        with open(os.path.join(spec["dir"], "dry.%d.json" % rank), "w") as f:
            json.dump({"rank": rank, "world": world, "device": devices[rank], "chain_base": s0,
                       "chains": per, "real": real,
                       "bootstrap_port": int(os.environ["NMC_BOOTSTRAP_PORT"]),
                       "libnestmc_mapped": "libnestmc" in open("/proc/self/maps").read()}, f)
        return 0
    from .parallel import HostGroup
    from .sampler import sample_posterior
    hg = HostGroup(world, rank)
    try:
        res = sample_posterior(**kw, devices=devices, _rank=(hg, world, rank))
        if rank == 0 and res is not None:
            with open(os.path.join(spec["dir"], "result.pkl"), "wb") as f:
                pickle.dump(res, f)
        hg.barrier()
    finally:
        hg.close()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
