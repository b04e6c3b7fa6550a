"""bench.py's multi-rank arithmetic (N > 1 on CPU): every workload's per-rank chain blocks
tile the job's chains exactly once, so value = job chains x groups x K / max-over-ranks
time counts each (chain, group, iteration) once; the host bootstrap's max over two real
processes is the slowest rank's time."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))

import bench  # noqa: E402


@pytest.mark.parametrize("name", sorted(bench.WORKLOADS))
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_rank_blocks_tile_the_job(name, world):
    wl = dict(bench.WORKLOADS[name])
    covered = []
    for r in range(world):
        c0, C = bench.rank_chains(wl, world, r)
        assert C >= 1
        covered.extend(range(c0, c0 + C))
    assert covered == list(range(bench.job_chains(wl, world)))
    if wl["scaling"] == "weak":   # fixed work per GPU
        assert bench.job_chains(wl, world) == world * wl["chains"]
    else:                         # fixed total work, blocks differ by at most one chain
        sizes = [bench.rank_chains(wl, world, r)[1] for r in range(world)]
        assert max(sizes) - min(sizes) <= 1 and sum(sizes) == wl["chains"]


_WORKER = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "mcmc-for-nested-data_amd"))
from nestmc import parallel
rank = int(os.environ["RANK"])
hg = parallel.HostGroup(2, rank)
t = parallel.max_over_ranks([0.25, 0.75][rank], hg)
hg.barrier()
hg.close()
print("T=%r torch=%d" % (t, "torch" in sys.modules))
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_max_over_ranks_two_processes():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), NMC_BOOTSTRAP_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _WORKER, ROOT], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=60) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
        assert "T=0.75 torch=0" in o, (o, e)


@pytest.mark.parametrize("kernel,inst", [
    ("nmc_k_run<FamLinreg<2>, NMC_MODE_SYNC_REG, true>", "FamLinreg<2>"),
    ("nmc_k_sweep<FamGaussMean<3>, NMC_MODE_HALF>", "FamGaussMean<3>"),
    ("nmc_k_run<FamUser, NMC_MODE_SYNC, false>", "FamUser"),
])
def test_family_instance_of_kernel_name(kernel, inst):
    """The roofline's per-row instruction count is keyed by the step kernel's family."""
    assert bench.fam_instance(kernel) == inst


@pytest.mark.parametrize("name", sorted(bench.WORKLOADS))
@pytest.mark.parametrize("n", [2, 4])
def test_gpus_flag_spawns_ranks(name, n):
    """``bench.py --gpus N`` without a launcher starts N ranks itself (torchrun's env, one
    per GPU) before any HIP call, and relays rank 0's line with n_gpus == N; every rank
    holds its own shard of the job (dry run: the ranks stop before GPU init)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--workload", name, "--spawn-dry-run"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    import json
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == n and line["rank"] == 0
    ranks = line["ranks"]
    assert [r["rank"] for r in ranks] == list(range(n))
    assert [r["local_rank"] for r in ranks] == list(range(n))
    assert all(r["n_gpus"] == n and not r["libnestmc_mapped"] for r in ranks)
    wl = dict(bench.WORKLOADS[name])
    for r in ranks:
        assert (r["chain_base"], r["chains"]) == bench.rank_chains(wl, n, r["rank"])
    covered = sorted(c for r in ranks for c in range(r["chain_base"], r["chain_base"] + r["chains"]))
    assert covered == list(range(bench.job_chains(wl, n)))


def test_cpu_cores_is_the_real_budget():
    """cpu_baseline's core count is the affinity mask bounded by the cgroup CPU quota, not
    OMP_NUM_THREADS."""
    cores, aff, quota = bench.cpu_cores()
    assert aff == len(os.sched_getaffinity(0))
    assert cores == (aff if quota is None else min(aff, max(1, int(quota))))


@pytest.mark.parametrize("W,K", [(5, 20), (200, 2000), (0, 7), (3, 1)])
def test_timed_call_records_every_iteration(W, K):
    """The bench schedule makes the warm-up the burn-in: every iteration of the timed call
    [W, W + K) and of the kernel-timing call after it writes a sample row, like the post-burn
    steady state of the reference's loop (posteriorSampling.py:883-891)."""
    from nestmc.sampler import record_iterations
    n_iter, burn, thin = bench.bench_schedule(W, K)
    assert n_iter == W + 2 * K and thin == 1
    rec = set(record_iterations(n_iter, burn, thin))
    assert all(i in rec for i in range(W, W + 2 * K))
    assert bench.recorded_in(W, W + K, n_iter, burn, thin) == K
    assert bench.recorded_in(0, W, n_iter, burn, thin) == 0
