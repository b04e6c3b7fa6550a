#!/usr/bin/env python
"""Benchmark: MCMC iterations of the nested-data sampler on MI355X.

Workload (BASELINE.json configs[2], SURVEY 8(d) cfg 3), per GPU: partial-pooling
linear regression (sigma = 1 known, 2 parameters per group), 256 chains x 64
groups x 1000 observations, synthetic data from RandomState(7).  One step = one
full reference iteration (Sampler._loop body: both parameters' Metropolis steps
over every (chain, group) + both Gibbs hyper updates + recording).

value = chains x groups x iterations / second over the whole job (weak scaling:
each rank runs its own 256 chains, global chain ids rank*256.., no collective in
the loop; one RCCL gather of the sample stores after the timed region).

Launch:  python bench.py [--gpus N --steps K --warmup W]
         (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py)
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
sys.path.insert(0, ROOT)

import numpy  # noqa: E402

METRIC = ("MCMC iterations/sec (all chains×groups) + achieved HBM GB/s, "
          "1/2/4/8 MI355X")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X fp64 vector (half the f32 vector rate, 157.3 TF)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--chains", type=int, default=256, help="chains per GPU")
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--obs", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget for the CPU baseline sample (0 disables)")
    ap.add_argument("--no-gather", action="store_true")
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def make_engine(args, rank, device):
    from nestmc.engine import Engine
    from nestmc.families import LinearRegression
    from nestmc import data
    from nestmc.init import init_chains
    G, N, C = args.groups, args.obs, args.chains
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    sizes = [N] * G
    chains = range(rank * C, (rank + 1) * C)
    # reference-exact host init (start point uniform in the example ranges) on a
    # few chains, replicated: init is outside the timed region and not the workload
    st = init_chains(fam, sizes, ("b0", "b1"), chains[:8], "partial", None,
                     {"b0": [-1, 1], "b1": [0, 3]}, False, threads=8)
    rep = lambda a: numpy.concatenate([a] * (C // 8 + 1))[:C]   # noqa: E731
    eng = Engine(fam, sizes, C, "partial", seed=1234, chain_base=rank * C, device=device)
    eng.set_state(rep(st["value"]), rep(st["log_prior"]), rep(st["ll"]), rep(st["mu"]),
                  rep(st["s2"]))
    return eng, fam


def cpu_baseline(args, budget_s):
    """Time the numpy oracle (a restatement of the reference's per-chain loop, legacy
    RNG, process per chain) on this host's cores over a bounded sample."""
    import multiprocessing as mp
    cores = min(16, os.cpu_count() or 1)
    # one probe iteration to size the sample
    t0 = time.time()
    _cpu_chain((0, 1, args.groups, args.obs))
    per_iter = max(time.time() - t0, 1e-3)
    iters = max(2, int(budget_s / per_iter))
    jobs = [(c, iters, args.groups, args.obs) for c in range(cores)]
    t0 = time.time()
    with mp.get_context("fork").Pool(cores) as pool:
        pool.map(_cpu_chain, jobs)
    wall = time.time() - t0
    rate = cores * args.groups * iters / wall
    return {"value": rate, "unit": "chain*group*iter/s", "cores": cores, "kind": "port",
            "sample": "%d chains x %d iterations of the cfg-3 workload (%d groups x %d obs, "
                      "partial pooling) in the numpy oracle, one process per chain"
                      % (cores, iters, args.groups, args.obs)}


def _cpu_chain(job):
    chain, iters, G, N = job
    from nestmc import data
    from oracle import restatement as rs
    from oracle.models import linreg_callback
    x, y, _, _ = data.linreg(G, N, seed=7)
    nested = rs.Nested(linreg_callback(x, y), [N] * G)
    st, r = rs.init_chain(nested, ("b0", "b1"), chain, "partial", None,
                          {"b0": [-1, 1], "b1": [0, 3]}, False)
    rs.run(nested, st, "partial", None, iters, iters, 1, rs.LegacyRNG(r))
    return chain


def main():
    args = parse()
    world, rank, local = dist_env()
    if args.gpus != world and world > 1:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
        pg = dist
    from nestmc import _lib
    from nestmc import parallel

    n_dev = _lib.device_count()
    assert n_dev >= 1, "no HIP device visible"
    device = local % n_dev
    eng, fam = make_engine(args, rank, device)
    K, W = args.steps, args.warmup
    n_iter = W + 2 * K
    # schedule: record the second half like the reference (burn = n_iter // 2)
    eng.set_schedule(n_iter, n_iter // 2, 1)

    # every launch covers the same number of iterations (the warmup length), so the
    # per-launch average below and rocprof's kernel average describe the same launch
    LAUNCH_ITERS = max(1, W)
    eng.set_launch_iters(LAUNCH_ITERS)
    # warmup (untimed)
    eng.run(0, W)
    eng.synchronize()

    def barrier():
        if pg is not None:
            pg.barrier()

    # timed region: exactly K iterations
    barrier()
    eng.synchronize()
    eng.event_record(0)
    t0 = time.perf_counter()
    eng.run(W, W + K)
    eng.event_record(1)
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    wall = t1 - t0
    ev_ms = eng.event_elapsed_ms(0, 1)
    t_rank = max(wall, ev_ms / 1e3)
    t_max = parallel.max_over_ranks(t_rank, pg)

    # second pass, same length: per-launch events on the engine's stream -> the
    # step kernel's average duration for the roofline
    eng.set_kernel_timing(True)
    eng.run(W + K, W + 2 * K)
    kt = eng.kernel_timing()
    eng.set_kernel_timing(False)

    gather_ms = None
    if world > 1 and not args.no_gather:
        comm = parallel.rccl_comm(pg, world, rank, device)
        tg = time.perf_counter()
        full = parallel.gather_samples(eng, comm, root=0, world=world)
        gather_ms = (time.perf_counter() - tg) * 1e3
        parallel.rccl_destroy(comm)
        del full

    C, G, N, P = args.chains, args.groups, args.obs, fam.n_params
    units = world * C * G * K
    value = units / t_max
    launches = kt["step_launches"]
    avg_step_ms = kt["step_ms"] / max(1, launches)
    iters_per_launch = kt["step_iters"] / max(1, launches)
    b_obs = fam.bytes_per_obs()
    # B_unit = P*N*b_obs per chain*group*iteration (each parameter step
    # evaluates the group's rows once per chain); a launch covers iters_per_launch
    # iterations (persistent: a whole variate chunk)
    bytes_per_launch = C * G * P * N * b_obs * iters_per_launch
    achieved_gbs = bytes_per_launch / (avg_step_ms * 1e-3) / 1e9
    # fp64 work: fma + sub + fma = 5 flops per (chain, obs, parameter step)
    flops_per_launch = C * G * P * N * 5 * iters_per_launch
    fp64_tflops = flops_per_launch / (avg_step_ms * 1e-3) / 1e12
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "hbm_traffic_r01.json")
    if os.path.exists(tfile):
        try:   # PMC bytes per iteration of this workload (tools/hbm_traffic.py), per launch
            traffic = json.load(open(tfile))["bytes_per_iteration"] * iters_per_launch
        except Exception:
            traffic = None
    lc = eng.launch_config()
    kname = "nmc_k_run<FamLinreg<2>, %s>" % (
        "NMC_MODE_SYNC_LDS" if lc["persistent"] else "NMC_MODE_LAUNCH")

    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            try:
                cpu = cpu_baseline(args, args.cpu_seconds)
            except Exception as e:     # reported, never fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "chain*group*iter/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": t_max * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "cfg3 partial-pooling linear regression (sigma=1), "
                                   "%d chains x %d groups x %d obs per GPU, P=%d" % (C, G, N, P),
                       "chains_per_gpu": C, "groups": G, "obs_per_group": N, "params": P,
                       "pooling": "partial", "parallelism": "chains sharded x%d" % world,
                       "launch": lc},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": kname,
                         "avg_launch_us": avg_step_ms * 1e3,
                         "iterations_per_launch": iters_per_launch,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "note": "rows are LDS-resident for the whole launch, so the "
                                 "algorithmic bytes exceed HBM: frac > 1 is expected; the "
                                 "kernel's real bound is fp64 VALU issue (fp64_valu)",
                         "fp64_valu": {"achieved": fp64_tflops, "peak": FP64_VALU_PEAK_TFLOPS,
                                       "unit": "TFLOP/s",
                                       "frac": fp64_tflops / FP64_VALU_PEAK_TFLOPS}},
            "cpu_baseline": cpu,
            "event_ms": ev_ms,
            "hyper_only_avg_us": (kt["hyper_ms"] / max(1, kt["hyper_launches"])) * 1e3,
            "gather_ms": gather_ms,
        }
        print(json.dumps(out))
    eng.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
