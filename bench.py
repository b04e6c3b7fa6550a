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
# fp64 VALU issue: 256 CUs x 4 SIMDs x 16 fp64 lanes x 2.4 GHz lane-instructions per second
# (the 78.6 TFLOP/s fp64 vector peak counts an FMA as 2 flops)
VALU_PEAK_TIPS = 256 * 4 * 16 * 2.4e9 / 1e12
VALU_PER_CHAIN_ROW = 3          # fp64 VALU lane-instructions per (chain, row, parameter step)


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
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the two rocprofv3 PMC passes that measure HBM traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
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
    eng = Engine(fam, sizes, C, "partial", seed=1234, chain_base=rank * C, device=device)
    # reference-order init of every chain (start point uniform in the example ranges),
    # likelihoods batched on the device; outside the timed region
    st = init_chains(fam, sizes, ("b0", "b1"), chains, "partial", None,
                     {"b0": [-1, 1], "b1": [0, 3]}, False, group_ll=eng.eval_group_ll)
    eng.set_state(st["value"], st["log_prior"], st["ll"], st["mu"], st["s2"])
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
    out = {"value": rate, "unit": "chain*group*iter/s", "cores": cores, "kind": "port",
           "sample": "%d chains x %d iterations of the cfg-3 workload (%d groups x %d obs, "
                     "partial pooling) in the numpy oracle, one process per chain"
                     % (cores, iters, args.groups, args.obs)}
    cal = os.path.join(ROOT, "profiles", "cpu_calibration_r03.json")
    if os.path.exists(cal):
        # the reference cannot travel to this box: its speed relative to the restatement
        # was measured side by side in the build container (oracle/calibrate_cpu.py)
        ratio = json.load(open(cal))["reference_over_restatement"]
        out["calibration"] = {"reference_over_restatement": ratio,
                              "source": "profiles/cpu_calibration_r03.json "
                                        "(oracle/calibrate_cpu.py, build container)"}
        out["reference_equivalent_value"] = rate * ratio
    return out


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


LDS_PEAK_GBS = 256.0 * 256 * 2.4   # 256 B/clk/CU (ds_read_b64/b128) x 256 CUs x 2.4 GHz


def pmc_child(args):
    """Runs under rocprofv3 --pmc: the same workload and launches as the timed region
    (warmup launch of W iterations, then one launch of K iterations)."""
    from nestmc import _lib
    eng, _ = make_engine(args, 0, 0)
    W, K = args.warmup, args.steps
    eng.set_schedule(W + K, (W + K) // 2, 1)
    eng.run(0, W)
    eng.run(W, W + K)
    eng.synchronize()
    eng.close()
    assert _lib.device_count() >= 1


def measure_traffic(args):
    """HBM bytes of the step kernel's K-iteration launch from two rocprofv3 PMC passes
    of this script (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), run as child
    processes before this process touches the GPU.  gfx950 correction
    (MI355X_MICROARCH.md, HBM): FETCH_SIZE tallies 128-B requests at 64 B -> x2;
    WRITE_SIZE as is; both in KiB per dispatch; Infinity-Cache hits are counted."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    out = {}
    base = tempfile.mkdtemp(prefix="nmc_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(base, counter)
            cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc",
                   "--", "python3", os.path.abspath(__file__), "--pmc-child",
                   "--steps", str(args.steps), "--warmup", str(args.warmup),
                   "--chains", str(args.chains), "--groups", str(args.groups),
                   "--obs", str(args.obs)]
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL, start_new_session=True)
            try:
                rc = p.wait(timeout=150)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait()
                return {"error": "rocprofv3 %s pass timed out" % counter}
            if rc != 0:
                return {"error": "rocprofv3 %s pass exited %d" % (counter, rc)}
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if row.get("Counter_Name") == counter and \
                                "nmc_k_run" in row.get("Kernel_Name", ""):
                            rows.append((int(row.get("Dispatch_Id", 0)),
                                         float(row["Counter_Value"])))
            if len(rows) < 2:
                return {"error": "no %s rows for nmc_k_run" % counter}
            out[counter] = sorted(rows)[-1][1]       # the K-iteration launch (the last)
    finally:
        shutil.rmtree(base, ignore_errors=True)
    read_b = 2.0 * out["FETCH_SIZE"] * 1024.0
    write_b = out["WRITE_SIZE"] * 1024.0
    return {"bytes_per_launch": read_b + write_b, "read_bytes": read_b, "write_bytes": write_b,
            "fetch_size_kib_raw": out["FETCH_SIZE"], "write_size_kib_raw": out["WRITE_SIZE"],
            "iterations_per_launch": args.steps,
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of this "
                      "script's K-iteration launch; FETCH_SIZE x2 (gfx950), KiB -> bytes"}


def main():
    args = parse()
    world, rank, local = dist_env()
    if args.pmc_child:
        return pmc_child(args)
    if args.gpus != world and world > 1:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # host-side legs first, before this process initialises the GPU: the PMC passes
    # run this script as rocprofv3 children, the CPU baseline forks a process pool
    pmc, cpu = None, None
    if world == 1:
        if not args.no_pmc:
            try:
                pmc = measure_traffic(args)
            except Exception as e:     # reported, never fatal for the GPU number
                pmc = {"error": repr(e)}
        if args.cpu_seconds > 0:
            try:
                cpu = cpu_baseline(args, args.cpu_seconds)
            except Exception as e:
                cpu = {"value": None, "error": repr(e)}
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
    # production launch length: one persistent launch per nmc_run call (up to the
    # variate chunk), exactly as samplePosterior drives the engine -- the warmup is
    # its own launch, the timed region one launch of K iterations
    eng.set_launch_iters(0)
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
    t_enq = time.perf_counter() - t0          # host time to enqueue the launch(es)
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

    gather_ms, gather_err = None, None
    if world > 1 and not args.no_gather:
        # after the timed region: the one RCCL gather of the sample stores; a
        # failure here is reported in the line, never lost with it
        try:
            comm = parallel.rccl_comm(pg, world, rank, device)
            tg = time.perf_counter()
            full = parallel.gather_samples(eng, comm, root=0)
            gather_ms = (time.perf_counter() - tg) * 1e3
            parallel.rccl_destroy(comm)
            del full
        except Exception as e:
            gather_err = repr(e)

    C, G, N, P = args.chains, args.groups, args.obs, fam.n_params
    units = world * C * G * K
    value = units / t_max
    launches = kt["step_launches"]
    avg_step_ms = kt["step_ms"] / max(1, launches)
    iters_per_launch = kt["step_iters"] / max(1, launches)
    b_obs = fam.bytes_per_obs()
    lc = eng.launch_config()
    # B_unit = P*N*b_obs per chain*group*iteration (each parameter step
    # evaluates the group's rows once per chain).  The rows are LDS-resident for the
    # launch, so these bytes never come from HBM; they are the rows delivered to the
    # chain lanes.
    bytes_per_launch = C * G * P * N * b_obs * iters_per_launch
    achieved_gbs = bytes_per_launch / (avg_step_ms * 1e-3) / 1e9
    # The binding resource is fp64 VALU issue.  The shipped row loop (kernels.h
    # nmc_rows_lds_linreg2_paired; profiles/isa_r03_linreg_paired.txt) issues 24 fp64 VALU
    # instructions (v_add_f64 x8, v_fma_f64 x16) per 8-row block for two chains per lane:
    # 3 per (chain, row, parameter step) -- the whole likelihood work.  achieved = those
    # lane-instructions per second; peak = 256 CUs x 4 SIMDs x 16 fp64 lanes x 2.4 GHz
    # (= the 78.6 TFLOP/s fp64 vector peak / 2 flops per FMA).
    lane_instr_per_launch = C * G * P * N * VALU_PER_CHAIN_ROW * iters_per_launch
    valu_tips = lane_instr_per_launch / (avg_step_ms * 1e-3) / 1e12
    # LDS bytes actually delivered: one ds_read_b128 serves a row pair to the 64 lanes, i.e.
    # each (row, chain pair) once -- half the algorithmic bytes in the paired loop
    lds_delivered = bytes_per_launch / (2.0 if lc.get("kernel", "").find("Linreg<2>") >= 0 else 1.0)
    lds_gbs = lds_delivered / (avg_step_ms * 1e-3) / 1e9
    traffic, hbm_meas = None, None
    if pmc and "bytes_per_launch" in pmc:
        # measured for a K-iteration launch; scaled if this run's launches differ
        traffic = pmc["bytes_per_launch"] * iters_per_launch / pmc["iterations_per_launch"]
        hbm_meas = traffic / (avg_step_ms * 1e-3) / 1e9
    kname = lc["kernel"]

    if rank == 0:
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
            "roofline": {"bound": "valu", "achieved": valu_tips, "peak": VALU_PEAK_TIPS,
                         "unit": "T fp64 lane-instr/s", "frac": valu_tips / VALU_PEAK_TIPS,
                         "traffic": traffic,
                         "kernel": kname,
                         "avg_launch_us": avg_step_ms * 1e3,
                         "iterations_per_launch": iters_per_launch,
                         "valu_lane_instr_per_launch": lane_instr_per_launch,
                         "derivation": "achieved = C*G*P*N*3 fp64 VALU lane-instructions per "
                                       "iteration (the shipped paired row loop: 24 per 8-row "
                                       "block per 2 chains) x iterations_per_launch / "
                                       "avg_launch_us; peak = 256 CUs x 4 SIMDs x 16 fp64 lanes "
                                       "x 2.4 GHz (78.6 TFLOP/s fp64 / 2)",
                         "lds": {"delivered_gbs": lds_gbs, "peak": LDS_PEAK_GBS,
                                 "frac": lds_gbs / LDS_PEAK_GBS,
                                 "note": "bytes the ds_read_b128 of the paired loop deliver "
                                         "(each serves a row pair to 64 lanes = 2 chains per "
                                         "row): half of C*G*P*N*b_obs"},
                         "hbm": {"algorithmic_gbs": achieved_gbs, "peak": HBM_PEAK_GBS,
                                 "algorithmic_frac": achieved_gbs / HBM_PEAK_GBS,
                                 "measured_gbs": hbm_meas,
                                 "measured_frac": None if hbm_meas is None
                                 else hbm_meas / HBM_PEAK_GBS,
                                 "note": "SURVEY 8(d) prices the path at HBM; the rows are "
                                         "read from HBM once per launch and served from LDS, "
                                         "so the algorithmic frac exceeds 1 by construction; "
                                         "measured = PMC bytes of the same launch"},
                         "pmc": pmc},
            "cpu_baseline": cpu,
            "event_ms": ev_ms,
            "wall_ms": wall * 1e3,
            "enqueue_ms": t_enq * 1e3,
            "hyper_only_avg_us": (kt["hyper_ms"] / max(1, kt["hyper_launches"])) * 1e3,
            "gather_ms": gather_ms,
            "gather_error": gather_err,
        }
        print(json.dumps(out))
    eng.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
