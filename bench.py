#!/usr/bin/env python
"""Benchmark: MCMC iterations of the nested-data sampler on MI355X.

Workloads (BASELINE.json configs); ``--workload`` picks one, default cfg3:

  cfg3  (the headline)  partial-pooling linear regression (sigma = 1 known, 2 parameters
        per group), 256 chains x 64 groups x 1000 observations PER GPU, synthetic data
        from RandomState(7); weak scaling (rank r runs global chains r*256..).
  cfg2  no-pooling Gaussian means (example.distribution), 256 chains x 32 groups x 500
        observations per GPU, 3 parameters; weak scaling.
  cfg4  partial-pooling regression, 1024 chains x 256 groups x 2000 observations IN TOTAL,
        sharded over the N ranks (128 per rank at N = 8); strong scaling.
  cfg5  partial pooling with the user-supplied 8-parameter logistic log-likelihood (a
        runtime-compiled DeviceLikelihood), 512 chains x 128 groups x 5000 observations in
        total, sharded over the N ranks; strong scaling.

One step = one full reference iteration (Sampler._loop body: every parameter's
Metropolis step over every (chain, group), the Gibbs hyper updates under partial
pooling, recording).  value = chains x groups x iterations / second over the whole job
(max over ranks of the timed region); no collective in the loop, one RCCL gather of the
sample stores after the timed region.

Launch:  python bench.py [--workload cfg3] [--gpus N --steps K --warmup W]
         (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py; the host
         bootstrap is nestmc.parallel.HostGroup, no PyTorch)
"""

import argparse
import json
import math
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
LDS_PEAK_GBS = 256.0 * 256 * 2.4   # 256 B/clk/CU (ds_read_b64/b128) x 256 CUs x 2.4 GHz

# fp64 VALU lane-instructions the shipped row loop issues per (chain, row, parameter step),
# by the family instance in the step kernel's name -- counted in the ISA of that loop
# (profiles/isa_*):
#   FamLinreg<2>     {x, y} rows: b0 - y (add), fma(x, b1, .), fma(e, e, acc) = 3, in the
#                    paired asm loop (24 per 8-row block for two chains per lane), the
#                    broadcast asm loop and the C++ loop alike
#   FamGaussMean<F>  per field: theta - m (add), fma(e, e, acc) = 2F
#   FamUser (cfg5)   the LOGISTIC8 row below: 7-fma dot product, y * eta, and
#                    logaddexp(0, eta) by csrc/softplus.h: 63 fp64 instructions
#                    (profiles/isa_r04_logistic8_row.txt)
VALU_PER_CHAIN_ROW = {"FamLinreg<2>": 3, "FamGaussMean<3>": 6, ("cfg5", "FamUser"): 63}

LOGISTIC8 = r"""
__device__ double nmc_user_loglik(const double* th, const double* row, const double* k) {
  double eta = th[0];
  for (int j = 0; j < 7; ++j) eta = fma(row[j], th[j + 1], eta);
  return row[7] * eta - nmc_logaddexp0(eta);
}
"""

WORKLOADS = {
    "cfg3": dict(kind="linreg", chains=256, groups=64, obs=1000, pooling="partial",
                 scaling="weak",
                 desc="cfg3 partial-pooling linear regression (sigma=1), %d chains x %d groups "
                      "x %d obs per GPU, P=%d"),
    "cfg2": dict(kind="gauss", chains=256, groups=32, obs=500, pooling="none", scaling="weak",
                 desc="cfg2 no-pooling Gaussian means (example.distribution), %d chains x %d "
                      "groups x %d obs per GPU, P=%d"),
    "cfg4": dict(kind="linreg", chains=1024, groups=256, obs=2000, pooling="partial",
                 scaling="strong",
                 desc="cfg4 partial-pooling linear regression (sigma=1), %d chains in total x "
                      "%d groups x %d obs sharded over the GPUs, P=%d"),
    "cfg5": dict(kind="user_logistic", chains=512, groups=128, obs=5000, pooling="partial",
                 scaling="strong",
                 desc="cfg5 partial pooling, user-supplied logistic log-likelihood "
                      "(DeviceLikelihood, hiprtc), %d chains in total x %d groups x %d obs "
                      "sharded over the GPUs, P=%d"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg3")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--chains", type=int, default=None,
                    help="chains per GPU (weak workloads) or in total (strong ones)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="timed window of the CPU baseline sample (0 disables)")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-resident", action="store_true",
                    help="a new step launch per call (nmc_set_resident off; the A/B)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the two rocprofv3 PMC passes that measure HBM traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--spawn-dry-run", action="store_true",
                    help="(tests) every spawned rank prints its shard and exits before any "
                         "HIP call")
    a = ap.parse_args()
    wl = dict(WORKLOADS[a.workload])
    if a.chains:
        wl["chains"] = a.chains
    a.wl = wl
    return a


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def rank_chains(wl, world, rank):
    """(first global chain id, count) of this rank: weak workloads run ``chains`` per rank,
    strong ones split the total (nestmc.parallel.shard, contiguous blocks)."""
    from nestmc.parallel import shard
    if wl["scaling"] == "weak":
        return rank * wl["chains"], wl["chains"]
    return shard(wl["chains"], world, rank)


def job_chains(wl, world):
    """Chains the whole job runs: ``chains`` per rank (weak) or in total (strong); the
    ranks' rank_chains blocks tile [0, job_chains) exactly (tests/test_bench_shard.py)."""
    return wl["chains"] * world if wl["scaling"] == "weak" else wl["chains"]


def make_problem(wl):
    """(family, names, priors, ranges) of a workload, data regenerated from its seed."""
    import scipy.stats
    from nestmc import data
    from nestmc.families import DeviceLikelihood, GaussianMean, LinearRegression, Logistic
    G, N = wl["groups"], wl["obs"]
    if wl["kind"] == "linreg":
        x, y, _, _ = data.linreg(G, N, seed=7)
        return (LinearRegression.simple(x, y, sigma=1.0), ("b0", "b1"), None,
                {"b0": [-1, 1], "b1": [0, 3]})
    if wl["kind"] == "gauss":
        mu, sd = data.example_distribution(3, G)
        return (GaussianMean.from_groups(mu, sd, [N] * G), ("a", "b", "c"),
                [scipy.stats.norm(0, 1)] * 3, None)
    X, y, _ = data.logistic(G, N, n_coef=8, seed=1)
    host = Logistic(X, y)
    fam = DeviceLikelihood(host.obs(), LOGISTIC8, 8, host_function=host)
    names = tuple("b%d" % j for j in range(8))
    return fam, names, None, {n: [-0.5, 0.5] for n in names}


def make_engine(wl, rank, world, device):
    from nestmc.engine import Engine
    from nestmc.init import init_chains
    fam, names, priors, ranges = make_problem(wl)
    G, N = wl["groups"], wl["obs"]
    sizes = [N] * G
    c0, C = rank_chains(wl, world, rank)
    eng = Engine(fam, sizes, C, wl["pooling"], priors, seed=1234, chain_base=c0,
                 device=device)
    # reference-order init of every chain (start point uniform in the example ranges /
    # drawn from the priors), likelihoods batched on the device; outside the timed region
    st = init_chains(fam, sizes, names, range(c0, c0 + C), wl["pooling"], priors, ranges,
                     False, threads=8, group_ll=eng.eval_group_ll)
    eng.set_state(st["value"], st["log_prior"], st["ll"], st["mu"], st["s2"])
    return eng, fam, C


# ---------------------------------------------------------------------------------------
# CPU baseline: the numpy oracle on this host's cores, loop-only timing
# ---------------------------------------------------------------------------------------
def _oracle_problem(wl):
    """The workload for the oracle: (Nested, names, priors, ranges), the likelihood in the
    reference's callable convention (parameter[P][n] -> ll[n])."""
    from oracle import restatement as rs
    from oracle.models import linreg_callback
    from nestmc import data
    G, N = wl["groups"], wl["obs"]
    if wl["kind"] == "linreg":
        # the reference's own callback form (example/regression.py:53-67, scipy norm)
        x, y, _, _ = data.linreg(G, N, seed=7)
        f, names, priors, ranges = (linreg_callback(x, y), ("b0", "b1"), None,
                                    {"b0": [-1, 1], "b1": [0, 3]})
    elif wl["kind"] == "gauss":
        f, names, priors, ranges = make_problem(wl)     # GaussianMean is callable
    else:
        from nestmc.families import Logistic
        X, y, _ = data.logistic(G, N, n_coef=8, seed=1)
        names = tuple("b%d" % j for j in range(8))
        f, priors, ranges = Logistic(X, y), None, {n: [-0.5, 0.5] for n in names}
    return rs.Nested(f, [N] * G), names, priors, ranges


_CPU = {}


def _cpu_init(job):
    """Pool worker: chain init (untimed), kept for the timed loop."""
    wl, chain = job
    from oracle import restatement as rs
    nested, names, priors, ranges = _oracle_problem(wl)
    st, r = rs.init_chain(nested, names, chain, wl["pooling"], priors, ranges, False)
    _CPU[chain] = (nested, st, r, priors)
    return chain


def _cpu_loop(job):
    """Pool worker: wait at the barrier, then time only the sampling loop (SURVEY 8(d):
    init excluded).  Returns (start, end) in time.time() seconds."""
    wl, chain, iters, barrier = job
    from oracle import restatement as rs
    nested, st, r, priors = _CPU[chain]
    barrier.wait()
    t0 = time.time()
    rs.run(nested, st, wl["pooling"], priors, iters, iters, 1, rs.LegacyRNG(r))
    return t0, time.time()


def _cpu_worker(args):
    (wl, chain, iters), barrier = args
    _cpu_init((wl, chain))
    return _cpu_loop((wl, chain, iters, barrier))


def cgroup_cpu_quota():
    """CPUs the cgroup's CFS quota grants this process (cgroup v2 cpu.max, or v1
    cpu.cfs_quota_us / cpu.cfs_period_us), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                return float(q) / float(per)
            return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read().strip())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read().strip())
        return q / per if q > 0 and per > 0 else None
    except (OSError, ValueError):
        return None


def cpu_cores():
    """The host cores this process may really use: the affinity mask, bounded by the cgroup's
    CPU quota when one is set (a quota of 16 CPUs runs 16 cores' worth of work however many
    processes share it).  OMP_NUM_THREADS is a BLAS-thread knob, not a core budget, and is
    ignored.  Returns (cores, affinity mask size, quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    n = aff if quota is None else min(aff, max(1, int(math.floor(quota + 1e-9))))
    return max(1, n), aff, quota


def cpu_baseline(wl, window_s):
    """The numpy oracle (a restatement of the reference's per-chain loop, legacy RNG, one
    process per chain) on this host's cores: a probe sizes the sample so the timed loop
    lasts ``window_s``; chain init is outside the timed window."""
    import multiprocessing as mp
    from oracle import restatement as rs
    cores, affinity, quota = cpu_cores()
    # warm the imports and size the sample: init one chain, one untimed iteration, then
    # time two
    nested, names, priors, ranges = _oracle_problem(wl)
    st, r = rs.init_chain(nested, names, 0, wl["pooling"], priors, ranges, False)
    rs.run(nested, st, wl["pooling"], priors, 1, 1, 1, rs.LegacyRNG(r))
    t0 = time.time()
    rs.run(nested, st, wl["pooling"], priors, 3, 3, 1, rs.LegacyRNG(r), iter_begin=1)
    per_iter = max((time.time() - t0) / 2.0, 1e-4)
    iters = max(2, int(math.ceil(window_s / per_iter)))
    ctx = mp.get_context("fork")
    with ctx.Manager() as man:
        barrier = man.Barrier(cores)
        with ctx.Pool(cores) as pool:
            spans = pool.map(_cpu_worker, [((wl, c, iters), barrier) for c in range(cores)],
                             chunksize=1)
    t_start = min(s for s, _ in spans)
    t_end = max(e for _, e in spans)
    wall = t_end - t_start
    # each process's own loop rate, summed: what the cores sustain together, without the
    # start skew of the fork pool or one straggler on a shared host stretching the window
    per = sorted(wl["groups"] * iters / (e - s) for s, e in spans)
    rate = sum(per)
    out = {"value": rate, "unit": "chain*group*iter/s", "cores": cores, "kind": "port",
           "sample": "%d chains x %d iterations of the %s workload (%d groups x %d obs, %s "
                     "pooling) in the numpy oracle, one process per chain on %d cores (the "
                     "process's affinity mask holds %d cores; cgroup CPU quota %s); timed loop "
                     "only (init excluded), each process's loop rate summed; %.1f s from the "
                     "first start to the last end"
                     % (cores, iters, wl.get("name", "?"), wl["groups"], wl["obs"],
                        wl["pooling"], cores, affinity,
                        "none" if quota is None else "%.1f CPUs" % quota, wall),
           "affinity_cores": affinity, "cgroup_quota_cpus": quota,
           "timed_seconds": wall, "iterations": iters,
           "value_wall": cores * wl["groups"] * iters / wall,
           "per_process_min_max": [per[0], per[-1]]}
    cal = os.path.join(ROOT, "profiles", "cpu_calibration_r03.json")
    if wl.get("name") == "cfg3" and os.path.exists(cal):
        # the reference cannot travel to this box: its speed relative to the restatement
        # was measured side by side in the build container (oracle/calibrate_cpu.py)
        ratio = json.load(open(cal))["reference_over_restatement"]
        out["calibration"] = {"reference_over_restatement": ratio,
                              "source": "profiles/cpu_calibration_r03.json "
                                        "(oracle/calibrate_cpu.py, build container)"}
        out["reference_equivalent_value"] = rate * ratio
    return out


# ---------------------------------------------------------------------------------------
# HBM traffic: two rocprofv3 PMC passes of this script's K-iteration launch
# ---------------------------------------------------------------------------------------
def pmc_child(args):
    """Runs under rocprofv3 --pmc: the same workload and launches as the timed region
    (warmup launch of W iterations, then one launch of K iterations)."""
    from nestmc import _lib
    eng, _, _ = make_engine(args.wl, 0, 1, 0)
    W, K = args.warmup, args.steps
    eng.set_schedule(*bench_schedule(W, K))
    eng.run(0, W)
    eng.prefill(W, W + K)
    eng.run(W, W + K)
    eng.synchronize()
    info = os.environ.get("NMC_PMC_INFO")
    if info:   # what the counted launches ran (the parent reports it beside the bytes)
        with open(info, "w") as f:
            json.dump({"kernel": eng.launch_config()["kernel"],
                       "gibbs_fallbacks": eng.gibbs_fallbacks()}, f)
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
    out, info = {}, {}
    base = tempfile.mkdtemp(prefix="nmc_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp", NMC_PMC_INFO=os.path.join(base, "info.json"))
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(base, counter)
            cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc",
                   "--", "python3", os.path.abspath(__file__), "--pmc-child",
                   "--workload", args.workload,
                   "--steps", str(args.steps), "--warmup", str(args.warmup),
                   "--chains", str(args.wl["chains"])]
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
                        kn = row.get("Kernel_Name", "")
                        if row.get("Counter_Name") == counter and \
                                ("nmc_k_run" in kn or "nmc_k_sweep" in kn) and \
                                "nmc_k_sweep_gibbs" not in kn:
                            rows.append((int(row.get("Dispatch_Id", 0)),
                                         float(row["Counter_Value"])))
            if len(rows) < 2:
                return {"error": "no %s rows for the step kernel" % counter}
            out[counter] = sorted(rows)[-1][1]       # the K-iteration launch (the last)
            try:
                info = json.load(open(env["NMC_PMC_INFO"]))
            except (OSError, ValueError):
                pass
    finally:
        shutil.rmtree(base, ignore_errors=True)
    read_b = 2.0 * out["FETCH_SIZE"] * 1024.0
    write_b = out["WRITE_SIZE"] * 1024.0
    res = {}
    if info.get("gibbs_fallbacks"):
        # counter collection serializes dispatches: the Gibbs kernel of the G > 128 path did
        # not run beside the step kernel, so the step kernel updated its Gibbs tasks itself
        # (the same results) -- these bytes are that serialized form's
        res["gibbs_fallbacks"] = info["gibbs_fallbacks"]
        res["note"] = ("rocprofv3 --pmc serializes kernels: the counted launches ran the "
                       "step kernel updating its own Gibbs tasks (nmc_gibbs_fallbacks = %d), "
                       "not beside its Gibbs kernel" % info["gibbs_fallbacks"])
    return dict(res, **{"bytes_per_launch": read_b + write_b, "read_bytes": read_b,
                        "write_bytes": write_b,
            "fetch_size_kib_raw": out["FETCH_SIZE"], "write_size_kib_raw": out["WRITE_SIZE"],
            "iterations_per_launch": args.steps,
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of this "
                      "script's K-iteration launch; FETCH_SIZE x2 (gfx950), KiB -> bytes"})


def fam_instance(kernel):
    """'FamLinreg<2>' out of 'nmc_k_run<FamLinreg<2>, NMC_MODE_..., true>', 'FamUser' out of
    'nmc_k_run<FamUser, NMC_MODE_SYNC, false>': the first template argument."""
    i = kernel.find("<")
    if i < 0:
        return kernel
    depth = 0
    for j in range(i + 1, len(kernel)):
        ch = kernel[j]
        if ch == "<":
            depth += 1
        elif ch == ">":
            if depth == 0:
                return kernel[i + 1:j].strip()
            depth -= 1
        elif ch == "," and depth == 0:
            return kernel[i + 1:j].strip()
    return kernel[i + 1:].strip()


def bench_schedule(W, K):
    """(n_iter, burn, thin) of a run of W warm-up and 2K measured iterations: the burn-in is
    the warm-up, so every iteration from W on -- the timed call [W, W + K) and the
    kernel-timing call after it -- is post-burn and recorded (thin 1), the steady state of
    the reference's sampling loop (posteriorSampling.py:883-891, every post-burn iteration
    of the cfg written as a sample row)."""
    return W + 2 * K, W, 1


def recorded_in(lo, hi, n_iter, burn, thin):
    """How many iterations of [lo, hi) write a sample row under (n_iter, burn, thin)
    (nmc_record_row: post-burn, on the thinning grid)."""
    first = ((burn + thin - 1) // thin) * thin
    return sum(1 for i in range(max(lo, first), min(hi, n_iter)) if i % thin == 0)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args):
    """``--gpus N`` (N > 1) without a launcher: this process starts N ranks itself, one per
    GPU, as child processes with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT) -- before it makes any HIP call -- and relays rank 0's JSON
    line; any failed rank fails the run.  The CPU-baseline leg runs here, before the
    spawn, and is attached to the line (the ranks skip it and the PMC passes).  Replaces the
    reference's process fan-out (posteriorSampling.py:182-201) at the GPU level."""
    import subprocess
    cpu = None
    if args.cpu_seconds > 0 and not args.spawn_dry_run:
        try:
            cpu = cpu_baseline(args.wl, args.cpu_seconds)
        except Exception as e:
            cpu = {"value": None, "error": repr(e)}
    n = args.gpus
    port, bport = _free_port(), _free_port()
    argv = [sys.executable, os.path.abspath(__file__)] + [
        a for a in sys.argv[1:] if a not in ("--no-pmc",)] + ["--no-pmc", "--cpu-seconds", "0"]
    import tempfile
    procs, files = [], []
    tmp = tempfile.mkdtemp(prefix="nmc_bench_ranks_")
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       NMC_BOOTSTRAP_PORT=str(bport))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            # (stdout to a file, not a pipe: the ranks are polled together, none can block
            #  on a full pipe while another is waited for)
            files.append(open(os.path.join(tmp, "rank%d.out" % r), "w+"))
            procs.append(subprocess.Popen(argv, env=env, stdout=files[-1], text=True,
                                          start_new_session=True))
        from nestmc.ranks import wait_all
        bad = wait_all(procs)
        if bad:
            print("bench.py: rank(s) failed: %s" % (bad,), file=sys.stderr)
            return 1
        outs = []
        for f in files:
            f.seek(0)
            outs.append(f.read())
    finally:
        for f in files:
            f.close()
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    lines = [[ln for ln in o.splitlines() if ln.startswith("{")] for o in outs]
    if not lines[0]:
        print("bench.py: rank 0 printed no JSON line", file=sys.stderr)
        return 1
    out = json.loads(lines[0][-1])
    if args.spawn_dry_run:
        out["ranks"] = [json.loads(ls[-1]) for ls in lines]
    else:
        out["cpu_baseline"] = cpu
        out["launcher"] = "bench.py --gpus %d: %d child ranks" % (n, n)
    print(json.dumps(out))
    return 0


def main():
    args = parse()
    wl = args.wl
    wl["name"] = args.workload
    world, rank, local = dist_env()
    if args.pmc_child:
        return pmc_child(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    if args.gpus != world and world > 1:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    if args.spawn_dry_run:
        # (tests) the rank's view of the job, before any HIP call
        c0, C = rank_chains(wl, world, rank)
        print(json.dumps({"dry_run": True, "rank": rank, "local_rank": local, "n_gpus": world,
                          "workload": args.workload, "chain_base": c0, "chains": C,
                          "chains_total": job_chains(wl, world), "scaling": wl["scaling"],
                          "libnestmc_mapped": "libnestmc" in open("/proc/self/maps").read()}))
        return 0
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
                cpu = cpu_baseline(wl, args.cpu_seconds)
            except Exception as e:
                cpu = {"value": None, "error": repr(e)}
    from nestmc import _lib
    from nestmc import parallel
    hg = parallel.HostGroup(world, rank) if world > 1 else None

    n_dev = _lib.device_count()
    assert n_dev >= 1, "no HIP device visible"
    device = local % n_dev
    eng, fam, C = make_engine(wl, rank, world, device)
    K, W = args.steps, args.warmup
    # schedule: the warm-up is the burn-in, every measured iteration records a sample row
    n_iter, burn, thin = bench_schedule(W, K)
    eng.set_schedule(n_iter, burn, thin)
    # the sampling loop's calls share one resident step launch (nmc_set_resident): a call
    # continuing the last is handed to the running launch, closed as a launch is closed
    if not args.no_resident:
        eng.set_resident(True)
    # production launch length: one persistent launch per nmc_run call (up to the
    # variate chunk), exactly as samplePosterior drives the engine -- the warmup is
    # its own launch, the timed region one launch of K iterations
    eng.set_launch_iters(0)
    eng.run(0, W)
    # the variates of the timed call, drawn as the previous call of a sampling loop draws
    # its successor's beside its own step launch (nmc_run's pipelined fill): the timed call
    # then draws the NEXT call's K iterations beside its step launch -- the timed region holds
    # exactly one K-iteration fill and one K-iteration step launch (checked below)
    eng.prefill(W, W + K)
    eng.synchronize()

    def barrier():
        if hg is not None:
            hg.barrier()

    # timed region: exactly K iterations
    barrier()
    eng.synchronize()
    pf0 = eng.prefill_stats()
    eng.event_record(0)
    t0 = time.perf_counter()
    eng.run(W, W + K)
    t_enq = time.perf_counter() - t0          # host time to enqueue the launch(es)
    eng.event_record(1)
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    pf1 = eng.prefill_stats()
    res1 = eng.resident_stats()
    # variate fill inside the timed region: iterations drawn on the prefill stream
    # (beside the step launches), iterations taken from the prefill made before it, and the
    # rest drawn on the step stream ahead of their launch
    fill = {"pipelined": pf1["issued"] > pf0["issued"] or pf1["used"] > pf0["used"],
            "drawn_beside_step_iters": pf1["issued"] - pf0["issued"],
            "taken_from_prefill_iters": pf1["used"] - pf0["used"],
            "drawn_ahead_iters": K - (pf1["used"] - pf0["used"])}
    fill["drawn_in_timed_region_iters"] = (fill["drawn_beside_step_iters"] +
                                           fill["drawn_ahead_iters"])
    wall = t1 - t0
    ev_ms = eng.event_elapsed_ms(0, 1)
    t_rank = max(wall, ev_ms / 1e3)
    t_max = parallel.max_over_ranks(t_rank, hg)
    c_total = job_chains(wl, world)

    # second pass, same length: per-launch events on the engine's stream -> the
    # step kernel's average duration for the roofline
    eng.set_kernel_timing(True)
    eng.run(W + K, W + 2 * K)
    kt = eng.kernel_timing()
    eng.set_kernel_timing(False)
    # (G > 128: launches whose step kernel updated its own Gibbs tasks because the Gibbs
    #  kernel did not run beside it -- 0 when the two kernels were co-scheduled)
    gibbs_fb = eng.gibbs_fallbacks()

    gather_ms, gather_err = None, None
    if world > 1 and not args.no_gather:
        # after the timed region: the one RCCL gather of the sample stores; a
        # failure here is reported in the line, never lost with it
        try:
            comm = parallel.rccl_comm(hg, world, rank, device)
            tg = time.perf_counter()
            full = parallel.gather_samples(eng, comm, root=0)
            gather_ms = (time.perf_counter() - tg) * 1e3
            parallel.rccl_destroy(comm)
            del full
        except Exception as e:
            gather_err = repr(e)

    G, N, P = wl["groups"], wl["obs"], fam.n_params
    units = c_total * G * K
    value = units / t_max
    launches = kt["step_launches"]
    avg_step_ms = kt["step_ms"] / max(1, launches)
    iters_per_launch = kt["step_iters"] / max(1, launches)
    b_obs = fam.bytes_per_obs()
    lc = eng.launch_config()
    kname = lc["kernel"]
    inst = fam_instance(kname)
    # B_unit = P*N*b_obs per chain*group*iteration (each parameter step
    # evaluates the group's rows once per chain), for THIS rank's chains per launch
    bytes_per_launch = C * G * P * N * b_obs * iters_per_launch
    achieved_gbs = bytes_per_launch / (avg_step_ms * 1e-3) / 1e9
    # The binding resource is fp64 VALU issue: the lane-instructions of the shipped row loop
    # per (chain, row, parameter step), counted in its ISA for this family instance (null
    # for an instance whose loop has not been counted)
    per_row = VALU_PER_CHAIN_ROW.get(inst, VALU_PER_CHAIN_ROW.get((args.workload, inst)))
    if per_row is not None:
        lane_instr_per_launch = C * G * P * N * per_row * iters_per_launch
        valu_tips = lane_instr_per_launch / (avg_step_ms * 1e-3) / 1e12
    else:
        lane_instr_per_launch, valu_tips = None, None
    # LDS bytes actually delivered: the paired loop's ds_read_b128 serves a row pair to the
    # 64 lanes, i.e. each (row, chain pair) once -- half the algorithmic bytes
    paired = "Linreg<2>" in inst or "GaussMean" in inst
    lds_delivered = bytes_per_launch / (2.0 if paired else 1.0)
    lds_gbs = lds_delivered / (avg_step_ms * 1e-3) / 1e9
    traffic, hbm_meas = None, None
    if pmc and "bytes_per_launch" in pmc:
        # measured for a K-iteration launch; scaled if this run's launches differ
        traffic = pmc["bytes_per_launch"] * iters_per_launch / pmc["iterations_per_launch"]
        hbm_meas = traffic / (avg_step_ms * 1e-3) / 1e9

    if rank == 0:
        desc = wl["desc"] % (wl["chains"], G, N, P)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "chain*group*iter/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": t_max * 1e3 / K,
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": desc, "name": args.workload,
                       "chains_total": c_total, "chains_per_gpu": C, "groups": G,
                       "obs_per_group": N, "params": P, "pooling": wl["pooling"],
                       "parallelism": "chains sharded x%d" % world, "launch": lc,
                       "recorded_iters_in_timed_region": recorded_in(W, W + K, n_iter, burn,
                                                                     thin),
                       "gibbs_fallbacks": gibbs_fb,
                       # the timed call ran inside the resident launch the warm-up started
                       # (its GPU span is event_ms); the kernel-timing pass and the PMC
                       # passes use separate launches of the same K iterations
                       "resident": dict(res1, timed_call_resident=res1["calls"] > 0)},
            "roofline": {"bound": "valu", "achieved": valu_tips, "peak": VALU_PEAK_TIPS,
                         "unit": "T fp64 lane-instr/s",
                         "frac": None if valu_tips is None else valu_tips / VALU_PEAK_TIPS,
                         "traffic": traffic,
                         "kernel": kname,
                         "avg_launch_us": avg_step_ms * 1e3,
                         "iterations_per_launch": iters_per_launch,
                         "valu_per_chain_row": per_row,
                         "valu_lane_instr_per_launch": lane_instr_per_launch,
                         "derivation": "achieved = C*G*P*N*valu_per_chain_row fp64 VALU "
                                       "lane-instructions per iteration (the shipped row loop "
                                       "of this family instance, counted in its ISA) x "
                                       "iterations_per_launch / avg_launch_us (this rank's "
                                       "chains); peak = 256 CUs x 4 SIMDs x 16 fp64 lanes x "
                                       "2.4 GHz (78.6 TFLOP/s fp64 / 2)",
                         "lds": {"delivered_gbs": lds_gbs, "peak": LDS_PEAK_GBS,
                                 "frac": lds_gbs / LDS_PEAK_GBS,
                                 "note": "bytes the row loop's LDS reads deliver (paired loop: "
                                         "one read serves a row pair to 64 lanes = 2 chains per "
                                         "row, half of C*G*P*N*b_obs)"},
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
            "variate_fill": fill,
        }
        print(json.dumps(out))
    eng.close()
    if hg is not None:
        hg.barrier()
        hg.close()


if __name__ == "__main__":
    sys.exit(main() or 0)
