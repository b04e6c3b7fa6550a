#!/usr/bin/env python
"""Kernel-level sweep (diagnostics, not the contract bench): per-launch step-kernel
time for the cfg-3 workload under different poolings / waves-per-group, so the
Metropolis step, the Gibbs update and launch overhead can be told apart."""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))

import numpy  # noqa: E402
import scipy.stats  # noqa: E402

from nestmc import data  # noqa: E402
from nestmc.engine import Engine  # noqa: E402
from nestmc.families import LinearRegression, Logistic, GaussianMean  # noqa: E402


def engine_for(kind, C, G, N, pooling, waves, persist=None):
    if persist is None:
        os.environ.pop("NMC_PERSIST", None)
    else:
        os.environ["NMC_PERSIST"] = str(int(persist))
    if waves:
        os.environ["NMC_WAVES"] = str(waves)
    else:
        os.environ.pop("NMC_WAVES", None)
    r = numpy.random.RandomState(0)
    if kind == "linreg":
        x, y, _, _ = data.linreg(G, N, seed=7)
        fam = LinearRegression.simple(x, y, sigma=1.0)
        start = numpy.array([0.0, 2.0])
    elif kind == "logistic":
        X, y, _ = data.logistic(G, N, n_coef=8, seed=1)
        fam = Logistic(X, y)
        if os.environ.get("KB_USER_SOURCE"):   # the same model as a user family (hiprtc)
            from nestmc.families import DeviceLikelihood
            fam = DeviceLikelihood(fam.obs(), os.environ["KB_USER_SOURCE"], fam.n_params,
                                   host_function=fam)
        start = numpy.zeros(8)
    else:
        mu, sd = data.example_distribution(3, G)
        fam = GaussianMean.from_groups(mu, sd, [N] * G)
        start = numpy.zeros(3)
    P = fam.n_params
    priors = [scipy.stats.norm(0, 10)] * P if pooling != "partial" else None
    eng = Engine(fam, [N] * G, C, pooling, priors, seed=1)
    value = start[None, :, None] + 0.1 * r.normal(size=(C, P, G))
    if pooling == "partial":
        mu = numpy.tile(start, (C, 1))
        s2 = numpy.full((C, P), 0.5)
        lp = numpy.zeros((C, P, G))
        ll = eng.eval_group_ll(value)
        eng.set_state(value, lp, ll, mu, s2)
    else:
        lp = numpy.zeros((C, P, G))
        eng.set_state(value, lp, numpy.full((C, G), numpy.nan))
    return eng, fam


def run(kind, C, G, N, pooling, waves, iters, persist=None):
    eng, fam = engine_for(kind, C, G, N, pooling, waves, persist)
    eng.set_schedule(3 * iters, 3 * iters, 1)
    eng.run(0, iters)
    eng.synchronize()
    eng.event_record(0)
    t0 = time.perf_counter()
    eng.run(iters, 2 * iters)
    eng.event_record(1)
    eng.synchronize()
    wall = time.perf_counter() - t0
    ms = eng.event_elapsed_ms(0, 1)
    eng.set_kernel_timing(True)
    eng.run(2 * iters, 3 * iters)
    kt = eng.kernel_timing()
    cfg = eng.launch_config()
    eng.close()
    rate = C * G * iters / (ms / 1e3)
    return dict(kind=kind, C=C, G=G, N=N, pooling=pooling, waves=cfg["waves_per_group"],
                persistent=cfg["persistent"], split_members=cfg["split_members"],
                us_per_iter=ms * 1e3 / iters, wall_us_per_iter=wall * 1e6 / iters,
                step_us_per_iter=kt["step_ms"] * 1e3 / max(1, kt["step_iters"]),
                hyper_us=kt["hyper_ms"] * 1e3 / max(1, kt["hyper_launches"]),
                rate=rate, kernel=cfg["kernel"], mode=cfg["mode"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="rows-per-group sweep (cost model)")
    ap.add_argument("--complete", action="store_true",
                    help="complete pooling at large n_total: row split vs one workgroup")
    a = ap.parse_args()
    if a.complete:
        cases = [(C, N, sp) for C, N in ((64, 100000), (256, 100000), (1024, 512000))
                 for sp in (None, "1")]
        if os.environ.get("KB_SPLITS"):   # explicit member counts (diagnostics)
            cases = [(int(C), int(N), sp) for C, N, sp in
                     (t.split(":") for t in os.environ["KB_SPLITS"].split(","))]
        for C, N, split in cases:
            if True:
                if split:
                    os.environ["NMC_SPLIT"] = split
                else:
                    os.environ.pop("NMC_SPLIT", None)
                iters = 40 if split == "1" else 200
                r = run("linreg", C, 1, N, "complete", 0, iters)
                r["split"] = "default" if split is None else split
                print(json.dumps(r), flush=True)
        os.environ.pop("NMC_SPLIT", None)
        return
    if a.sweep:
        for rows in ("lds", "smem"):
            if rows == "smem":
                os.environ["NMC_NO_LDS_ROWS"] = "1"
            for pooling in ("none", "partial"):
                for N in (250, 1000, 2000, 4000):
                    r = run("linreg", 256, 64, N, pooling, 16, a.iters)
                    r["rows"] = rows
                    print(json.dumps(r), flush=True)
            os.environ.pop("NMC_NO_LDS_ROWS", None)
        return
    cases = [("linreg", 256, 64, 1000, "partial", w) for w in (0, 4, 8, 16)]
    cases += [("linreg", 256, 64, 1000, "none", w) for w in (0, 8)]
    if not a.quick:
        cases += [("linreg", 1024, 256, 2000, "partial", 0),
                  ("linreg", 128, 256, 2000, "partial", 0),      # cfg 4, one rank of 8
                  ("gauss", 256, 32, 500, "none", 0),
                  ("logistic", 64, 128, 5000, "partial", 0)]
    for c in cases:
        iters = a.iters if c[3] * c[1] * c[2] < 5e7 else max(20, a.iters // 10)
        print(json.dumps(run(*c, iters)), flush=True)
    # launch-per-iteration partial pooling (the non-resident fallback)
    print(json.dumps(run("linreg", 256, 64, 1000, "partial", 0, a.iters, persist=False)),
          flush=True)


if __name__ == "__main__":
    main()
