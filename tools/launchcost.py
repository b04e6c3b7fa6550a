#!/usr/bin/env python
"""Fixed cost of one nmc_run (diagnostics, not the contract bench): the cfg-3 engine of
bench.py, one launch of K iterations for K in a sweep, timed four ways --
  wall      host clock around run() + synchronize() (what bench.py's value uses),
  event     HIP events on the engine stream around the whole call (fill + step kernel),
  kernel    HIP events around the step kernel alone,
  sync      host clock of synchronize() on an idle stream.
A least-squares fit kernel(K) = a + b K separates the in-kernel ramp/drain (a) from the
steady-state iteration (b).  Run under rocprofv3 --kernel-trace to see the fill and gaps.

    python tools/launchcost.py [K ...]
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))

import numpy  # noqa: E402


def main():
    import bench
    ks = [int(a) for a in sys.argv[1:]] or [1, 2, 5, 10, 20, 50, 100, 400]

    wl = dict(bench.WORKLOADS[os.environ.get("WORKLOAD", "cfg3")])
    eng, _, _ = bench.make_engine(wl, 0, 1, 0)
    total = 5 + 3 * 3 * sum(ks) + 10
    eng.set_schedule(total, total // 2, 1)
    eng.set_launch_iters(0)
    it = 0
    eng.run(it, it + 5)
    it += 5
    eng.synchronize()
    # idle synchronize
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        eng.synchronize()
        ts.append(time.perf_counter() - t0)
    rows = []
    for K in ks:
        walls, evs, kers = [], [], []
        for rep in range(3):
            eng.synchronize()
            eng.event_record(0)
            t0 = time.perf_counter()
            eng.run(it, it + K)
            eng.event_record(1)
            eng.synchronize()
            walls.append(time.perf_counter() - t0)
            evs.append(eng.event_elapsed_ms(0, 1) * 1e-3)
            it += K
            eng.set_kernel_timing(True)
            eng.run(it, it + K)
            kt = eng.kernel_timing()
            eng.set_kernel_timing(False)
            eng.synchronize()
            kers.append(kt["step_ms"] * 1e-3 / max(1, kt["step_launches"]))
            it += K
        rows.append(dict(K=K, wall_us=1e6 * min(walls), event_us=1e6 * min(evs),
                         kernel_us=1e6 * min(kers), wall_us_med=1e6 * float(numpy.median(walls))))
    K = numpy.array([r["K"] for r in rows], float)
    kern = numpy.array([r["kernel_us"] for r in rows])
    b, a = numpy.polyfit(K, kern, 1)
    out = dict(rows=rows, fit_kernel_us={"fixed": a, "per_iter": b},
               idle_sync_us=1e6 * float(numpy.median(ts)), launch=eng.launch_config())
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
