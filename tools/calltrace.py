#!/usr/bin/env python
"""Host cost of one nmc_run call (diagnostics): bench.py's timed call (cfg 3, K iterations,
the variates prefilled by the previous call) repeated R times with NMC_TRACE_CALLS=1, so
libnestmc prints the host time of nmc_run's and nmc_synchronize's phases; this script
prints per call the Python-side wall time, the event time on the stream and the step
kernel's own time (kernel-timing events).

    python tools/calltrace.py [K] [R] [resident] [norec]

(resident=1: the calls share one resident step launch, nmc_set_resident; no kernel-timing
calls then, which would park it; norec=1: the calls' iterations are burn-in, no sample rows
written -- the recording's cost; norec=2: post-burn, thinned to one row)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
os.environ.setdefault("NMC_TRACE_CALLS", "1")


def main():
    import bench
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    res = len(sys.argv) > 3 and sys.argv[3] == "1"
    wl = dict(bench.WORKLOADS["cfg3"])
    eng, _, _ = bench.make_engine(wl, 0, 1, 0)
    W = 5
    n_iter = W + (R + 1) * K
    norec = sys.argv[4] if len(sys.argv) > 4 else "0"
    # (2: post-burn but thinned to one row -- recording off, tuning off too)
    eng.set_schedule(n_iter, n_iter - 1 if norec == "1" else W,
                     n_iter - W if norec == "2" else 1)
    eng.set_launch_iters(0)
    if res:
        eng.set_resident(True)
    eng.run(0, W)
    eng.prefill(W, W + K)
    eng.synchronize()
    for r in range(R):
        i0 = W + r * K
        kt_on = r % 2 == 1 and not res
        eng.set_kernel_timing(kt_on)
        eng.event_record(0)
        t0 = time.perf_counter()
        eng.run(i0, i0 + K)
        t_enq = time.perf_counter() - t0
        eng.event_record(1)
        eng.synchronize()
        wall = time.perf_counter() - t0
        ev = eng.event_elapsed_ms(0, 1)
        kt = eng.kernel_timing() if kt_on else None
        sys.stderr.flush()
        print("call %d: wall_us %.1f event_us %.1f enqueue_us %.1f kernel_us %s"
              % (r, wall * 1e6, ev * 1e3, t_enq * 1e6,
                 "%.1f" % (kt["step_ms"] * 1e3 / max(1, kt["step_launches"])) if kt else "-"),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
