#!/usr/bin/env python
"""Where a cfg-3 parameter step's time goes (diagnostics): nmc_k_run's control-path stamps
(kernels.h NMC_CS) of workgroup 0 in the diagnostic build.

    make -C mcmc-for-nested-data_amd/csrc cstamps
    python tools/cstamps.py [WORKLOAD] [K]

Runs bench.py's engine for WORKLOAD (default cfg3), a warm-up launch, then one launch of K
(default 20) iterations with stamps, and prints per step (shader clocks, relative to the
step's start = the control wave passing the previous barrier B): every wave's arrival at
barrier A, the first tile of every wave, the control wave's barrier-A pass, decision and
barrier-B pass; then the medians over steps 2..15.
"""

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
os.environ.setdefault("NESTMC_LIB", os.path.join(ROOT, "mcmc-for-nested-data_amd", "nestmc",
                                                 "libnestmc_cst.so"))
import numpy  # noqa: E402

WORDS = 1024 + 4 * 4096 + 512   # NMC_STAMP_WORDS


def main():
    import bench
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    wl = dict(bench.WORKLOADS[name])
    eng, _, _ = bench.make_engine(wl, 0, 1, 0)
    eng.set_schedule(5 + 3 * K, 5 + 3 * K, 1)
    eng.set_launch_iters(0)
    eng.run(0, 5)
    eng.synchronize()
    lc = eng.launch_config()
    W = lc["waves_per_group"]
    rc = eng.lib.nmc_debug_stamps(eng.h, 1, None)
    assert rc == 0, "not a stamps build"
    eng.run(5, 5 + K)
    out = (ctypes.c_uint64 * WORDS)()
    eng.lib.nmc_debug_stamps(eng.h, 0, out)
    s = numpy.frombuffer(out, dtype=numpy.uint64)[:16 * 32].astype(numpy.int64).reshape(16, 32)
    rows = []
    for si in range(1, 16):
        t0 = s[si - 1, 10]   # previous step's barrier B passed (control wave)
        if t0 == 0 or s[si, 8] == 0:
            continue
        rel = lambda v: int(v - t0) if v else None  # noqa: E731
        arrive = [rel(s[si, w]) for w in range(W)]
        first = [rel(s[si, 16 + w]) for w in range(W)]
        rows.append({"step": si, "arrive_A": arrive, "first_tile": first,
                     "A_passed": rel(s[si, 8]), "decided": rel(s[si, 9]),
                     "B_passed": rel(s[si, 10]), "w2_B_prev": rel(s[si - 1, 11]),
                     "w2_lik_entry": rel(s[si, 12]), "w2_prepared": rel(s[si, 13]),
                     "ctl_sums": rel(s[si, 14]), "ctl_finished": rel(s[si, 15]),
                     # the register-mode Gibbs wave (wave 1): entered its task, poll
                     # succeeded, payload fetched, update done, priors done
                     "g_enter": rel(s[si, 24]), "g_polled": rel(s[si, 25]),
                     "g_fetched": rel(s[si, 26]), "g_updated": rel(s[si, 27]),
                     "g_priors": rel(s[si, 28])})
    med = {}
    if rows:
        sel = [r for r in rows if r["step"] >= 2]
        arr = numpy.array([[a if a is not None else numpy.nan for a in r["arrive_A"]] for r in sel])
        fst = numpy.array([[a if a is not None else numpy.nan for a in r["first_tile"]]
                           for r in sel])
        med = {"arrive_A_per_wave": numpy.nanmedian(arr, 0).round().tolist(),
               "last_arrival_wave": numpy.bincount(numpy.nanargmax(arr, 1)).tolist(),
               "first_tile_per_wave": numpy.nanmedian(fst, 0).round().tolist(),
               "A_passed": float(numpy.median([r["A_passed"] for r in sel])),
               "decided": float(numpy.median([r["decided"] for r in sel])),
               "B_passed": float(numpy.median([r["B_passed"] for r in sel])),
               "step_cycles": float(numpy.median([r["B_passed"] for r in sel]))}
        for k in ("w2_B_prev", "w2_lik_entry", "w2_prepared", "ctl_sums", "ctl_finished",
                  "g_enter", "g_polled", "g_fetched", "g_updated", "g_priors"):
            v = [r[k] for r in sel if r[k] is not None]
            med[k] = float(numpy.median(v)) if v else None
    print(json.dumps({"workload": name, "K": K, "launch": lc, "median_steps_2_15": med,
                      "steps": rows}))
    eng.close()


if __name__ == "__main__":
    main()
