#!/usr/bin/env python
"""Timeline of the one-barrier step kernel nmc_k_step (diagnostics, stamps build only).

    make -C mcmc-for-nested-data_amd/csrc stamps
    python tools/steptl.py [kind C G N pooling iters]     (default: cfg 3, 20 iterations)

Runs a warm-up launch, then one launch of `iters` iterations with the stamps armed, and
prints one JSON line:
  * steps: workgroup 0, launch steps 1..7, medians over steps of each wave's phases in
    shader cycles -- role work (control: bookkeeping, operands, next z; Gibbs: poll,
    fetch, update), tiles, barrier wait, decision -- and the step period;
  * launch: over every workgroup (s_memrealtime, 100 MHz): entry spread after the first
    workgroup's entry, prologue, loop and closing (drain) durations, in microseconds.
"""

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("NESTMC_LIB", os.path.join(ROOT, "mcmc-for-nested-data_amd", "nestmc",
                                                 "libnestmc_stamps.so"))
import numpy  # noqa: E402

from kbench import engine_for  # noqa: E402

WORDS = 1024 + 4 * 4096 + 512


def main():
    a = sys.argv[1:]
    kind = a[0] if len(a) > 0 else "linreg"
    C, G, N = (int(v) for v in a[1:4]) if len(a) > 3 else (256, 64, 1000)
    pooling = a[4] if len(a) > 4 else "partial"
    iters = int(a[5]) if len(a) > 5 else 20
    eng, fam = engine_for(kind, C, G, N, pooling, 0)
    eng.set_schedule(200 + iters, 200 + iters, 1)
    eng.run(0, 200)
    eng.synchronize()
    eng.lib.nmc_debug_stamps(eng.h, 1, None)
    eng.event_record(0)
    eng.run(200, 200 + iters)
    eng.event_record(1)
    ms = eng.event_elapsed_ms(0, 1)
    out = (ctypes.c_uint64 * WORDS)()
    eng.lib.nmc_debug_stamps(eng.h, 0, out)
    st = numpy.frombuffer(out, dtype=numpy.uint64).astype(numpy.float64)
    cfg = eng.launch_config()
    W = cfg["waves_per_group"]
    ph = st[:512].reshape(8, 8, 8)[:W]            # [wave][step][slot]
    steps = {}
    for w in range(W):
        s = ph[w, 1:8]
        period = numpy.diff(ph[w, :, 0])[1:7]
        steps["w%d" % w] = {
            "role": float(numpy.median(s[:, 1] - s[:, 0])),
            "tiles": float(numpy.median(s[:, 2] - s[:, 1])),
            "barrier": float(numpy.median(s[:, 3] - s[:, 2])),
            "decide": float(numpy.median(s[:, 4] - s[:, 3])),
            "period": float(numpy.median(period)),
        }
    nb = cfg["chain_blocks"] * G * cfg["split_members"]
    lt = st[1024:1024 + 4 * nb].reshape(nb, 4) / 100.0   # microseconds
    ok = lt[:, 0] > 0
    lt = lt[ok]
    e0 = lt[:, 0].min()
    q = lambda v: [float(numpy.percentile(v, p)) for p in (0, 50, 100)]   # noqa: E731
    launch = {"workgroups": int(ok.sum()),
              "entry_after_first_us": q(lt[:, 0] - e0),
              "prologue_us": q(lt[:, 1] - lt[:, 0]),
              "loop_us": q(lt[:, 2] - lt[:, 1]),
              "closing_us": q(lt[:, 3] - lt[:, 2]),
              "first_entry_to_last_exit_us": float(lt[:, 3].max() - e0),
              "event_ms": ms, "iterations": iters}
    print(json.dumps(dict(kind=kind, C=C, G=G, N=N, pooling=pooling, config=cfg,
                          steps_cycles=steps, launch=launch)))
    eng.close()


if __name__ == "__main__":
    main()
