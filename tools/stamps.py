#!/usr/bin/env python
"""Phase timing of one step launch from the diagnostic stamps build.

    make -C mcmc-for-nested-data_amd/csrc stamps
    NESTMC_LIB=.../libnestmc_stamps.so python tools/stamps.py

Slots (100 MHz s_memrealtime, 10 ns ticks), wave 0: 0 entry, 1 prologue done
(rows staged, state loaded, Gibbs update), 2 all parameter steps done, 3 end.
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("NESTMC_LIB", os.path.join(ROOT, "mcmc-for-nested-data_amd", "nestmc",
                                                 "libnestmc_stamps.so"))

import ctypes  # noqa: E402

import numpy  # noqa: E402

from kbench import engine_for  # noqa: E402


def main():
    kind, C, G, N, pooling = "linreg", 256, 64, 1000, sys.argv[1] if len(sys.argv) > 1 else "partial"
    waves = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    eng, fam = engine_for(kind, C, G, N, pooling, waves)
    eng.set_schedule(400, 400, 1)
    eng.run(0, 200)
    eng.synchronize()
    cfg = eng.launch_config()
    CB = cfg["chain_blocks"]
    nb = CB * G
    res = []
    for it in range(200, 210):
        eng.lib.nmc_debug_stamps(eng.h, nb, None)
        eng.run(it, it + 1)
        out = (ctypes.c_uint64 * (nb * 8))()
        eng.lib.nmc_debug_stamps(eng.h, 0, out)
        st = numpy.frombuffer(out, dtype=numpy.uint64).reshape(nb, 8).astype(numpy.float64)
        t0 = st[:, 0].min()
        q = lambda a: (float(numpy.percentile(a, 50)) * 10, float(numpy.max(a)) * 10)  # noqa
        res.append(dict(
            entry_spread_ns=q(st[:, 0] - t0),
            prologue_ns=q(st[:, 1] - st[:, 0]),
            steps_ns=q(st[:, 2] - st[:, 1]),
            epilogue_ns=q(st[:, 3] - st[:, 2]),
            step0_ll_ns=q(st[:, 7] - st[:, 1]),
            step0_barrier1_ns=q(st[:, 4] - st[:, 1]),
            step0_decision_ns=q(st[:, 5] - st[:, 4]),
            step0_barrier2_ns=q(st[:, 6] - st[:, 5]),
            wg_total_ns=q(st[:, 3] - st[:, 0]),
            launch_span_ns=float(st[:, 3].max() - t0) * 10))
    print(json.dumps(dict(config=cfg, pooling=pooling, phases=res[-1],
                          span_all=[r["launch_span_ns"] for r in res])))
    eng.close()


if __name__ == "__main__":
    main()
