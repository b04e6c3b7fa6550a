#!/usr/bin/env python
"""Per-tile timeline of the step kernel (diagnostic stamps build): for the first steps
of a launch, which wave ran which likelihood tile and when, relative to the step's
first tile start.  make -C mcmc-for-nested-data_amd/csrc stamps; python tools/tilegantt.py"""

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


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    eng, fam = engine_for("linreg", 256, 64, N, "partial", 0)
    eng.set_schedule(400, 400, 1)
    eng.run(0, 100)
    eng.synchronize()
    eng.lib.nmc_debug_stamps(eng.h, 1, None)
    eng.run(100, 120)
    out = (ctypes.c_uint64 * (1024 + 4 * 4096 + 512))()   # NMC_STAMP_WORDS
    eng.lib.nmc_debug_stamps(eng.h, 0, out)
    st = numpy.frombuffer(out, dtype=numpy.uint64).astype(numpy.float64)
    ph = st[:512].reshape(2, 2, 8, 16)
    ts = st[512:1024].reshape(8, 16, 4)
    res = []
    for s in range(2, 8):
        tiles = [(k, int(ts[s, k, 2]), ts[s, k, 0], ts[s, k, 1]) for k in range(16) if ts[s, k, 1] > 0]
        t0 = min(a for _, _, a, _ in tiles)
        waves = {}
        for k, w, a, b in tiles:
            waves.setdefault(w, []).append((k, int(a - t0), int(b - a)))
        res.append({"step": s, "span": int(max(b for _, _, _, b in tiles) - t0),
                    "waves": {str(w): v for w, v in sorted(waves.items())}})
    print(json.dumps(dict(N=N, config=eng.launch_config(), tiles=res)))
    eng.close()


if __name__ == "__main__":
    main()
