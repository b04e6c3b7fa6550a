#!/usr/bin/env python
"""Launch timeline of the step kernel nmc_k_run (diagnostics, stamps build only):
where a short launch's fixed cost goes.

    make -C mcmc-for-nested-data_amd/csrc stamps
    python tools/launchtl.py [K ...]          (cfg 3; default K = 1 2 20)

For each K: a warm-up, then one launch of K iterations with the stamps armed; over every
workgroup (s_memrealtime, 100 MHz): entry spread after the first workgroup's entry, the
prologue (state and rows to LDS, first variates), the loop, and the closing (last Gibbs
tasks, state back to HBM), in microseconds (min / median / max), beside the HIP-event
time of the launch.
"""

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
os.environ.setdefault("NESTMC_LIB", os.path.join(ROOT, "mcmc-for-nested-data_amd", "nestmc",
                                                 "libnestmc_stamps.so"))
import numpy  # noqa: E402

WORDS = 1024 + 4 * 4096 + 512


def main():
    import bench
    ks = [int(v) for v in sys.argv[1:]] or [1, 2, 20]

    class A:
        chains, groups, obs = 256, 64, 1000
    eng, _ = bench.make_engine(A, 0, 0)
    total = 10 + 2 * sum(ks)
    eng.set_schedule(total, total // 2, 1)
    it = 0
    eng.run(it, it + 5)
    it += 5
    eng.synchronize()
    cfg = eng.launch_config()
    nb = cfg["chain_blocks"] * A.groups * cfg["split_members"]
    q = lambda v: [round(float(numpy.percentile(v, p)), 2) for p in (0, 50, 100)]   # noqa: E731
    for K in ks:
        eng.run(it, it + K)          # same-length warm-up
        it += K
        eng.synchronize()
        eng.lib.nmc_debug_stamps(eng.h, 1, None)
        eng.set_kernel_timing(True)
        eng.run(it, it + K)
        kt = eng.kernel_timing()
        eng.set_kernel_timing(False)
        it += K
        out = (ctypes.c_uint64 * WORDS)()
        eng.lib.nmc_debug_stamps(eng.h, 0, out)
        st = numpy.frombuffer(out, dtype=numpy.uint64).astype(numpy.float64)
        lt = st[1024:1024 + 4 * nb].reshape(nb, 4) / 100.0
        ok = lt[:, 0] > 0
        lt = lt[ok]
        e0 = lt[:, 0].min()
        print(json.dumps({"K": K, "workgroups": int(ok.sum()),
                          "kernel_event_us": round(kt["step_ms"] * 1e3, 2),
                          "entry_after_first_us": q(lt[:, 0] - e0),
                          "prologue_us": q(lt[:, 1] - lt[:, 0]),
                          "loop_us": q(lt[:, 2] - lt[:, 1]),
                          "loop_end_after_first_us": q(lt[:, 2] - e0),
                          "closing_us": q(lt[:, 3] - lt[:, 2]),
                          "exit_after_first_us": q(lt[:, 3] - e0),
                          "config": cfg["mode"]}))
    eng.close()


if __name__ == "__main__":
    main()
