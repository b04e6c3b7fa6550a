#!/usr/bin/env python
"""Phase timing of the step kernel from the diagnostic stamps build (diagnostics).

    make -C mcmc-for-nested-data_amd/csrc stamps
    python tools/stamps.py [none|partial] [N] [waves] [chains] [groups]

Shader-clock stamps, workgroups 0 and last, waves 0 and W-1, 8 iterations of one
launch.  Slots: 0 iteration start, 1/4 step-0/1 likelihood done, 2/5 after the
step barrier (3: end of step 0 incl. the Gibbs update), 6 steps done, 7 published;
9 (partial): Gibbs update done.
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


def main():
    pooling = sys.argv[1] if len(sys.argv) > 1 else "partial"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    waves = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    C = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    G = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    eng, fam = engine_for("linreg", C, G, N, pooling, waves)
    eng.set_schedule(400, 400, 1)
    eng.run(0, 100)
    eng.synchronize()
    eng.lib.nmc_debug_stamps(eng.h, 1, None)
    eng.run(100, 120)
    out = (ctypes.c_uint64 * (1024 + 4 * 4096 + 512))()   # NMC_STAMP_WORDS
    eng.lib.nmc_debug_stamps(eng.h, 0, out)
    st = numpy.frombuffer(out, dtype=numpy.uint64)[:512].reshape(2, 2, 8, 16).astype(numpy.float64)
    res = {}
    for b in range(2):
        for wv in range(2):
            s = st[b, wv, 1:7, :8]                  # iterations 1..6 of the launch
            d = numpy.diff(s, axis=1)               # slot k -> k+1
            hy = st[b, wv, 1:7, 9:13] - st[b, wv, 1:7, 2:3]   # barrier -> Gibbs done, sum, finish, decided
            ax = st[b, wv, 1:7][:, [13, 14, 15, 12]] - st[b, wv, 1:7, 0:1] if (b, wv) == (0, 1) else None
            it = numpy.diff(st[b, wv, :, 0])[1:7]
            res["blk%d_w%d" % (b, wv)] = {
                "iter_cycles": float(numpy.median(it)),
                "phase_cycles": [float(x) for x in numpy.median(d, axis=0)],
                "hyper_wait_done": [float(x) for x in numpy.median(hy, axis=0)]}
            if ax is not None:   # block 0: auxiliary wave 1 at step 0 (poll, load, join, computed)
                res["blk0_w1"]["aux_poll_load_join_done"] = [float(x) for x in numpy.median(ax, axis=0)]
            if (b, wv) == (0, 0):   # block 0: the compute wave at step 0 (start, updated, priors)
                cx = st[0, 0, 1:7][:, [13, 14, 15]] - st[0, 0, 1:7, 0:1]
                res["blk0_w0"]["compute_start_done_priors"] = [float(x) for x in
                                                               numpy.median(cx, axis=0)]
                res["blk0_w0"]["cw_poll_done"] = float(numpy.median(st[0, 0, 1:7, 8] -
                                                                st[0, 0, 1:7, 0]))
    # tile timeline of workgroup 0, steps 2..7 of the launch: [entry, wave, start, cycles],
    # start relative to the step's first take
    tw = numpy.frombuffer(out, dtype=numpy.uint64)[512:1024].reshape(8, 16, 4).astype(numpy.float64)
    tiles = {}
    for si in range(2, 8):
        e = [(k, tw[si, k]) for k in range(16) if tw[si, k, 0] > 0 and tw[si, k, 1] > 0]
        if not e:
            continue
        t0 = min(x[1][0] for x in e)
        tiles["step%d" % si] = [[k, int(x[2]), int(x[0] - t0), int(x[1] - x[0])] for k, x in e]
        # each wave's arrival at barrier A, relative to the same origin
        tiles["arrive%d" % si] = [[w, int(tw[si, w, 3] - t0)] for w in range(12) if tw[si, w, 3] > 0]
        tiles["ctl%d" % si] = [int(tw[si, 12 + k, 3] - t0) for k in range(3)]   # A, decided, B
        tiles["t0_%d" % si] = int(t0)
        rs = numpy.frombuffer(out, dtype=numpy.uint64)[17408:17920].reshape(8, 16, 4).astype(numpy.float64)
        tiles["restart%d" % si] = [[w] + [int(rs[si, w, k] - t0) for k in range(4)]
                                   for w in range(12) if rs[si, w, 0] > 0]
    # the separate Gibbs kernel (chain block 0): per iteration it of the launch and q,
    # [start of wait, published seen, update done, ready counted], absolute shader clocks
    # rebased on the main kernel's step-0 origin of that iteration
    gib = {}
    for it in range(8):
        for q in range(4):
            row = rs[it, 12 + q]
            if row[0] > 0 and "t0_%d" % (2 * it) in tiles:
                base = tiles["t0_%d" % (2 * it)]
                gib["it%d_q%d" % (it, q)] = [int(row[3] - base), int(row[0] - base),
                                             int(row[1] - base), int(row[2] - base)]
                if q < 2 and rs[it, 14 + q, 0] > 0:   # pass 1, mean, pass 2 (stamps build)
                    gib["it%d_q%d_phases" % (it, q)] = [int(rs[it, 14 + q, k] - row[0])
                                                        for k in range(3)]
    tiles["gibbs"] = gib
    print(json.dumps(dict(pooling=pooling, N=N, config=eng.launch_config(), stamps=res,
                          tiles=tiles)))
    eng.close()


if __name__ == "__main__":
    main()
