#!/usr/bin/env python
"""Phase timing of nmc_k_duo from the diagnostic stamps build (diagnostics only).

    make -C mcmc-for-nested-data_amd/csrc duostamps
    python tools/duo_stamps.py [chains] [groups] [obs] [waves]

Workgroup 0 of a 30-iteration launch (after a 10-iteration one): per half, the decision
period and its parts (detected -> waits done -> released -> bookkeeping done), the Gibbs
tasks (loop top -> poll done -> computed) and when each lands relative to the decision
that needs it, and the tiles of each release (first start after the release, span, waves).
Shader-clock cycles.  Prints one JSON object.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
os.environ.setdefault("NESTMC_LIB", os.path.join(ROOT, "mcmc-for-nested-data_amd", "nestmc",
                                                 "libnestmc_ds.so"))
import numpy  # noqa: E402

from nestmc import data  # noqa: E402
from nestmc.engine import Engine  # noqa: E402
from nestmc.families import LinearRegression  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    if len(sys.argv) > 4:
        os.environ["NMC_DUO_WAVES"] = sys.argv[4]
    x, y, _, _ = data.linreg(G, N, seed=7)
    fam = LinearRegression.simple(x, y, sigma=1.0)
    eng = Engine(fam, [N] * G, C, "partial", seed=3)
    r = numpy.random.RandomState(0)
    P = 2
    mu = numpy.zeros((C, P)) + [0.0, 2.0]
    s2 = numpy.full((C, P), 0.5)
    value = mu[:, :, None] + 0.5 * r.normal(size=(C, P, G))
    lp = numpy.zeros((C, P, G))
    ll = numpy.full((C, G), -1e3)
    eng.set_state(value, lp, ll, mu, s2)
    eng.set_schedule(400, 400, 1)
    eng.run(0, 10)
    eng.synchronize()
    eng.lib.nmc_debug_stamps(eng.h, 1, None)
    eng.run(10, 40)
    out = (ctypes.c_uint64 * (1024 + 4 * 4096 + 512))()
    eng.lib.nmc_debug_stamps(eng.h, 0, out)
    cfg = eng.launch_config()
    eng.close()
    st = numpy.frombuffer(out, dtype=numpy.uint64).astype(numpy.float64)
    dec = st[:640].reshape(2, 64, 5)
    gib = st[640:1152].reshape(2, 64, 4)
    til = st[1152:1152 + 128 * 16 * 3].reshape(128, 16, 3)
    t0 = numpy.min(st[:1152][st[:1152] > 0])
    res = {"config": cfg, "halves": {}}
    nst = 60   # steps of the 30-iteration launch (P = 2)
    for h in range(2):
        d = dec[h, :nst]
        ok = d[:, 0] > 0
        dd = d[ok] - t0
        per = numpy.diff(dd[:, 0])
        g = gib[h, :nst]
        # decision s waits for task s - 2: when did it land (computed) relative to detection?
        land = [g[s - 2, 2] - d[s, 0] for s in range(2, nst) if g[s - 2, 2] > 0 and d[s, 0] > 0]
        res["halves"][h] = {
            "decisions": int(ok.sum()),
            "period_median": float(numpy.median(per)) if len(per) else None,
            "detect_to_release": float(numpy.median(dd[:-1, 2] - dd[:-1, 0])),
            "release_to_end": float(numpy.median(dd[:, 3] - dd[:, 2])),
            "gibbs_top_to_poll": float(numpy.median(g[g[:, 1] > 0, 1] - g[g[:, 1] > 0, 0])),
            "gibbs_poll_to_computed": float(numpy.median(g[g[:, 2] > 0, 2] - g[g[:, 2] > 0, 1])),
            "gibbs_computed_minus_detect_median": float(numpy.median(land)) if land else None,
            "publish_to_gibbs_computed": float(numpy.median(
                [g[s, 2] - d[s, 3] for s in range(nst) if g[s, 2] > 0 and d[s, 3] > 0])),
        }
    # tiles: per record, first start relative to the record's release, span, waves
    recs = []
    for rec in range(min(128, 2 * nst)):
        tt = til[rec]
        okt = tt[:, 0] > 0
        if not okt.any():
            continue
        recs.append({"rec": rec, "first": float(tt[okt, 0].min() - t0),
                     "tickets": [[int(k), int(tt[k, 0] - t0), int(tt[k, 1] - tt[k, 0]),
                                  int(tt[k, 2])] for k in range(16) if okt[k]],
                     "span": float(tt[okt, 1].max() - tt[okt, 0].min()),
                     "tile_med": float(numpy.median(tt[okt, 1] - tt[okt, 0])),
                     "waves": sorted(set(int(v) for v in tt[okt, 2]))})
    res["tiles_first12"] = recs[:12]
    res["tile_dur_median"] = float(numpy.median([r["tile_med"] for r in recs]))
    res["record_span_median"] = float(numpy.median([r["span"] for r in recs]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
