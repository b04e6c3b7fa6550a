#!/usr/bin/env python
"""CPU calibration (TEST/MEASUREMENT INFRASTRUCTURE, never the product): the speed
ratio between the reference's own sampling loop and the numpy restatement
(oracle/restatement.py) on the cfg-3 workload, measured side by side on THIS
container's host cores.

The reference cannot travel to the GPU box, so bench.py times the restatement
there (``cpu_baseline.kind = "port"``) and converts it to a reference-equivalent
rate with the ratio written here (SURVEY.md 8(d) "CPU baseline").

Both sides run one chain in one process, cfg 3 (partial-pooling regression,
sigma = 1, 64 groups x 1000 obs, P = 2), saveLogLikelihood off, and are timed
over their iteration loops only:
  * reference  ``Sampler._loop`` (posteriorSampling.py:862-896), wrapped at run
    time in this process to read the clock around it (the reference files are
    unmodified; /root/reference is imported read-only, no bytecode written);
  * restatement ``oracle.restatement.run`` with the legacy RandomState stream.

Usage: python oracle/calibrate_cpu.py [iters] > profiles/cpu_calibration_r02.json
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))
sys.dont_write_bytecode = True

import numpy  # noqa: E402

REF = "/root/reference"
G, N = 64, 1000


def _callback(x, y):
    import scipy.stats

    def ll(parameter):          # example/regression.py:53-67 with sigma = 1 known
        yhat = numpy.asarray(parameter[0]) + numpy.asarray(parameter[1]) * x
        return scipy.stats.norm(loc=y, scale=1.0).logpdf(yhat)
    return ll


def time_reference(iters, x, y, out_dir):
    sys.path.insert(0, REF)
    import posteriorSampling as ps
    spent = []
    orig = ps.Sampler._loop

    def timed(self):
        t0 = time.perf_counter()
        orig(self)
        spent.append(time.perf_counter() - t0)
    ps.Sampler._loop = timed
    try:
        ps.samplePosterior(1, iters, iters // 2, ("b0", "b1"), G, N, "partial",
                           _callback(x, y), out_dir, saveLogLikelihood=False,
                           startingPointValueRange={"b0": [-1, 1], "b1": [0, 3]},
                           nProcesses=1, displayProgress=False, loggingLevel="error")
    finally:
        ps.Sampler._loop = orig
    return spent[0]


def time_restatement(iters, x, y):
    from oracle import restatement as rs
    nested = rs.Nested(_callback(x, y), [N] * G)
    st, r = rs.init_chain(nested, ("b0", "b1"), 0, "partial", None,
                          {"b0": [-1, 1], "b1": [0, 3]}, False)
    t0 = time.perf_counter()
    rs.run(nested, st, "partial", None, iters, iters // 2, 1, rs.LegacyRNG(r))
    return time.perf_counter() - t0


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    from nestmc import data
    x, y, _, _ = data.linreg(G, N, seed=7)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        t_ref = time_reference(iters, x, y, d + "/")
    t_rs = time_restatement(iters, x, y)
    rate_ref = G * iters / t_ref
    rate_rs = G * iters / t_rs
    print(json.dumps({
        "workload": "cfg3 partial-pooling regression (sigma=1), 1 chain x %d groups x %d obs, "
                    "P=2, %d iterations, one process" % (G, N, iters),
        "reference_chain_group_iter_per_s": rate_ref,
        "restatement_chain_group_iter_per_s": rate_rs,
        "reference_over_restatement": rate_ref / rate_rs,
        "host": "this container (%d CPUs)" % (os.cpu_count() or 0),
        "note": "bench.py multiplies the restatement rate it measures on the GPU box's host "
                "by reference_over_restatement to state a reference-equivalent CPU rate",
    }, indent=1))


if __name__ == "__main__":
    main()
