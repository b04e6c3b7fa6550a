#!/usr/bin/env python
"""Per-rank shard timings of the multi-GPU configs (diagnostics, not the contract
bench): cfg 2 (256 chains x 32 groups x 500 obs, Gaussian means, no pooling, one GPU),
cfg 4 (1024 chains x 256 groups x 2000 obs over 8 GPUs -> 128 chains per rank,
partial-pooling regression) and cfg 5 (512 x 128 x 5000 over 8 -> 64 chains per rank,
8-parameter logistic, built-in family and the same model as a runtime-compiled user
family)."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd"))

from kbench import run  # noqa: E402

LOGISTIC8 = r"""
__device__ double nmc_user_loglik(const double* th, const double* row, const double* k) {
  double eta = th[0];
  for (int j = 0; j < 7; ++j) eta = fma(row[j], th[j + 1], eta);
  return row[7] * eta - nmc_logaddexp0(eta);
}
"""


def main():
    which = sys.argv[1:] or ["cfg2", "cfg4", "cfg5", "cfg5user"]
    for w in which:
        if w == "cfg2":     # example.distribution, none pooling, 256 x 32 x 500, one GPU
            r = run("gauss", 256, 32, 500, "none", 0, 200)
        elif w == "cfg4":
            r = run("linreg", 128, 256, 2000, "partial", 0, 40)
        elif w == "cfg4c64":   # one chain block of the cfg-4 geometry (half a shard)
            r = run("linreg", 64, 256, 2000, "partial", 0, 40)
        elif w == "cfg4w4":   # four waves per workgroup: two workgroups per CU, resident
            r = run("linreg", 128, 256, 2000, "partial", 4, 40)
        elif w == "cfg5":
            r = run("logistic", 64, 128, 5000, "partial", 0, 10)
        else:
            os.environ["KB_USER_SOURCE"] = LOGISTIC8
            r = run("logistic", 64, 128, 5000, "partial", 0, 10)
            os.environ.pop("KB_USER_SOURCE")
        r["config"] = w
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
