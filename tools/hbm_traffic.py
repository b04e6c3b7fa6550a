#!/usr/bin/env python
"""HBM traffic per launch of the iteration kernel from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python tools/hbm_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ITERS > profiles/...json

ITERS: iterations the profiled run's step launches covered (bench.py --steps K
--warmup W runs W + 2K), so the bytes can be normalised per iteration.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (MI355X_MICROARCH.md
"rocprofv3 PMC slots": they do not fit one TCC pass) and are reported by rocprofv3
in KiB per dispatch.  gfx950 correction (same guide, section HBM): FETCH_SIZE
tallies 128-B fabric requests at 64 B, so it is doubled; WRITE_SIZE is taken as is.
Both count Infinity-Cache hits, so they are an upper bound on DRAM bytes.
"""

import csv
import glob
import json
import os
import sys

KERNEL = os.environ.get("NMC_TRAFFIC_KERNEL", "nmc_k_run")


def per_dispatch(root, counter):
    vals = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                if KERNEL not in row.get("Kernel_Name", ""):
                    continue
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit("no %s rows for %s under %s" % (counter, KERNEL, root))
    return sum(vals) / len(vals), len(vals), sum(vals)


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3])
    f_kib, nf, f_tot = per_dispatch(fetch_dir, "FETCH_SIZE")
    w_kib, nw, w_tot = per_dispatch(write_dir, "WRITE_SIZE")
    read_b = 2.0 * f_kib * 1024.0
    write_b = w_kib * 1024.0
    out = {
        "kernel": KERNEL,
        "dispatches": {"fetch": nf, "write": nw},
        "fetch_size_kib_raw": f_kib,
        "write_size_kib_raw": w_kib,
        "read_bytes_per_launch": read_b,
        "write_bytes_per_launch": write_b,
        "bytes_per_step_launch": read_b + write_b,
        "iterations": iters,
        "bytes_per_iteration": (2.0 * f_tot + w_tot) * 1024.0 / iters,
        "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); WRITE_SIZE as is",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
