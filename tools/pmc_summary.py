#!/usr/bin/env python
"""Summarise rocprofv3 --pmc counter_collection.csv files (diagnostics): per counter,
the step kernel's (nmc_k_run / nmc_k_step) values of its last dispatch and its sum over
all dispatches, plus the derived ratios the roofline discussion uses.

    python tools/pmc_summary.py gpurun_out/pmc_TAG_cfg3_p0 [more dirs...] > summary.json
"""

import csv
import glob
import json
import os
import sys


def load(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "")
                if "nmc_k_run" not in k and "nmc_k_step" not in k:
                    continue
                did = int(r.get("Dispatch_Id", 0))
                out.setdefault(r["Counter_Name"], {})[did] = (float(r["Counter_Value"]), k)
    return out


def main():
    res = {}
    for d in sys.argv[1:]:
        for name, per in load(d).items():
            ids = sorted(per)
            res[name] = {"last_dispatch": per[ids[-1]][0], "sum": sum(v for v, _ in per.values()),
                         "dispatches": len(ids), "kernel": per[ids[-1]][1][:80], "dir": d}
    last = {k: v["last_dispatch"] for k, v in res.items()}
    der = {}
    if "SQ_ACTIVE_INST_VALU" in last and "SQ_BUSY_CYCLES" in last:
        der["valu_active_per_busy_cycle"] = last["SQ_ACTIVE_INST_VALU"] / max(1.0, last["SQ_BUSY_CYCLES"])
    if "SQ_INSTS_VALU" in last and "SQ_WAVES" in last:
        der["valu_insts_per_wave"] = last["SQ_INSTS_VALU"] / max(1.0, last["SQ_WAVES"])
    if "SQ_WAIT_INST_ANY" in last and "SQ_WAVE_CYCLES" in last:
        der["wait_inst_any_frac_of_wave_cycles"] = last["SQ_WAIT_INST_ANY"] / max(1.0, last["SQ_WAVE_CYCLES"])
    f64 = [k for k in last if k.startswith("SQ_INSTS_VALU_") and k.endswith("F64")]
    if f64:
        der["f64_valu_insts"] = sum(last[k] for k in f64)
    print(json.dumps({"counters": res, "derived": der}, indent=1))


if __name__ == "__main__":
    main()
