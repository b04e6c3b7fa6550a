"""Sum each counter of the step kernel's last dispatch in rocprofv3 counter CSVs:
python tools/pmcsum.py gpurun_out/pmc_NAME [...]  (diagnostics)."""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "nmc_k_run" in kn or "nmc_k_sweep" in kn:
                di = int(r["Dispatch_Id"])
                per[di][r["Counter_Name"]] += float(r["Counter_Value"])
                names[di] = kn
    if not per:
        print(d, "no rows")
        continue
    last = max(per)
    c = per[last]
    print(os.path.basename(d), names[last][:60])
    for k in sorted(c):
        print("   %-24s %.4g" % (k, c[k]))
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                print("   %s / SQ_WAVE_CYCLES = %.3f" % (k, c[k] / wc))
