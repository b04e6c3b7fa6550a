# round-6 diagnostics: where the resident launch's next call waits (call trace, kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
B="bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
NMC_TRACE_CALLS=1 timeout -k 10 120 python -u $B > $O/trace_res.txt 2>&1
echo "trace rc $?"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/kt -o kt -- python3 $PWD/bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/kt.txt 2>&1
echo "kt rc $?"
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r06o/kernel_trace.csv")))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in rows:
    if "nmc_k" in r["Kernel_Name"]:
        print("%6s q%s %10.1f %10.1f %8.1f %s vgpr=%s" % (r["Dispatch_Id"], r["Queue_Id"], (int(r["Start_Timestamp"]) - t0) / 1e3,
              (int(r["End_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
              r["Kernel_Name"][:60], r["VGPR_Count"]))
PY
