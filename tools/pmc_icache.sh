#!/bin/bash
# Instruction-cache and wait-state counters of the step kernel (one short bench run per
# PMC pass; each pass holds few counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES\|SQ_INSTS_VALU\b\|SQ_ACTIVE_INST_[A-Z]*\|SQ_INSTS_LDS\|SQ_WAIT_ANY\|SQ_INST_LEVEL_LDS\|SQ_INSTS_SALU" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_pick.txt
cat gpurun_out/counters_pick.txt | tr '\n' ' '; echo
run() {
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_ic" -o "p_$1" -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --cpu-seconds 0 --no-pmc --no-gather > /dev/null 2>&1)
}
run SQC_ICACHE_MISSES SQC_ICACHE_HITS && run SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES && run SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS || echo "pmc pass failed"
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob('gpurun_out/pmc_ic/**/*counter_collection.csv', recursive=True):
    rows = list(csv.DictReader(open(f)))
    runs = [r for r in rows if 'nmc_k_run' in r.get('Kernel_Name', '')]
    if not runs: continue
    last = max(int(r['Dispatch_Id']) for r in runs)
    for r in runs:
        if int(r['Dispatch_Id']) == last:
            tot[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(tot.items()): print(k, v)
PY
