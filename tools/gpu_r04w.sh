#!/bin/bash
# Round-4: counters and kernel trace of the cfg-4 shard (128 chains) on the final build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
./tools/pmc_pass.sh cfg4_sq64 cfg4 "$SQ" 64 && echo sq ok &&
./tools/pmc_pass.sh cfg4_sq_run cfg4 "$SQ" 128 NMC_SWEEP=0 && echo sqrun ok &&
./tools/pmc_pass.sh cfg3_sq cfg3 "$SQ" 0 && echo sq3 ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r04w_stats_cfg4" -o run -- python3 bench.py --workload cfg4 --chains 128 --steps 200 --warmup 20 --no-pmc --cpu-seconds 0 > gpurun_out/r04w_stats_cfg4.json 2> gpurun_out/r04w_stats_cfg4.err
echo "done rc=$?"
