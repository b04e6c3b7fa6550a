#!/bin/bash
# One rocprofv3 PMC pass of the bench's child workload (diagnostics): pmc_pass.sh NAME WORKLOAD "COUNTERS..." [env...]
# -> gpurun_out/pmc_NAME/ (counter_collection CSV)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; wl=$2; ctrs=$3; shift 3
mkdir -p gpurun_out/pmc_$name
env "$@" timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$PWD/gpurun_out/pmc_$name" -o pmc \
  -- python3 "$PWD/bench.py" --pmc-child --workload $wl --steps 100 --warmup 10 > gpurun_out/pmc_$name.log 2>&1
