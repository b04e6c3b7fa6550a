#!/bin/bash
# One rocprofv3 PMC pass of the bench's child workload (diagnostics):
#   pmc_pass.sh NAME WORKLOAD "COUNTERS..." [CHAINS] [env...]   -> gpurun_out/pmc_NAME/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; wl=$2; ctrs=$3; chains=${4:-0}; shift 4 2>/dev/null || shift $#
extra=""
[ "$chains" != "0" ] && extra="--chains $chains"
mkdir -p gpurun_out/pmc_$name
env "$@" timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$PWD/gpurun_out/pmc_$name" -o pmc \
  -- python3 "$PWD/bench.py" --pmc-child --workload $wl --steps 100 --warmup 10 $extra > gpurun_out/pmc_$name.log 2>&1
