#!/bin/bash
# rocprofv3 PMC counter passes (one counter group per run, each under its own time limit)
# for the step kernel of: the contract bench command (cfg 3), the cfg-4 shard and the
# cfg-5 shard (tools/cfgbench.py).  Summaries -> gpurun_out/pmc_TAG_<workload>_<pass>/.
#   usage: tools/pmc_profiles.sh TAG
set -o pipefail
TAG=${1:-r03}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=("SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES"
        "SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
run_pass() {   # name, pass index, command...
  local name=$1 k=$2; shift 2
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${PASSES[$k]} --output-format csv \
      -d "$ROOT/gpurun_out/pmc_${TAG}_${name}_p$k" -o pmc -- "$@" \
      > "$ROOT/gpurun_out/pmc_${TAG}_${name}_p$k.log" 2>&1)
}
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/pmc_${TAG}_counters.txt" 2>&1) || true
for k in 0 1; do
  echo "== cfg3 pass $k $(date +%T)"
  run_pass cfg3 $k python3 "$ROOT/bench.py" --steps 2000 --warmup 200 --cpu-seconds 0 --no-pmc || exit $?
  echo "== cfg4 pass $k $(date +%T)"
  run_pass cfg4 $k python3 "$ROOT/tools/cfgbench.py" cfg4 || exit $?
  echo "== cfg5 pass $k $(date +%T)"
  run_pass cfg5 $k python3 "$ROOT/tools/cfgbench.py" cfg5 || exit $?
done
echo "== done $(date +%T)"
