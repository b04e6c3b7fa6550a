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
        "SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU")
run_pass() {   # name, pass index, command...
  local name=$1 k=$2; shift 2
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${PASSES[$k]} --output-format csv \
      -d "$ROOT/gpurun_out/pmc_${TAG}_${name}_p$k" -o pmc -- "$@" \
      > "$ROOT/gpurun_out/pmc_${TAG}_${name}_p$k.log" 2>&1)
}
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/pmc_${TAG}_counters.txt" 2>&1) || true
# pass 2: only the counters this device lists
P2=""
for c in ${PASSES[2]}; do
  grep -qw "$c" "$ROOT/gpurun_out/pmc_${TAG}_counters.txt" && P2="$P2 $c"
done
PASSES[2]="${P2:-SQ_INSTS_SALU}"
echo "pass 2 counters: ${PASSES[2]}"
for k in 0 1 2; do
  echo "== cfg3 (the driver's bench command) pass $k $(date +%T)"
  run_pass cfg3 $k python3 "$ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 --no-pmc || exit $?
  echo "== cfg3 2000 iterations pass $k $(date +%T)"
  run_pass cfg3long $k python3 "$ROOT/bench.py" --steps 2000 --warmup 200 --cpu-seconds 0 --no-pmc || exit $?
  echo "== cfg4 pass $k $(date +%T)"
  run_pass cfg4 $k python3 "$ROOT/tools/cfgbench.py" cfg4 || exit $?
  echo "== cfg5 pass $k $(date +%T)"
  run_pass cfg5 $k python3 "$ROOT/tools/cfgbench.py" cfg5 || exit $?
done
for w in cfg3 cfg3long cfg4 cfg5; do
  python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_${w}_p0 gpurun_out/pmc_${TAG}_${w}_p1 \
      gpurun_out/pmc_${TAG}_${w}_p2 > gpurun_out/pmc_${TAG}_${w}_summary.json || exit $?
done
echo "== done $(date +%T)"
