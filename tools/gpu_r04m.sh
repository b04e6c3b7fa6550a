#!/bin/bash
# Round-4: sweep vs run on every bench workload (value includes the fill kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ab() {   # name, workload, steps, env...
  local name=$1 wl=$2 k=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --workload $wl --steps $k --warmup 20 --no-pmc --cpu-seconds 0 > gpurun_out/m_$name.json 2> gpurun_out/m_$name.err
  echo "$name rc=$?"
}
ab cfg3_sw cfg3 400 NMC_SWEEP=1 && ab cfg3_run cfg3 400 NMC_SWEEP=0 &&
ab cfg2_sw cfg2 400 NMC_SWEEP=1 && ab cfg2_run cfg2 400 NMC_SWEEP=0 &&
ab cfg4_sw cfg4 200 NMC_SWEEP=1 && ab cfg4_run cfg4 200 NMC_SWEEP=0 &&
ab cfg5 cfg5 100 &&
ab cfg3_sw20 cfg3 20 NMC_SWEEP=1 && ab cfg3_run20 cfg3 20 NMC_SWEEP=0
echo "done rc=$?"
