#!/bin/bash
# Round-4 A/B: split in-kernel variates (NMC_ZIN=1) vs the fill's ring vs nmc_k_run; stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread"
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
timeout -k 10 400 $T tests/test_gpu_parity.py -x -q -m gpu -k "paired_rows" > gpurun_out/t1.log 2>&1
echo "t1 rc=$?"
tail -3 gpurun_out/t1.log
ab() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 $B > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name rc=$?"
}
ab run NMC_SWEEP=0 &&
ab sw12 NMC_SWEEP=1 &&
ab sw12zin NMC_ZIN=1 &&
ab sw8zin NMC_ZIN=1 NMC_SWEEP_WAVES=8 &&
ab sw8 NMC_SWEEP_WAVES=8 &&
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_sw12.json 2>&1 &&
NMC_ZIN=1 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_sw12zin.json 2>&1 &&
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_sweep.jsonl 2> gpurun_out/cfg_sweep.err
echo "done rc=$?"
NMC_SWEEP_WAVES=4 timeout -k 10 120 python tools/stamps.py partial 2000 0 128 256 > gpurun_out/stamps_cfg4.json 2>&1; echo "cfg4 stamps rc=$?"
