#!/bin/bash
# Round-4: fixed LDS step constants + static first entries; parity subset, A/B, stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread"
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu > gpurun_out/t1.log 2>&1
echo "t1 rc=$?"
tail -3 gpurun_out/t1.log
ab() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 $B > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name rc=$?"
}
ab j_ct1 NMC_CTL_TILES=1 &&
ab j_ct2 NMC_CTL_TILES=2 &&
ab j_run NMC_SWEEP=0 &&
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_j.json 2>&1 &&
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_j.jsonl 2> gpurun_out/cfg_j.err
echo "done rc=$?"
