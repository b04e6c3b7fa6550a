#!/bin/bash
# Round-4 A/B: per-SIMD tile queues (NMC_SQ) x control tile policy; tile timelines.
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
ab sq1 NMC_SQ=1 &&
ab sq0 NMC_SQ=0 &&
ab sq1ct0 NMC_CTL_TILES=0 &&
ab sq1ct2 NMC_CTL_TILES=2 &&
ab sq1zin NMC_ZIN=1 &&
ab sq1sw8 NMC_SWEEP_WAVES=8 &&
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_sq1.json 2>&1 &&
NMC_ZIN=1 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_sq1zin.json 2>&1 &&
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_sq1.jsonl 2> gpurun_out/cfg_sq1.err
echo "done rc=$?"
