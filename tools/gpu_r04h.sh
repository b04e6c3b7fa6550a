#!/bin/bash
# Round-4: LDS step constants; restart stamps; A/B vs nmc_k_run.
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
ab h_sq0ct2 NMC_SQ=0 NMC_CTL_TILES=2 &&
ab h_sq0 NMC_SQ=0 &&
ab h_sq1 NMC_SQ=1 &&
NMC_SQ=0 NMC_CTL_TILES=2 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_h_orig.json 2>&1
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_h_sq1.json 2>&1
echo "done rc=$?"
