#!/bin/bash
# Round-4 A/B session: nmc_k_sweep variants vs nmc_k_run at cfg 3 (400-iteration launches),
# the stamps build's phase timeline, then the GPU test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread"
S32=mcmc-for-nested-data_amd/nestmc/libnestmc_s32.so
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
timeout -k 10 300 $T tests/test_gpu_parity.py -x -q -m gpu -k "paired_rows" > gpurun_out/t1.log 2>&1
echo "t1 rc=$?"
ab() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 150 $B > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name rc=$?"
}
ab run NMC_SWEEP=0 &&
ab sw12 NMC_SWEEP=1 &&
ab sw12zin NMC_ZIN=1 &&
ab sw8 NMC_SWEEP_WAVES=8 &&
ab s32sw12t32 NESTMC_LIB=$S32 NMC_TILE_ROWS=32 &&
ab s32sw12t48 NESTMC_LIB=$S32 NMC_TILE_ROWS=48 &&
ab s32run8t32 NESTMC_LIB=$S32 NMC_TILE_ROWS=32 NMC_SWEEP=0 &&
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_sweep.jsonl 2> gpurun_out/cfg_sweep.err &&
NMC_SWEEP=0 timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_run.jsonl 2> gpurun_out/cfg_run.err &&
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_sw12.json 2>&1 &&
timeout -k 10 600 $T tests -m gpu -q -rf > gpurun_out/t2.log 2>&1
echo "t2 rc=$?"
tail -5 gpurun_out/t2.log
