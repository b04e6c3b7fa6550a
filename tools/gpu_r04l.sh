#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu > gpurun_out/t1.log 2>&1
echo "t1 rc=$?"; tail -2 gpurun_out/t1.log
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg2 > gpurun_out/cfg_l.jsonl 2> gpurun_out/cfg_l.err &&
NMC_GIBBS_TILES=0 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/cfg_l_g0.jsonl 2> gpurun_out/cfg_l_g0.err &&
timeout -k 10 120 python tools/stamps.py partial 2000 0 128 256 > gpurun_out/stamps_cfg4_l.json 2>&1 &&
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0 > gpurun_out/ab_l.json 2> gpurun_out/ab_l.err
echo "done rc=$?"
