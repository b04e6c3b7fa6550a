#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r_t.log 2>&1
rc=$?; echo "t rc=$rc"; tail -3 gpurun_out/r_t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg4c64 > gpurun_out/r_cfg.jsonl 2> gpurun_out/r_cfg.err; echo "cfg rc=$?"
timeout -k 10 300 python bench.py --workload cfg4 --steps 100 --warmup 10 --no-pmc --cpu-seconds 0 > gpurun_out/r_cfg4.json 2> gpurun_out/r_cfg4.err; echo "b4 rc=$?"
NMC_CTL_TILES=2 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/r_ct2.jsonl 2>&1; echo "ct2 rc=$?"
NMC_GIBBS_TILES=0 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/r_g0.jsonl 2>&1; echo "g0 rc=$?"
