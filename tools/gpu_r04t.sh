#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k cfg4 --timeout 120 --timeout-method thread > gpurun_out/t_t.log 2>&1
rc=$?; echo "t rc=$rc"; tail -2 gpurun_out/t_t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg4c64 > gpurun_out/t_cfg.jsonl 2> gpurun_out/t_cfg.err; echo "cfg rc=$?"
timeout -k 10 120 python tools/stamps.py partial 2000 0 128 256 > gpurun_out/stamps_cfg4_t.json 2>&1; echo "s rc=$?"
