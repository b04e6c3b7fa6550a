#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k "cfg4" --timeout 200 --timeout-method thread > gpurun_out/h2_t.log 2>&1
echo "t rc=$?"; tail -8 gpurun_out/h2_t.log
