#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k cfg4 --timeout 120 --timeout-method thread > gpurun_out/q_t.log 2>&1
echo "t rc=$?"; tail -3 gpurun_out/q_t.log
NMC_SWEEP=1 timeout -k 10 200 python tools/cfgbench.py cfg4 cfg4c64 > gpurun_out/q_sw.jsonl 2> gpurun_out/q_sw.err; echo "sw rc=$?"
NMC_SWEEP=1 NMC_GSEP=1 timeout -k 10 200 python tools/cfgbench.py cfg4c64 > gpurun_out/q_sw1.jsonl 2> gpurun_out/q_sw1.err; echo "sw1 rc=$?"
