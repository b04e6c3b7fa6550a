#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
NMC_SWEEP=1 timeout -k 10 200 python tools/cfgbench.py cfg4c64 cfg4 > gpurun_out/o_sw.jsonl 2> gpurun_out/o_sw.err &&
NMC_SWEEP=0 timeout -k 10 200 python tools/cfgbench.py cfg4c64 cfg4 > gpurun_out/o_run.jsonl 2> gpurun_out/o_run.err
echo "done rc=$?"
