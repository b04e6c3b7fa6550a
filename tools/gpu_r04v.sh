#!/bin/bash
# Round-4 final: the whole GPU suite, smoke, cfg-4 numbers of the final build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/v_gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/v_smoke.txt 2>&1; echo "smoke rc=$?"
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg4c64 > gpurun_out/v_cfg.jsonl 2> gpurun_out/v_cfg.err; echo "cfg rc=$?"
timeout -k 10 400 python bench.py --workload cfg4 --steps 100 --warmup 10 > gpurun_out/v_cfg4.json 2> gpurun_out/v_cfg4.err; echo "b4 rc=$?"
