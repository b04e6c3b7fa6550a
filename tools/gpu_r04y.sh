#!/bin/bash
# Round-4 final build: the whole GPU suite, smoke, the default bench line with PMC and CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/y_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/y_gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/y_smoke.txt 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/y_bench.json 2> gpurun_out/y_bench.err; echo "bench rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/y_bench20.json 2> gpurun_out/y_bench20.err; echo "bench20 rc=$?"
timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/y_cfg4.jsonl 2> gpurun_out/y_cfg4.err; echo "cfg4 rc=$?"
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
timeout -k 10 150 $B > gpurun_out/y_st1.json 2>&1; echo "st1 rc=$?"
NMC_STATIC_TILES=0 timeout -k 10 150 $B > gpurun_out/y_st0.json 2>&1; echo "st0 rc=$?"
timeout -k 10 150 $B > gpurun_out/y_st1b.json 2>&1; echo "st1b rc=$?"
NMC_STATIC_TILES=0 timeout -k 10 150 $B > gpurun_out/y_st0b.json 2>&1; echo "st0b rc=$?"
