#!/bin/bash
# Round-4 final build (no machine LICM in the linreg / Gaussian-means TUs): suite, smoke, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f2_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/f2_gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f2_smoke.txt 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/f2_bench.json 2> gpurun_out/f2_bench.err; echo "bench rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/f2_bench20.json 2> gpurun_out/f2_bench20.err; echo "bench20 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/f2_stats" -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > gpurun_out/f2_stats_bench.json 2> gpurun_out/f2_stats_bench.err; echo "stats rc=$?"
