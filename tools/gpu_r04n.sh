#!/bin/bash
# Round-4 close-out 1/2: the whole GPU suite and the kernel-trace summary of the driver's bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_gpu_tests.txt 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r04_gpu_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r04_stats" -o run -- python3 bench.py --no-pmc --cpu-seconds 0 > gpurun_out/r04_stats_bench.json 2> gpurun_out/r04_stats_bench.err
echo "stats rc=$?"
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
timeout -k 10 150 $B > gpurun_out/n_def.json 2> gpurun_out/n_def.err && echo def ok &&
NESTMC_LIB=$PWD/mcmc-for-nested-data_amd/nestmc/libnestmc_nl.so timeout -k 10 150 $B > gpurun_out/n_nl.json 2> gpurun_out/n_nl.err && echo nl ok
