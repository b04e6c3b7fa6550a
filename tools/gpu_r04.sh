#!/bin/bash
# Round-4 GPU session: parity tests of the sweep kernel first (a short subset, then the whole
# GPU suite), then the cfg-3 bench A/B (nmc_k_sweep vs nmc_k_run) and a kernel-trace profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_softplus.py -x -v -m gpu \
    -k "paired_rows or softplus" > gpurun_out/t1.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu -q -rf > gpurun_out/t2.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 \
      > gpurun_out/b_sweep20.json 2> gpurun_out/b_sweep20.err &&
  NMC_SWEEP=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 \
      > gpurun_out/b_run20.json 2> gpurun_out/b_run20.err &&
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-pmc --cpu-seconds 0 \
      > gpurun_out/b_sweep2000.json 2> gpurun_out/b_sweep2000.err &&
  NMC_SWEEP=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-pmc --cpu-seconds 0 \
      > gpurun_out/b_run2000.json 2> gpurun_out/b_run2000.err &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o p -- \
      python3 bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > gpurun_out/prof.log 2>&1
  echo "bench rc=$?"
fi
tail -3 gpurun_out/t2.log
