#!/bin/bash
# Quick GPU iteration: GPU tests (optionally a -k filter), the bench line without the
# CPU leg and PMC passes, and the phase stamps of the diagnostic build.
#   usage: tools/gpu_quick.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-q}
K=${2:-}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider -k "$K" > gpurun_out/tests_$TAG.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
fi
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-pmc > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value %.4g  us/iter %.3f  kernel us/launch %.0f' % (d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us']))"
if [ -f mcmc-for-nested-data_amd/nestmc/libnestmc_stamps.so ]; then
  timeout -k 10 120 python tools/stamps.py partial > gpurun_out/stamps_$TAG.json 2>&1 || exit $?
  cat gpurun_out/stamps_$TAG.json
fi
