#!/bin/bash
# One GPU session: the GPU test suite, the driver's bench command, the default-length
# bench, the rocprofv3 kernel-trace summary of the driver's command, an fp64 peak probe.
# Every GPU step has its own time limit and the steps are chained with &&: a failure or
# fault ends the session.
#   usage: tools/gpu_round.sh TAG [pytest-args...]     (TESTS=0 skips the tests)
set -o pipefail
TAG=${1:-r03}
shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" != 0 ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      --maxfail=5 -p no:cacheprovider "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?
  tail -5 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
echo "== bench20 $(date +%T)"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.json \
    2> gpurun_out/bench20_$TAG.err && cut -c1-300 gpurun_out/bench20_$TAG.json && \
echo "== bench $(date +%T)" && \
timeout -k 10 300 python3 bench.py --no-pmc --cpu-seconds 0 > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err && cut -c1-300 gpurun_out/bench_$TAG.json && \
echo "== rocprof $(date +%T)" && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$ROOT/gpurun_out/prof_$TAG" -o $TAG -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 --no-pmc \
    > "$ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$ROOT/gpurun_out/bench_prof_$TAG.err") && \
find gpurun_out/prof_$TAG -name "*stats*" && \
echo "== launchcost $(date +%T)" && \
timeout -k 10 200 python3 tools/launchcost.py > gpurun_out/launchcost_$TAG.json 2>&1 && \
cut -c1-600 gpurun_out/launchcost_$TAG.json && \
echo "== cfgbench $(date +%T)" && \
timeout -k 10 300 python3 tools/cfgbench.py cfg2 cfg4 cfg5 > gpurun_out/cfgbench_$TAG.jsonl 2>&1 && \
cut -c1-400 gpurun_out/cfgbench_$TAG.jsonl && \
echo "== done $(date +%T)"
