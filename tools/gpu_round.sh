#!/bin/bash
# One GPU session: the GPU test suite, the contract bench line, and the rocprofv3
# kernel-trace summary of the same bench command.  Every GPU step has its own time
# limit and the steps are chained with &&: a failure or fault ends the session.
#   usage: tools/gpu_round.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-r02}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    --maxfail=5 -p no:cacheprovider "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cat gpurun_out/bench_$TAG.json && \
echo "== rocprof $(date +%T)" && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o $TAG -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --no-pmc \
    > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err") && \
find gpurun_out/prof_$TAG -name "*stats*" && echo "== done $(date +%T)"
