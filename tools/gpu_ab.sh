#!/bin/bash
# A/B of step-kernel geometries on one MI355X: the GPU tests (optional -k filter), then
# the bench line without the CPU leg and PMC passes once per environment setting.
#   usage: tools/gpu_ab.sh TAG "pytest -k expr or empty" "ENV=V ENV2=V" "ENV=V" ...
set -o pipefail
TAG=${1:-ab}; K=${2:-}; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$K" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/tests_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --cpu-seconds 0 --no-pmc > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || exit $?
  python3 -c "import json,sys;d=json.load(open('gpurun_out/bench_${TAG}_$i.json'));print(sys.argv[1], 'value %.4g  us/iter %.3f  kernel us/launch %.0f' % (d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us']), d['config']['launch'])" "$e"
done
