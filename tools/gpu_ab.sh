#!/bin/bash
# A/B of the shipped library against a variant library at cfg 3 (bench.py 2000 iterations,
# kernel us/iter from its HIP-event pass), alternating A B A B.
#   usage: tools/gpu_ab.sh TAG VARIANT_LIB [ENV...]
set -o pipefail
TAG=${1:-ab}; LIB=$2; shift 2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-pmc --cpu-seconds 0 \
      > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$name.json')); r=d['roofline']; print('$name', '%.4g' % d['value'], 'kernel us/iter %.3f' % (r['avg_launch_us'] / r['iterations_per_launch']), d['config']['launch']['mode'], 'W', d['config']['launch']['waves_per_group'])"
}
for k in 1 2; do
  run base$k || exit $?
  run var$k NESTMC_LIB=$LIB "$@" || exit $?
done
