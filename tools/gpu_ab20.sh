#!/bin/bash
# A/B of the shipped library against a variant at the driver's bench command
# (bench.py --steps 20 --warmup 5), alternating A B three times; prints value and wall.
#   usage: tools/gpu_ab20.sh TAG VARIANT_LIB
set -o pipefail
TAG=${1:-ab20}; LIB=$2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 \
      > gpurun_out/ab20_${TAG}_$name.json 2> gpurun_out/ab20_${TAG}_$name.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab20_${TAG}_$name.json')); print('$name', '%.4g' % d['value'], 'wall us %.1f event us %.1f' % (d['wall_ms'] * 1e3, d['event_ms'] * 1e3))"
}
for k in 1 2 3; do
  run base$k || exit $?
  run var$k NESTMC_LIB=$LIB || exit $?
done
