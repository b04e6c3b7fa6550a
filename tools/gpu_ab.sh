#!/bin/bash
# A/B of step-kernel builds on one box: each variant runs the driver's bench command and the
# default-length bench (no PMC, no CPU leg).  usage: tools/gpu_ab.sh TAG "NAME:ENV ..."
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  echo "== $name ($envs) $(date +%T)"
  env $envs timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 \
      > gpurun_out/ab_${TAG}_${name}_20.json 2> gpurun_out/ab_${TAG}_${name}_20.err || exit $?
  env $envs timeout -k 10 200 python3 bench.py --no-pmc --cpu-seconds 0 \
      > gpurun_out/ab_${TAG}_${name}.json 2> gpurun_out/ab_${TAG}_${name}.err || exit $?
  python3 -c "
import json,sys
a=json.load(open('gpurun_out/ab_${TAG}_${name}_20.json')); b=json.load(open('gpurun_out/ab_${TAG}_${name}.json'))
print('$name', 'bench20 %.4g' % a['value'], 'bench2000 %.4g' % b['value'], 'kernel_us/iter %.3f' % (b['roofline']['avg_launch_us']/b['roofline']['iterations_per_launch']), b['config']['launch']['waves_per_group'], b['roofline']['kernel'])"
done
