#!/bin/bash
# A/B of the shipped library against a variant on tools/cfgbench.py workloads.
#   usage: tools/gpu_abcfg.sh TAG VARIANT_LIB CFG...
set -o pipefail
TAG=$1; LIB=$2; shift 2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 200 python3 tools/cfgbench.py "$@" > gpurun_out/abcfg_${TAG}_base$k.jsonl 2>&1 || exit $?
  timeout -k 10 200 env NESTMC_LIB=$LIB python3 tools/cfgbench.py "$@" > gpurun_out/abcfg_${TAG}_var$k.jsonl 2>&1 || exit $?
  for v in base$k var$k; do
    python3 -c "
import json
for l in open('gpurun_out/abcfg_${TAG}_$v.jsonl'):
    d = json.loads(l); print('$v', d['config'], 'us/iter %.2f' % d['us_per_iter'])"
  done
done
