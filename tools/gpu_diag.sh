#!/bin/bash
# Diagnostics session: launch timeline of short launches (stamps build), then the PMC
# counter passes of tools/pmc_profiles.sh.  Each GPU step under its own time limit.
#   usage: tools/gpu_diag.sh TAG
set -o pipefail
TAG=${1:-r03}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== launchtl $(date +%T)"
timeout -k 10 120 python3 tools/launchtl.py 1 2 5 20 > gpurun_out/launchtl_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/launchtl_$TAG.jsonl
echo "== phase stamps $(date +%T)"
timeout -k 10 120 python3 tools/stamps.py partial > gpurun_out/stamps_$TAG.json 2>&1 || exit $?
timeout -k 10 120 python3 tools/tilegantt.py > gpurun_out/tilegantt_$TAG.json 2>&1 || exit $?
cut -c1-1500 gpurun_out/stamps_$TAG.json
[ "${PMC:-1}" = 0 ] && exit 0
echo "== pmc $(date +%T)"
bash tools/pmc_profiles.sh $TAG || exit $?
for w in cfg3 cfg3long cfg4 cfg5; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/pmc_${TAG}_${w}_summary.json')); print('$w', {k: v['last_dispatch'] for k, v in d['counters'].items()}, d['derived'])"
done
