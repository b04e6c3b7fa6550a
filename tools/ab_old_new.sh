#!/bin/bash
# A/B of the contract bench: the current library under env settings ($@) against a
# reference build unpacked under ab_old/ (not tracked), alternating, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for e in "$@" old; do
    i=$((i+1))
    if [ "$e" = old ]; then
      timeout -k 10 200 python ab_old/bench.py --cpu-seconds 0 --no-pmc > gpurun_out/ab_$i.json 2>/dev/null || exit 1
    else
      env $e timeout -k 10 200 python bench.py --cpu-seconds 0 --no-pmc > gpurun_out/ab_$i.json 2>/dev/null || exit 1
    fi
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$i.json'));print(sys.argv[1], '%.4g'%d['value'], '%.3f us/iter'%(d['ms_per_step']*1e3), 'kernel %.0f us/launch'%d['roofline']['avg_launch_us'])" "$e"
  done
done
