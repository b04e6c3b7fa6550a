# round-6: host-side timing of the resident call (post -> ack, post -> done seen)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz
mkdir -p $O
for i in 1 2 3; do
  NMC_TRACE_CALLS=1 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/t_$i.txt 2>&1 || exit 1
  grep "resident call\|nmc_run\|nmc_synchronize" $O/t_$i.txt | tail -5
  grep '^{' $O/t_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))'
done
