# round-6: where the resident call's loop time goes -- the prefill's fill beside it (its
# instance, or none) against the kernel alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06q
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
for v in "" "NMC_RES_FILL_MINB=5" "NMC_RES_FILL_MINB=8" "NMC_RES_PREFILL=0" ""; do
  tag=${v:-default}
  env NMC_TRACE_CALLS=1 $v timeout -k 10 120 $B > $O/t_$tag.txt 2>&1 || exit 1
  echo "$tag $(grep 'resident call\|resident instance' $O/t_$tag.txt | tr '\n' ' ') $(grep '^{' $O/t_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))')"
done
timeout -k 10 120 $B --no-resident > $O/nores.txt 2>&1 || exit 1
echo "nores $(grep '^{' $O/nores.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f launch %.1f" % (d["wall_ms"], d["event_ms"], d["roofline"]["avg_launch_us"]))')"
