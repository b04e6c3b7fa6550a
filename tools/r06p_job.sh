# round-6: resident-launch tests, the resident call's phases (NMC_TRACE_CALLS), bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
B="python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
NMC_TRACE_CALLS=1 timeout -k 10 120 $B > $O/trace_res.txt 2>&1 || exit 1
grep "resident" $O/trace_res.txt
for i in 1 2; do
  timeout -k 10 120 $B > $O/res_$i.txt 2>&1 || exit 1
  timeout -k 10 120 $B --no-resident > $O/nores_$i.txt 2>&1 || exit 1
done
for f in $O/res_*.txt $O/nores_*.txt $O/trace_res.txt; do
  echo "$f $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]), "launch_us %.1f" % d["roofline"]["avg_launch_us"], d["config"]["resident"])')"
done
