# round-6: resident gate with closers + reload: tests, the call's phases, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -2 $O/tests.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
B="python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
for i in 1 2 3; do
  env NMC_TRACE_CALLS=1 timeout -k 10 120 $B > $O/t_res_$i.txt 2>&1 || exit 1
  echo "res $(grep 'resident call\|resident instance' $O/t_res_$i.txt | tr '\n' ' ') $(grep '^{' $O/t_res_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))')"
  timeout -k 10 120 $B --no-resident > $O/nores_$i.txt 2>&1 || exit 1
  echo "nores $(grep '^{' $O/nores_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f launch %.1f" % (d["wall_ms"], d["event_ms"], d["roofline"]["avg_launch_us"]))')"
done
