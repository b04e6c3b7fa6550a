# round-6: prefill-landed pinned word instead of the event query (resident calls)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_api.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2 3; do
  NMC_TRACE_CALLS=1 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/t_$i.txt 2>&1 || exit 1
  grep "resident call\|nmc_run\|nmc_synchronize" $O/t_$i.txt | tail -5
  grep '^{' $O/t_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))'
done
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/b_$i.txt 2>&1 || exit 1
  grep '^{' $O/b_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("plain %.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))'
done
