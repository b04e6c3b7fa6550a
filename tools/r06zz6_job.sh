# round-6: record-row fast path (thin 1): resident call loop, recorded vs burn-in; bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in 0 1 0 1; do
  timeout -k 10 120 python -u tools/calltrace.py 20 8 1 $m > $O/res_norec$m.txt 2>&1 || { tail -20 $O/res_norec$m.txt; exit 1; }
  echo "norec=$m"; grep "relay" $O/res_norec$m.txt | tail -4 | sed 's/.*relay/relay/'
done
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/b_$i.txt 2>&1 || { tail -20 $O/b_$i.txt; exit 1; }
  grep '^{' $O/b_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))'
done
