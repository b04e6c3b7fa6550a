# round-6 final build: GPU suite, smoke, default bench, the driver's command x3, rocprof
# kernel trace / stats of the driver's command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06zzf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench_default.txt 2>&1 || { tail -20 $O/bench_default.txt; exit 1; }
grep '^{' $O/bench_default.txt > $O/bench.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b_$i.txt 2>&1 || { tail -20 $O/b_$i.txt; exit 1; }
  grep '^{' $O/b_$i.txt >> $O/bench.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/r06zzf/bench.jsonl"):
    d = json.loads(l)
    print("%.4g" % d["value"], d["steps"], "frac %.3f" % d["roofline"]["frac"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]), d["config"].get("resident"))
PY
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/kt -o kt -- python3 $PWD/bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/kt.txt 2>&1 || { tail -20 $O/kt.txt; exit 1; }
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace_driver.csv \;
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_driver.csv \;
cut -c1-200 $O/kernel_stats_driver.csv | head -8
