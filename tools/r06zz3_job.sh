# round-6 final: GPU suite, smoke and the driver's bench commands on the shipped build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
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
for l in open("gpurun_out/r06zz3/bench.jsonl"):
    d = json.loads(l)
    print("%.4g" % d["value"], d["steps"], d["roofline"]["frac"], d["config"].get("resident"))
PY
