# round-6 final build: the other workloads' bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zzw
mkdir -p $O
for w in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --workload $w --no-pmc --cpu-seconds 0 > $O/b_$w.txt 2>&1 || { tail -20 $O/b_$w.txt; exit 1; }
  grep '^{' $O/b_$w.txt >> $O/bench.jsonl
  grep '^{' $O/b_$w.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$w' %.4g" % d["value"], d["steps"], "frac %.3f" % d["roofline"]["frac"])'
done
