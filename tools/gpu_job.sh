#!/bin/bash
# One GPU call (run through gpurun): each task under its own time limit, chained -- the first
# failure ends the call.  Usage:
#
#   gpurun --timeout 900 -- 'bash tools/gpu_job.sh TAG TASK [TASK ...]'
#
# TASKs (outputs under gpurun_out/TAG_*):
#   tests[:EXPR]        pytest -m gpu [-k EXPR]                      TAG_tests.txt
#   tfile:FILE[:EXPR]   pytest FILE -m gpu [-k EXPR]                 TAG_tests.txt (appended)
#   smoke               __graft_entry__.smoke()                      TAG_smoke.txt
#   bench:ARGS          python bench.py ARGS (ARGS: commas for spaces) TAG_bench.jsonl (appended)
#   kstats:ARGS         rocprofv3 --kernel-trace --stats of bench.py ARGS   TAG_kstats/
#   pmc:CTR[+CTR]:ARGS  rocprofv3 --pmc CTR ... of bench.py ARGS     TAG_pmc_<n>/
#   py:SCRIPT[:ARGS]    python SCRIPT ARGS                           TAG_py.txt (appended)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=$1
shift
n=0
for task in "$@"; do
  n=$((n + 1))
  kind=${task%%:*}
  rest=${task#*:}
  [ "$rest" = "$task" ] && rest=""
  echo "== [$TAG] task $n: $task ($(date +%T))"
  case $kind in
    tests)
      sel=()
      [ -n "$rest" ] && sel=(-k "$rest")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread "${sel[@]}" >> "$OUT/${TAG}_tests.txt" 2>&1 || {
        tail -30 "$OUT/${TAG}_tests.txt"; exit 1; }
      tail -3 "$OUT/${TAG}_tests.txt" ;;
    tfile)
      f=${rest%%:*}
      e=${rest#*:}
      sel=()
      [ "$e" != "$rest" ] && [ -n "$e" ] && sel=(-k "$e")
      timeout -k 10 900 python -u -m pytest "$f" -m gpu -x -v --timeout 300 \
        --timeout-method thread "${sel[@]}" >> "$OUT/${TAG}_tests.txt" 2>&1 || {
        tail -30 "$OUT/${TAG}_tests.txt"; exit 1; }
      tail -3 "$OUT/${TAG}_tests.txt" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$OUT/${TAG}_smoke.txt" 2>&1 || { tail -20 "$OUT/${TAG}_smoke.txt"; exit 1; }
      tail -2 "$OUT/${TAG}_smoke.txt" ;;
    bench)
      args=${rest//,/ }
      timeout -k 10 600 python -u bench.py $args > "$OUT/${TAG}_bench.tmp" 2> "$OUT/${TAG}_bench.err" || {
        tail -20 "$OUT/${TAG}_bench.err"; exit 1; }
      grep '^{' "$OUT/${TAG}_bench.tmp" >> "$OUT/${TAG}_bench.jsonl"
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); \
r=d.get('roofline') or {}; print('value %.4g ms/step %.4f frac %s launch_us %s kernel %s' % \
(d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), r.get('kernel')))" \
        "$OUT/${TAG}_bench.tmp" ;;
    kstats)
      args=${rest//,/ }
      d="$OUT/${TAG}_kstats"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$d" -o k --output-format csv \
        -- python3 bench.py $args --no-pmc --cpu-seconds 0 > "$OUT/${TAG}_kstats.log" 2>&1 || {
        tail -20 "$OUT/${TAG}_kstats.log"; exit 1; }
      find "$d" -name '*kernel_stats.csv' -exec head -6 {} \; ;;
    pmc)
      ctrs=${rest%%:*}
      args=${rest#*:}
      [ "$args" = "$rest" ] && args=""
      args=${args//,/ }
      d="$OUT/${TAG}_pmc_$n"
      timeout -s KILL 120 rocprofv3 --pmc ${ctrs//+/ } -d "$d" -o p --output-format csv \
        -- python3 bench.py $args --no-pmc --cpu-seconds 0 > "$OUT/${TAG}_pmc_$n.log" 2>&1 || {
        tail -20 "$OUT/${TAG}_pmc_$n.log"; exit 1; } ;;
    py)
      s=${rest%%:*}
      a=${rest#*:}
      [ "$a" = "$rest" ] && a=""
      timeout -k 10 600 python -u "$s" ${a//,/ } >> "$OUT/${TAG}_py.txt" 2>&1 || {
        tail -30 "$OUT/${TAG}_py.txt"; exit 1; }
      tail -5 "$OUT/${TAG}_py.txt" ;;
    *)
      echo "unknown task $task"; exit 2 ;;
  esac
done
echo "== [$TAG] done ($(date +%T))"
