# round-6: the sample recording's share of a resident call's loop (burn-in calls vs recorded)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz5
mkdir -p $O
for m in 0 1 0 1; do
  timeout -k 10 120 python -u tools/calltrace.py 20 8 1 $m > $O/res_norec$m.txt 2>&1 || { tail -20 $O/res_norec$m.txt; exit 1; }
  echo "norec=$m"; grep "relay" $O/res_norec$m.txt | tail -4 | sed 's/.*relay/relay/'
done
