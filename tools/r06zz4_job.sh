# round-6: resident call loop time against the call length (intercept = per-call loop excess)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zz4
mkdir -p $O
for k in 5 10 20 40 100; do
  timeout -k 10 120 python -u tools/calltrace.py $k 8 1 > $O/res_k$k.txt 2>&1 || { tail -20 $O/res_k$k.txt; exit 1; }
  echo "K=$k"; grep "relay" $O/res_k$k.txt | tail -5 | sed 's/.*relay/relay/'
done
timeout -k 10 120 python -u tools/calltrace.py 20 6 0 > $O/launch_k20.txt 2>&1 || { tail -20 $O/launch_k20.txt; exit 1; }
grep "^call" $O/launch_k20.txt
