# round-6 GPU job: resident-launch tests, then the driver's bench command with and without
# the resident launch (each step under its own limit; the first failure ends the job)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
# (an assertion failure goes on to the bench; a fault, abort or time limit ends the job)
case $rc in 0|1) ;; *) exit $rc ;; esac
B="python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
for i in 1 2; do
  timeout -k 10 120 $B > $O/res_$i.txt 2>&1 || { tail -20 $O/res_$i.txt; exit 1; }
  timeout -k 10 120 $B --no-resident > $O/nores_$i.txt 2>&1 || { tail -20 $O/nores_$i.txt; exit 1; }
done
NMC_XMAP=0 timeout -k 10 120 $B > $O/noxmap_1.txt 2>&1 || exit 1
NMC_XMAP=0 timeout -k 10 120 $B --no-resident > $O/noxmap_nores.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 $B --no-resident > $O/devk.txt 2>&1 || exit 1
NMC_TRACE_CALLS=1 timeout -k 10 120 $B > $O/trace_res.txt 2>&1 || exit 1
for f in $O/res_*.txt $O/nores_*.txt $O/noxmap*.txt $O/devk.txt $O/trace_res.txt; do
  echo "$f $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]), "launch_us %.1f" % d["roofline"]["avg_launch_us"], d["config"]["resident"])')"
done
