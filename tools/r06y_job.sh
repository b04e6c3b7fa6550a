# round-6: the gate branch marked cold (__builtin_expect): A/B against the previous build on
# one box (NESTMC_LIB=libnestmc_prev.so), driver's command and the 2 000-iteration run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
PREV=$PWD/mcmc-for-nested-data_amd/nestmc/libnestmc_prev.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
S20="--steps 20 --warmup 5 --no-pmc --cpu-seconds 0"
S2k="--no-pmc --cpu-seconds 0"
for i in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export NESTMC_LIB=$PREV; else unset NESTMC_LIB; fi
    timeout -k 10 120 python -u bench.py $S20 > $O/${lib}_d_$i.txt 2>&1 || exit 1
    timeout -k 10 120 python -u bench.py $S20 --no-resident > $O/${lib}_dn_$i.txt 2>&1 || exit 1
    timeout -k 10 120 python -u bench.py $S2k --no-resident > $O/${lib}_l_$i.txt 2>&1 || exit 1
  done
done
unset NESTMC_LIB
for f in $O/*_d_*.txt $O/*_dn_*.txt $O/*_l_*.txt; do
  echo "$f $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4g" % d["value"], "wall %.4f ev %.4f launch %.1f" % (d["wall_ms"], d["event_ms"], d["roofline"]["avg_launch_us"]))')"
done
