# round-6: same-box A/B of the burn-in tuning test without a division on the driver's command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zzt
mkdir -p $O
for i in 1 2 3 4; do
  for v in head tm; do
    NESTMC_LIB=abtmp/libnestmc_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --cpu-seconds 0 > $O/b_${v}_$i.txt 2>&1 || { tail -20 $O/b_${v}_$i.txt; exit 1; }
    grep '^{' $O/b_${v}_$i.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' %.4g" % d["value"], "wall %.4f ev %.4f" % (d["wall_ms"], d["event_ms"]))'
  done
done
for v in head tm; do
  NESTMC_LIB=abtmp/libnestmc_$v.so timeout -k 10 300 python -u bench.py --no-pmc --cpu-seconds 0 > $O/long_$v.txt 2>&1 || { tail -20 $O/long_$v.txt; exit 1; }
  grep '^{' $O/long_$v.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' 2000-it %.4g" % d["value"], "ev %.4f" % d["event_ms"])'
done
