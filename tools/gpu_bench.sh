# Round-end style measurement on one MI355X: bench line, kernel-trace stats, and the
# two PMC passes for HBM traffic (FETCH_SIZE / WRITE_SIZE in separate runs).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=${1:-r01}
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $R -- python3 bench.py --cpu-seconds 0 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o $R -- python3 bench.py --steps 200 --warmup 200 --cpu-seconds 0 > gpurun_out/pf.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o $R -- python3 bench.py --steps 200 --warmup 200 --cpu-seconds 0 > gpurun_out/pw.log 2>&1
python tools/hbm_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write 600 > gpurun_out/hbm_traffic.json
cat gpurun_out/bench.json gpurun_out/hbm_traffic.json
find gpurun_out/prof -name "*stats*"
