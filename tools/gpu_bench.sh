set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r01 -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o r01 -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/pf.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o r01 -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/pw.log 2>&1
python tools/hbm_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/hbm_traffic.json
cat gpurun_out/bench.json gpurun_out/hbm_traffic.json
find gpurun_out/prof -name "*stats*"
