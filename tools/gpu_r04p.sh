#!/bin/bash
# Round-4 close-out 2/2: bench lines with PMC traffic and the CPU baseline, per workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/p_cfg3_a.json 2> gpurun_out/p_cfg3_a.err; echo "cfg3a rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/p_cfg3_b.json 2> gpurun_out/p_cfg3_b.err; echo "cfg3b rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/p_cfg3_20.json 2> gpurun_out/p_cfg3_20.err; echo "cfg3_20 rc=$?"
timeout -k 10 400 python bench.py --workload cfg2 > gpurun_out/p_cfg2.json 2> gpurun_out/p_cfg2.err; echo "cfg2 rc=$?"
timeout -k 10 500 python bench.py --workload cfg4 --steps 200 --warmup 20 > gpurun_out/p_cfg4.json 2> gpurun_out/p_cfg4.err; echo "cfg4 rc=$?"
timeout -k 10 500 python bench.py --workload cfg5 --steps 40 --warmup 5 > gpurun_out/p_cfg5.json 2> gpurun_out/p_cfg5.err; echo "cfg5 rc=$?"
timeout -k 10 300 python tools/cfgbench.py cfg5 cfg5user cfg4 cfg2 > gpurun_out/p_cfgbench.jsonl 2> gpurun_out/p_cfgbench.err; echo "cfgbench rc=$?"
