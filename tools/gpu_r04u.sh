#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/cfgbench.py cfg4 cfg4c64 > gpurun_out/u_cfg.jsonl 2> gpurun_out/u_cfg.err; echo "cfg rc=$?"
NMC_NOPRIO=2 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/u_np.jsonl 2> gpurun_out/u_np.err; echo "np rc=$?"
NMC_CTL_TILES=0 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/u_ct0.jsonl 2> gpurun_out/u_ct0.err; echo "ct0 rc=$?"
NMC_PUB_EARLY=1 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/u_pe.jsonl 2> gpurun_out/u_pe.err; echo "pe rc=$?"
NMC_PUB_EARLY=1 timeout -k 10 150 python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0 > gpurun_out/u_pe3.json 2> gpurun_out/u_pe3.err; echo "pe3 rc=$?"
NMC_PUB_EARLY=1 NMC_SWEEP=1 timeout -k 10 150 python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0 > gpurun_out/u_pe3s.json 2> gpurun_out/u_pe3s.err; echo "pe3s rc=$?"
