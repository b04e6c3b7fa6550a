#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
L=$PWD/mcmc-for-nested-data_amd/nestmc/libnestmc_lic.so
timeout -k 10 150 $B > gpurun_out/z_def1.json 2>&1; echo "d1 rc=$?"
NESTMC_LIB=$L timeout -k 10 150 $B > gpurun_out/z_lic1.json 2>&1; echo "l1 rc=$?"
timeout -k 10 150 $B > gpurun_out/z_def2.json 2>&1; echo "d2 rc=$?"
NESTMC_LIB=$L timeout -k 10 150 $B > gpurun_out/z_lic2.json 2>&1; echo "l2 rc=$?"
timeout -k 10 150 $B --workload cfg2 > gpurun_out/z_def_c2.json 2>&1; echo "dc2 rc=$?"
NESTMC_LIB=$L timeout -k 10 150 $B --workload cfg2 > gpurun_out/z_lic_c2.json 2>&1; echo "lc2 rc=$?"
timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/z_c4.jsonl 2>&1; echo "c4 rc=$?"
NMC_ZIN=1 timeout -k 10 200 python tools/cfgbench.py cfg4 > gpurun_out/z_c4zin.jsonl 2>&1; echo "c4zin rc=$?"
