#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/mcmc-for-nested-data_amd/nestmc/libnestmc_lic.so
timeout -k 10 300 python tools/cfgbench.py cfg5 > gpurun_out/g2_def.jsonl 2>&1; echo "d rc=$?"
NESTMC_LIB=$L timeout -k 10 300 python tools/cfgbench.py cfg5 > gpurun_out/g2_lic.jsonl 2>&1; echo "l rc=$?"
timeout -k 10 300 python tools/cfgbench.py cfg5 > gpurun_out/g2_def2.jsonl 2>&1; echo "d2 rc=$?"
NESTMC_LIB=$L timeout -k 10 300 python tools/cfgbench.py cfg5 > gpurun_out/g2_lic2.jsonl 2>&1; echo "l2 rc=$?"
