#!/bin/bash
# Round-4: per-wave barrier-A arrivals in the sweep kernel (stamps build), three policies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
NMC_SQ=0 NMC_CTL_TILES=2 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_g_orig.json 2>&1 &&
NMC_SQ=0 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_g_sq0.json 2>&1 &&
timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_g_sq1.json 2>&1
echo "done rc=$?"
