#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
NMC_SQ=0 NMC_CTL_TILES=2 timeout -k 10 120 python tools/stamps.py partial 1000 > gpurun_out/stamps_i_orig.json 2>&1
echo "done rc=$?"
