#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py partial 2000 0 128 256 > gpurun_out/stamps_cfg4_s.json 2>&1; echo "s rc=$?"
timeout -k 10 120 python tools/stamps.py partial 2000 0 64 256 > gpurun_out/stamps_cfg4_s64.json 2>&1; echo "s64 rc=$?"
