#!/bin/bash
# Step-kernel phase stamps (diagnostic build) for several likelihood tile sizes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in ${TILES:-32 64 128}; do
  NMC_TILE_ROWS=$T timeout -k 10 120 python tools/stamps.py partial > gpurun_out/stamps_t$T.json 2>&1 || exit $?
  echo "tile $T: $(python3 -c "import json;d=json.load(open('gpurun_out/stamps_t$T.json'));print({k:(v['iter_cycles'],v['phase_cycles'][:2]) for k,v in d['stamps'].items()})")"
done
