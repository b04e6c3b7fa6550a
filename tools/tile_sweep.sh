#!/bin/bash
# Bench line per likelihood tile size (NMC_TILE_ROWS, diagnostics).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in ${TILES:-48 64 80 96 128}; do
  NMC_TILE_ROWS=$T timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --cpu-seconds 0 --no-pmc > gpurun_out/tile_$T.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/tile_$T.json'));print('tile $T: %.4g /s  %.3f us/iter' % (d['value'], d['ms_per_step']*1e3))"
done
