#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 400 --warmup 20 --no-pmc --cpu-seconds 0"
ab() { local name=$1; shift; env "$@" timeout -k 10 150 $B > gpurun_out/x_$name.json 2> gpurun_out/x_$name.err; echo "$name rc=$?"; }
ab run NMC_SWEEP=0 && ab sw NMC_SWEEP=1 && ab sw8 NMC_SWEEP=1 NMC_SWEEP_WAVES=8 &&
ab swpe NMC_SWEEP=1 NMC_PUB_EARLY=1 && ab swg0 NMC_SWEEP=1 NMC_GIBBS_TILES=0 &&
ab swct2 NMC_SWEEP=1 NMC_CTL_TILES=2 && ab sw8pe NMC_SWEEP=1 NMC_SWEEP_WAVES=8 NMC_PUB_EARLY=1 NMC_GIBBS_TILES=0
echo "done rc=$?"
