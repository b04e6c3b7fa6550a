#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
./tools/pmc_pass.sh ic_sweep cfg3 "SQC_ICACHE_MISSES SQC_ICACHE_HITS" && echo ic1 ok &&
./tools/pmc_pass.sh ic_run cfg3 "SQC_ICACHE_MISSES SQC_ICACHE_HITS" NMC_SWEEP=0 && echo ic2 ok &&
./tools/pmc_pass.sh sq_sweep cfg3 "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS" && echo sq1 ok &&
./tools/pmc_pass.sh sq_run cfg3 "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS" NMC_SWEEP=0 && echo sq2 ok
echo "done rc=$?"
