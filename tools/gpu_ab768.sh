#!/bin/bash
# A/B: the shipped 512-thread step kernel against the 768-thread build (make t768: 12 waves,
# 168 VGPRs, 32 tile slots) at cfg 3, kernel us/iter from bench.py's HIP-event pass.
#   usage: tools/gpu_ab768.sh TAG
set -o pipefail
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
LIB768=mcmc-for-nested-data_amd/nestmc/libnestmc_t768.so
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-pmc --cpu-seconds 0 \
      > gpurun_out/ab768_${TAG}_$name.json 2> gpurun_out/ab768_${TAG}_$name.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab768_${TAG}_$name.json')); r=d['roofline']; print('$name', '%.4g' % d['value'], 'kernel us/iter %.3f' % (r['avg_launch_us'] / r['iterations_per_launch']), d['config']['launch']['mode'], 'W', d['config']['launch']['waves_per_group'])"
}
run base || exit $?
run t768_w8 NESTMC_LIB=$LIB768 || exit $?
run t768_w12_lds NESTMC_LIB=$LIB768 NMC_WAVES=12 NMC_NO_HREG=1 || exit $?
run t768_w12_lds_t32 NESTMC_LIB=$LIB768 NMC_WAVES=12 NMC_NO_HREG=1 NMC_TILE_ROWS=32 || exit $?
run t768_w12_reg NESTMC_LIB=$LIB768 NMC_WAVES=12 || exit $?
run base_lds NMC_NO_HREG=1 || exit $?
