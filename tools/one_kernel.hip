// one_kernel.hip -- diagnostics (not shipped): instantiates the cfg-3 step kernel alone so its
// register use and spills can be read in seconds (tools/regusage.py compiles whole TUs):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-machine-licm \
//     -mllvm -amdgpu-atomic-optimizer-strategy=None --cuda-device-only \
//     -Rpass-analysis=kernel-resource-usage -I mcmc-for-nested-data_amd/csrc -I include \
//     -c tools/one_kernel.hip -o /tmp/one.o
#include "kernels.h"   // (-I mcmc-for-nested-data_amd/csrc)
template __global__ void nmc_k_run<FamLinreg<2>, NMC_MODE_SYNC_REG, true>(Dev, FamLinreg<2>,
                                                                          const double*, int,
                                                                          int, int);
#ifdef NMC_ONE_SWEEP   // the cfg-4 step kernel (-DNMC_ONE_SWEEP)
#include "sweep.h"
template __global__ void nmc_k_sweep<FamLinreg<2>, NMC_MODE_SYNC_OWN>(nmc_sweep_args<FamLinreg<2>>);
#endif
#ifdef NMC_ONE_RES   // the resident cfg-3 step kernel (-DNMC_ONE_RES)
template __global__ void nmc_k_run<FamLinreg<2>, NMC_MODE_SYNC_REG, true, true>(
    Dev, FamLinreg<2>, const double*, int, int, int);
#endif
