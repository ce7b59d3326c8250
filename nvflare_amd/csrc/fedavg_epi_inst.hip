// fedavg_epi_inst.hip -- instantiations of the fp32 aggregation + server-optimizer epilogue kernels for ONE
// (arithmetic mode, finalisation) pair.  The build compiles this file once per pair (nvflare_amd/_build.py
// EPI_UNITS: -DFEDAVG_EPI_OP, -DFEDAVG_EPI_FIN, -DFEDAVG_EPI_FN = the entry's name) so the nine objects --
// every optimizer kind x acc_in x launch form each -- compile in parallel.
#include "fedavg_epi.h"

#if !defined(FEDAVG_EPI_OP) || !defined(FEDAVG_EPI_FIN) || !defined(FEDAVG_EPI_FN)
// a plain `hipcc -c` of this file (no defines) builds the torch / div unit
#define FEDAVG_EPI_OP FEDAVG_OP_TORCH
#define FEDAVG_EPI_FIN FEDAVG_FIN_DIV
#define FEDAVG_EPI_FN launch_epi_torch_div
#endif

namespace fedavg {

hipError_t FEDAVG_EPI_FN(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    return launch_epi_f<FEDAVG_EPI_OP, FEDAVG_EPI_FIN>(L, E, s, nl);
}

}  // namespace fedavg
