// fedavg_epi_inst.hip -- instantiations of the fp32 aggregation + server-optimizer epilogue kernels for ONE
// (arithmetic mode, finalisation) pair.  The build compiles this file once per pair (nvflare_amd/_build.py
// EPI_UNITS: -DFEDAVG_EPI_OP, -DFEDAVG_EPI_FIN, -DFEDAVG_EPI_FN = the entry's name) so the objects -- every optimizer
// kind x launch form each -- compile in parallel.  -DFEDAVG_EPI_STEP builds launch_epi_step instead: the server step
// alone (no clients, the aggregate as the chained sum, FIN_NONE; product builds, fedavg_internal.h epi_direct).
#include "fedavg_epi.h"

#if !defined(FEDAVG_EPI_STEP) && (!defined(FEDAVG_EPI_OP) || !defined(FEDAVG_EPI_FIN) || !defined(FEDAVG_EPI_FN))
// a plain `hipcc -c` of this file (no defines) builds the torch / div unit
#define FEDAVG_EPI_OP FEDAVG_OP_TORCH
#define FEDAVG_EPI_FIN FEDAVG_FIN_DIV
#define FEDAVG_EPI_FN launch_epi_torch_div
#endif

namespace fedavg {

#if defined(FEDAVG_EPI_STEP)
hipError_t launch_epi_step(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    if (L.k != 0 || !L.acc_in || L.fin != FEDAVG_FIN_NONE) return hipErrorNotSupported;
    return launch_epi_a<FEDAVG_OP_TORCH, FEDAVG_FIN_NONE, true>(L, E, s, nl);  // no clients: the mode is never used
}
#else
// The build compiles each pair twice (nvflare_amd/_build.py): FEDAVG_EPI_PART=1 is the pair's entry with every kind
// but these, =2 these -- Adam and NAdam, three sqrt forms each, the heaviest kernels -- as FEDAVG_EPI_FN2, so the
// pair's kernels compile in two halves in parallel (product build 5m40 -> 4m46 on 8 cores).  Without FEDAVG_EPI_PART
// one unit carries every kind.
constexpr unsigned kEpiKindsPart2 = (1u << FEDAVG_EPI_ADAM) | (1u << FEDAVG_EPI_NADAM);
#if defined(FEDAVG_EPI_PART) && FEDAVG_EPI_PART == 2
hipError_t FEDAVG_EPI_FN2(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    return launch_epi_f<FEDAVG_EPI_OP, FEDAVG_EPI_FIN, kEpiKindsPart2>(L, E, s, nl);
}
#elif defined(FEDAVG_EPI_PART) && FEDAVG_EPI_PART == 1
hipError_t FEDAVG_EPI_FN2(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl);
hipError_t FEDAVG_EPI_FN(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    if (E.kind >= 0 && E.kind < 32 && ((kEpiKindsPart2 >> E.kind) & 1u)) return FEDAVG_EPI_FN2(L, E, s, nl);
    return launch_epi_f<FEDAVG_EPI_OP, FEDAVG_EPI_FIN, ~kEpiKindsPart2>(L, E, s, nl);
}
#else
hipError_t FEDAVG_EPI_FN(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    return launch_epi_f<FEDAVG_EPI_OP, FEDAVG_EPI_FIN>(L, E, s, nl);
}
#endif
#endif

}  // namespace fedavg
