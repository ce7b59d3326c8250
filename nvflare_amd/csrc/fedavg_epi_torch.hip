// fedavg_epi_torch.hip -- instantiations of the fp32 aggregation + server-optimizer epilogue kernels for the
// torch arithmetic (one translation unit per mode: the three compile in parallel).
#include "fedavg_epi.h"

namespace fedavg {

hipError_t launch_tiles_epi_f32x4_torch(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    return launch_epi_o<FEDAVG_OP_TORCH>(L, E, s, nl);
}

}  // namespace fedavg
