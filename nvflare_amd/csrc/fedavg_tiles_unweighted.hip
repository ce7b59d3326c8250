// fedavg_tiles_unweighted.hip -- instantiations of the fp32 tiled aggregation kernels for the unweighted arithmetic
// (one translation unit per mode: the three compile in parallel).
#include "fedavg_tiles.h"

namespace fedavg {

hipError_t launch_tiles_f32x4_unweighted(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    return launch_tiles_o<FEDAVG_OP_UNWEIGHTED>(L, s, nl);
}

}  // namespace fedavg
