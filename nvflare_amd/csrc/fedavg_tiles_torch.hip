// fedavg_tiles_torch.hip -- instantiations of the fp32 tiled aggregation kernels for the torch arithmetic
// (one translation unit per mode: the three compile in parallel).
#include "fedavg_tiles.h"

namespace fedavg {

hipError_t launch_tiles_f32x4_torch(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    return launch_tiles_o<FEDAVG_OP_TORCH>(L, s, nl);
}

}  // namespace fedavg
