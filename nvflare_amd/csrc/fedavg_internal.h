// fedavg_internal.h -- shared between the HIP kernels and the C-ABI layer (not installed).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nvflare_amd_fedavg.h"

namespace fedavg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;          // 4 waves of 64 lanes
constexpr int kMaxRowsPerLaunch = 128;  // rows per launch carried in the kernel-argument segment

// Row table passed BY VALUE in the kernarg segment: wave-uniform pointers/weights live in SGPRs.
struct RowTableF32 {
    const f32x4* rows[kMaxRowsPerLaunch];
    float w[kMaxRowsPerLaunch];
};

// Tiled slab: per launch, the slot (client row inside each tile) and weight of every client in arrival order.
struct SlotTableF32 {
    int slot[kMaxRowsPerLaunch];
    float w[kMaxRowsPerLaunch];
};

struct RowTableGeneric {
    const void* rows[kMaxRowsPerLaunch];
    double w[kMaxRowsPerLaunch];
};

hipError_t launch_rows_f32x4(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4, int op,
                             int fin, float fin_val, int grid, int unroll, int variant, hipStream_t s);
hipError_t launch_tiled_f32x4(const SlotTableF32& tab, int K, const float* slab, int64_t seg4, int64_t tstride4,
                              int64_t tile4,
                              const float* acc_in, float* out, int64_t n4, int op, int fin, float fin_val, int grid,
                              int unroll, int variant, hipStream_t s);
hipError_t launch_fill_synthetic_tiled_f32(float* slab, int64_t k_max, int64_t tile_elems, int64_t seg, int64_t tstride,
                                           int64_t n, uint64_t seed, uint64_t col0, int grid, hipStream_t s);
hipError_t launch_rows_generic(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n,
                               int in_dtype, int acc_dtype, int op, int fin, double fin_val, int grid,
                               hipStream_t s);
hipError_t launch_fill_synthetic_f32(float* dst, int64_t n, uint64_t seed, uint64_t row, uint64_t col0, int grid,
                                     hipStream_t s);
hipError_t launch_gather_f32(const float* src, const uint64_t* idx, float* dst, int64_t m, hipStream_t s);

}  // namespace fedavg
