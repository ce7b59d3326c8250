// fedavg_kernels.hip -- CDNA4 (gfx950) kernels for the FedAvg weighted accumulate-and-scale.
//
// Reference arithmetic (NVFlare nvflare/app_common/aggregators/weighted_aggregation_helper.py):
//   numpy branch  :188-193 (first T = v*w), :210-214 (T = T + v*w), :236 (T * (1.0/count))
//   torch branch  :181-187 (first T = v.mul(w)), :203-209 (T.add_(v, alpha=w) == one FMA), :233 (T.div_(count))
//   weigh_by_local_iter=False :186-199, :208-215 (T = v; T = T + v)
//
// Design:
//   * One pass: every parameter reads its K client values once and writes its result once -- 4K + 4 bytes
//     per fp32 parameter, no temporaries.  HBM-bound; no MFMA (elementwise, not a contraction).
//   * The per-element operation sequence is the reference's, in arrival order, so results are bitwise
//     equal to the reference.  Compile with -ffp-contract=off (numpy mode rounds the multiply and the add
//     separately); the torch mode calls __builtin_fmaf.  fp32 denormals are preserved (IEEE mode).
//   * Client data is TILED: element i of client k is at  base[k] + (i / TILE) * tile_stride + i % TILE.
//     With tile_stride == TILE this is a contiguous row; the engine's slabs interleave the K clients per
//     tile (tile_stride = slots * TILE) so one tile's K client segments are contiguous in HBM and a block
//     streams them as one sequential run.  Measured on MI355X (profiles/r01): 83 % of HBM spec = 96 % of
//     the chip's own streaming-read ceiling, against 75 % for K independent row streams.
//   * Base pointers and fp32 weights travel in the kernel-argument segment: wave-uniform, kept in SGPRs.
//   * Each lane owns CPL float4 columns of a tile (a wave reads 1 KiB contiguous per client and column
//     group); UNROLL clients' loads are issued before their arrival-ordered arithmetic.  Loads and the
//     result stores are nontemporal: every byte is touched exactly once.
#include <hip/hip_runtime.h>
//
// This file: the generic / fp64 kernels, the synthetic-input and gather kernels, and the dispatchers of the
// fp32 tiled kernels, whose templates live in fedavg_tiles.h / fedavg_epi.h and are instantiated per
// arithmetic mode in fedavg_tiles_*.hip / fedavg_epi_*.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fedavg_arith.h"

namespace fedavg {

// ---------------------------------------------------------------------------------------------
// generic scalar kernel: any (Tin, Tacc) pair, contiguous rows, any alignment (ragged tails, fp64, ints)
// ---------------------------------------------------------------------------------------------
// The step and the finalisation are launch arguments here (round 5: one instantiation per (Tin, Tacc, ACC_IN) instead
// of nine -- this is the path for odd dtypes, unaligned rows and ragged tails, not the streaming one); the per-element
// sequence is fedavg_arith.h's first_op / step_op / fin_op for that op and fin.
template <int OP, typename Tacc>
__device__ __forceinline__ Tacc step_any(const Tacc acc, const Tacc v, const Tacc w) {
    return step_op<OP>(acc, v, w);
}

template <typename Tin, typename Tacc, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_rows_generic(const RowTableGeneric tab, const int K,
                                                               const Tacc* acc_in, Tacc* out, const int64_t n,
                                                               const double fin_val_d, const int op, const int fin) {
    const Tacc fin_val = (Tacc)fin_val_d;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        Tacc acc;
        int k = 0;
        if constexpr (ACC_IN) {
            acc = acc_in[i];
        } else {
            const Tacc v = (Tacc)(static_cast<const Tin*>(tab.rows[0])[i]);
            acc = op == FEDAVG_OP_UNWEIGHTED ? first_op<FEDAVG_OP_UNWEIGHTED>(v, (Tacc)tab.w[0])
                                             : first_op<FEDAVG_OP_NUMPY>(v, (Tacc)tab.w[0]);
            k = 1;
        }
        for (; k < K; ++k) {
            const Tacc v = (Tacc)(static_cast<const Tin*>(tab.rows[k])[i]);
            const Tacc w = (Tacc)tab.w[k];
            acc = op == FEDAVG_OP_TORCH        ? step_any<FEDAVG_OP_TORCH>(acc, v, w)
                  : op == FEDAVG_OP_UNWEIGHTED ? step_any<FEDAVG_OP_UNWEIGHTED>(acc, v, w)
                                               : step_any<FEDAVG_OP_NUMPY>(acc, v, w);
        }
        out[i] = fin == FEDAVG_FIN_SCALE ? fin_op<FEDAVG_FIN_SCALE>(acc, fin_val)
                 : fin == FEDAVG_FIN_DIV ? fin_op<FEDAVG_FIN_DIV>(acc, fin_val)
                                         : acc;
    }
}

// ---------------------------------------------------------------------------------------------
// fp64 rows (numpy's default dtype), every pointer 16-byte aligned: each lane owns two consecutive values
// (one 16-byte load per client), four clients' loads in flight before their arrival-ordered arithmetic,
// nontemporal loads and stores.  n2 = pairs; an odd last element goes to the scalar kernel.
// ---------------------------------------------------------------------------------------------
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int OP, int FIN, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_rows_f64x2(const RowTableGeneric tab, const int K,
                                                             const f64x2* acc_in, f64x2* out, const int64_t n2,
                                                             const double fin_val) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < n2; g += stride) {
        f64x2 acc;
        int k = 0;
        if constexpr (ACC_IN) {
            acc = __builtin_nontemporal_load(acc_in + g);
        } else {
            const f64x2 v = __builtin_nontemporal_load(static_cast<const f64x2*>(tab.rows[0]) + g);
            acc = f64x2{first_op<OP>(v[0], tab.w[0]), first_op<OP>(v[1], tab.w[0])};
            k = 1;
        }
        for (; k + 4 <= K; k += 4) {
            f64x2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(static_cast<const f64x2*>(tab.rows[k + u]) + g);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc = f64x2{step_op<OP>(acc[0], v[u][0], tab.w[k + u]), step_op<OP>(acc[1], v[u][1], tab.w[k + u])};
        }
        for (; k < K; ++k) {
            const f64x2 v = __builtin_nontemporal_load(static_cast<const f64x2*>(tab.rows[k]) + g);
            acc = f64x2{step_op<OP>(acc[0], v[0], tab.w[k]), step_op<OP>(acc[1], v[1], tab.w[k])};
        }
        __builtin_nontemporal_store(f64x2{fin_op<FIN>(acc[0], fin_val), fin_op<FIN>(acc[1], fin_val)}, out + g);
    }
}

// ---------------------------------------------------------------------------------------------
// TILED fp64 (the engine's fp64 arena, numpy's default dtype): element i of client k lives at
//   bases[k] + (i / 4096) * tile_stride + i % 4096          (fp64 elements)
// A block owns a tile (4096 values = 32 KiB per client); each lane owns 8 f64x2 columns, so a wave reads
// 1 KiB contiguous per client and column, two clients' loads (16 x 16 B per lane) in flight before their
// arrival-ordered arithmetic.  Units below are pairs (f64x2).
// ---------------------------------------------------------------------------------------------
constexpr int kCpl64 = kTile64Elems / (2 * kBlock);  // 8
#ifndef FEDAVG_F64_UNROLL
#define FEDAVG_F64_UNROLL 2  // clients whose loads are in flight together (16 x 16 B per lane)
#endif
constexpr int kBurstTiles64 = 4;  // tiles per block per burst launch: 4 x kCpl64 staged pairs = 128 VGPRs
constexpr int kBurstLdsTiles64 = 2;  // and 2 more in LDS: 2 x 32 KiB per block (2 blocks fit a CU)

// One tile's arrival-ordered sum for this lane's kCpl64 pairs, finalised.
template <int OP, int FIN, bool ACC_IN>
__device__ __forceinline__ void tile_sum64(f64x2 (&res)[kCpl64], const RowTableGeneric& tab, const int K,
                                           const int64_t off, const int64_t col, const f64x2* acc_in, const int64_t b2,
                                           const int64_t e2, const double fin_val) {
    constexpr int UNROLL = FEDAVG_F64_UNROLL;
    f64x2 acc[kCpl64];
    int k = 0;
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < kCpl64; ++c) {
            const int64_t i = col + c * kBlock;
            acc[c] = (i >= b2 && i < e2) ? acc_in[i] : f64x2{0, 0};
        }
    } else {
        const f64x2* r = static_cast<const f64x2*>(tab.rows[0]) + off;
#pragma unroll
        for (int c = 0; c < kCpl64; ++c) {
            const f64x2 v = __builtin_nontemporal_load(r + c * kBlock);
            acc[c] = f64x2{first_op<OP>(v[0], tab.w[0]), first_op<OP>(v[1], tab.w[0])};
        }
        k = 1;
    }
    for (; k + UNROLL <= K; k += UNROLL) {
        f64x2 v[UNROLL][kCpl64];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const f64x2* r = static_cast<const f64x2*>(tab.rows[k + u]) + off;
#pragma unroll
            for (int c = 0; c < kCpl64; ++c) v[u][c] = __builtin_nontemporal_load(r + c * kBlock);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int c = 0; c < kCpl64; ++c)
                acc[c] = f64x2{step_op<OP>(acc[c][0], v[u][c][0], tab.w[k + u]),
                               step_op<OP>(acc[c][1], v[u][c][1], tab.w[k + u])};
    }
    for (; k < K; ++k) {
        const f64x2* r = static_cast<const f64x2*>(tab.rows[k]) + off;
#pragma unroll
        for (int c = 0; c < kCpl64; ++c) {
            const f64x2 v = __builtin_nontemporal_load(r + c * kBlock);
            acc[c] = f64x2{step_op<OP>(acc[c][0], v[0], tab.w[k]), step_op<OP>(acc[c][1], v[1], tab.w[k])};
        }
    }
#pragma unroll
    for (int c = 0; c < kCpl64; ++c) res[c] = f64x2{fin_op<FIN>(acc[c][0], fin_val), fin_op<FIN>(acc[c][1], fin_val)};
}

// per-tile-store form (launch variant bit 3)
template <int OP, int FIN, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_tiles_f64x2(const RowTableGeneric tab, const int K,
                                                              const int64_t tstride2, const f64x2* acc_in, f64x2* out,
                                                              const int64_t b2, const int64_t e2, const double fin_val) {
    constexpr int64_t T2 = (int64_t)kCpl64 * kBlock;
    const int64_t t_last = (e2 - 1) / T2;
    for (int64_t t = b2 / T2 + blockIdx.x; t <= t_last; t += gridDim.x) {
        f64x2 res[kCpl64];
        tile_sum64<OP, FIN, ACC_IN>(res, tab, K, t * tstride2 + threadIdx.x, t * T2 + threadIdx.x, acc_in, b2, e2, fin_val);
#pragma unroll
        for (int c = 0; c < kCpl64; ++c) {
            const int64_t i = t * T2 + threadIdx.x + c * kBlock;
            if (i >= b2 && i < e2) __builtin_nontemporal_store(res[c], out + i);
        }
    }
}

// BURST form (the default; fedavg_tiles.h fedavg_tiles_burst_f32x4): TPB tiles per block per launch, results
// held in registers (kCpl64 pairs per tile) and stored after the block's last tile.
// TPB_LDS > 0 (the default, burst mode 2): that many more tiles per block, results held in LDS (32 KiB per tile;
// each lane reads back only what it wrote), in rolled loops so the tile body is not copied TPB_LDS more times.
template <int OP, int FIN, bool ACC_IN, int TPB, int TPB_LDS = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
fedavg_tiles_f64x2_burst(const RowTableGeneric tab, const int K, const int64_t tstride2, const f64x2* acc_in,
                         f64x2* out, const int64_t b2, const int64_t e2, const double fin_val, const int64_t t0,
                         const int64_t t_end) {
    constexpr int64_t T2 = (int64_t)kCpl64 * kBlock;
    f64x2 res[TPB][kCpl64];
    __shared__ f64x2 staged[TPB_LDS > 0 ? TPB_LDS * kCpl64 * kBlock : 1];
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end)
            tile_sum64<OP, FIN, ACC_IN>(res[m], tab, K, t * tstride2 + threadIdx.x, t * T2 + threadIdx.x, acc_in, b2, e2,
                                        fin_val);
    }
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f64x2 r[kCpl64];
            tile_sum64<OP, FIN, ACC_IN>(r, tab, K, t * tstride2 + threadIdx.x, t * T2 + threadIdx.x, acc_in, b2, e2,
                                        fin_val);
#pragma unroll
            for (int c = 0; c < kCpl64; ++c) staged[((m - TPB) * kCpl64 + c) * kBlock + threadIdx.x] = r[c];
        }
    }
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < kCpl64; ++c) {
                const int64_t i = t * T2 + threadIdx.x + c * kBlock;
                if (i >= b2 && i < e2)
                    __builtin_nontemporal_store(staged[((m - TPB) * kCpl64 + c) * kBlock + threadIdx.x], out + i);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < kCpl64; ++c) {
                const int64_t i = t * T2 + threadIdx.x + c * kBlock;
                if (i >= b2 && i < e2) __builtin_nontemporal_store(res[m][c], out + i);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// synthetic inputs (bit-identical host twin: oracle/fedavg_oracle.c oracle_synth_value), written to a
// tiled row: logical element i goes to dst[(i / tile) * tile_stride + i % tile]
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void __launch_bounds__(kBlock) fedavg_fill_synthetic_f32(float* dst, const int64_t n, const int64_t tile,
                                                                     const int64_t tstride, const uint64_t seed,
                                                                     const uint64_t row, const uint64_t col0) {
    const uint64_t base = (seed * 0x9E3779B97F4A7C15ULL) ^ (row * 0xD1B54A32D192ED03ULL);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t col = col0 + (uint64_t)i;
        int32_t s = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) s += (int32_t)(mix32(base + col * 4ULL + (uint64_t)j) >> 8);
        s -= (int32_t)(1 << 25);
        const int64_t t = i / tile;
        dst[t * tstride + (i - t * tile)] = (float)s * 1.0323827e-07f;
    }
}

__global__ void __launch_bounds__(kBlock) fedavg_gather_f32(const float* src, const uint64_t* idx, float* dst,
                                                             const int64_t m) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < m) dst[i] = src[idx[i]];
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
bool tiles_use_burst(int64_t tile4, int unroll, int variant) {
    const int64_t cpl = tile4 / kBlock;
    return !(variant & (kVariantTileStores | kVariantTemporalLoads | kVariantTemporalStores)) &&
           cpl * (unroll + kBurstTiles) <= 64;
}

hipError_t launch_tiles_f32x4(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    switch (L.op) {
        case FEDAVG_OP_TORCH:
            return launch_tiles_f32x4_torch(L, s, nl);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_tiles_f32x4_unweighted(L, s, nl);
        default:
            return launch_tiles_f32x4_numpy(L, s, nl);
    }
}

hipError_t launch_tiles_epi_f32x4(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    using Fn = hipError_t (*)(const TileLaunch&, const EpiParams&, hipStream_t, uint64_t*);
    if (!epi_direct(L.op, L.fin, L.k, L.acc_in != nullptr)) return hipErrorNotSupported;  // fedavg_capi.cpp splits it
#if defined(FEDAVG_AB)
    static constexpr Fn kFns[3][3] = {  // [mode][finalisation]: numpy (and any other op), torch, unweighted
        {launch_epi_numpy_none, launch_epi_numpy_scale, launch_epi_numpy_div},
        {launch_epi_torch_none, launch_epi_torch_scale, launch_epi_torch_div},
        {launch_epi_unweighted_none, launch_epi_unweighted_scale, launch_epi_unweighted_div}};
#else
    if (L.acc_in) return launch_epi_step(L, E, s, nl);  // the server step alone (no clients, FIN_NONE)
    static constexpr Fn kFns[3][3] = {  // the product's (mode, finalisation) pairs (epi_direct)
        {nullptr, launch_epi_numpy_scale, nullptr},
        {nullptr, launch_epi_torch_scale, launch_epi_torch_div},
        {nullptr, launch_epi_unweighted_scale, launch_epi_unweighted_div}};
#endif
    const int o = L.op == FEDAVG_OP_TORCH ? 1 : (L.op == FEDAVG_OP_UNWEIGHTED ? 2 : 0);
    const int f = L.fin == FEDAVG_FIN_SCALE ? 1 : (L.fin == FEDAVG_FIN_DIV ? 2 : 0);
    return kFns[o][f] ? kFns[o][f](L, E, s, nl) : hipErrorNotSupported;
}

template <typename Tin, typename Tacc>
static hipError_t launch_generic_t(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int op,
                                   int fin, double fin_val, int grid, hipStream_t s) {
    if (fin != FEDAVG_FIN_SCALE && fin != FEDAVG_FIN_DIV) fin = FEDAVG_FIN_NONE;
    if (op != FEDAVG_OP_TORCH && op != FEDAVG_OP_UNWEIGHTED) op = FEDAVG_OP_NUMPY;
    if (acc_in) {
        hipLaunchKernelGGL((fedavg_rows_generic<Tin, Tacc, true>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const Tacc*>(acc_in), static_cast<Tacc*>(out), n, fin_val, op, fin);
    } else {
        hipLaunchKernelGGL((fedavg_rows_generic<Tin, Tacc, false>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const Tacc*>(acc_in), static_cast<Tacc*>(out), n, fin_val, op, fin);
    }
    return hipGetLastError();
}

template <int OP, int FIN>
static hipError_t launch_f64x2_f(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n2,
                                 double fin_val, int grid, hipStream_t s) {
    if (acc_in) {
        hipLaunchKernelGGL((fedavg_rows_f64x2<OP, FIN, true>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const f64x2*>(acc_in), static_cast<f64x2*>(out), n2, fin_val);
    } else {
        hipLaunchKernelGGL((fedavg_rows_f64x2<OP, FIN, false>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const f64x2*>(acc_in), static_cast<f64x2*>(out), n2, fin_val);
    }
    return hipGetLastError();
}

template <int OP>
static hipError_t launch_f64x2_o(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n2, int fin,
                                 double fin_val, int grid, hipStream_t s) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_f64x2_f<OP, FEDAVG_FIN_SCALE>(tab, K, acc_in, out, n2, fin_val, grid, s);
        case FEDAVG_FIN_DIV:
            return launch_f64x2_f<OP, FEDAVG_FIN_DIV>(tab, K, acc_in, out, n2, fin_val, grid, s);
        default:
            return launch_f64x2_f<OP, FEDAVG_FIN_NONE>(tab, K, acc_in, out, n2, fin_val, grid, s);
    }
}

// fp64 -> fp64 rows with every pointer 16-byte aligned: the paired kernel over n / 2 pairs, the odd last
// element (if any) on the scalar kernel.  Returns hipErrorNotSupported when the rows do not qualify.
static hipError_t launch_rows_f64x2(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int op,
                                    int fin, double fin_val, int grid, hipStream_t s) {
    auto aligned = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
    bool ok = aligned(out) && aligned(acc_in) && n >= 2;
    for (int k = 0; ok && k < K; ++k) ok = aligned(tab.rows[k]);
    if (!ok) return hipErrorNotSupported;
    const int64_t n2 = n / 2;
    hipError_t e;
    switch (op) {
        case FEDAVG_OP_TORCH:
            e = launch_f64x2_o<FEDAVG_OP_TORCH>(tab, K, acc_in, out, n2, fin, fin_val, grid, s);
            break;
        case FEDAVG_OP_UNWEIGHTED:
            e = launch_f64x2_o<FEDAVG_OP_UNWEIGHTED>(tab, K, acc_in, out, n2, fin, fin_val, grid, s);
            break;
        default:
            e = launch_f64x2_o<FEDAVG_OP_NUMPY>(tab, K, acc_in, out, n2, fin, fin_val, grid, s);
    }
    if (e != hipSuccess || n % 2 == 0) return e;
    RowTableGeneric tail = tab;
    for (int k = 0; k < K; ++k) tail.rows[k] = static_cast<const double*>(tab.rows[k]) + 2 * n2;
    const void* tail_in = acc_in ? static_cast<const void*>(static_cast<const double*>(acc_in) + 2 * n2) : nullptr;
    return launch_generic_t<double, double>(tail, K, tail_in, static_cast<double*>(out) + 2 * n2, 1, op, fin, fin_val, 1, s);
}

// FEW-CLIENT fp64 burst form (round 5): 1-3 client reads, no chained sum -- fedavg_tiles.h fedavg_tiles_few_f32x4's
// shape with 32 KiB tiles: every load unconditional (a launch's slot past its last tile re-reads that tile; only real
// tiles are stored), the R register-held tiles' loads first, the L LDS-held tiles in groups of G, every store at the
// end.  The burst form's tile guard puts a basic-block boundary between its tiles' loads (fp64 x 1e9 at 1 / 2 clients:
// 74.2 / 74.2 % of 8 TB/s, profiles/r05/s8/f64.jsonl).  Per-element sequence as tile_sum64's: the same bits.
template <int OP, int FIN, int KC, int R, int L, int G, int B>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(B, 2)))
fedavg_tiles_f64x2_few(const RowTableGeneric tab, const int64_t tstride2, f64x2* out, const int64_t b2, const int64_t e2,
                       const double fin_val, const int64_t t0, const int64_t t_end) {
    static_assert(KC >= 1 && KC <= 3, "one to three row reads");
    static_assert(L == 0 || L % G == 0, "whole LDS groups");
    constexpr int CPL = kCpl64;
    constexpr int64_t T2 = (int64_t)CPL * kBlock;
    __shared__ f64x2 staged[L > 0 ? L * CPL * kBlock : 1];
    const int64_t t_first = t0 + blockIdx.x;
    auto load_tile = [&](f64x2 (&v)[KC][CPL], const int m) __attribute__((always_inline)) {
        int64_t t = t_first + (int64_t)m * gridDim.x;
        t = t < t_end ? t : t_end - 1;
        const int64_t off = t * tstride2 + threadIdx.x;
#pragma unroll
        for (int j = 0; j < KC; ++j)
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                v[j][c] = __builtin_nontemporal_load(static_cast<const f64x2*>(tab.rows[j]) + off + c * kBlock);
    };
    auto finish = [&](f64x2 (&res)[CPL], const f64x2 (&v)[KC][CPL]) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            f64x2 acc = f64x2{first_op<OP>(v[0][c][0], tab.w[0]), first_op<OP>(v[0][c][1], tab.w[0])};
#pragma unroll
            for (int j = 1; j < KC; ++j)
                acc = f64x2{step_op<OP>(acc[0], v[j][c][0], tab.w[j]), step_op<OP>(acc[1], v[j][c][1], tab.w[j])};
            res[c] = f64x2{fin_op<FIN>(acc[0], fin_val), fin_op<FIN>(acc[1], fin_val)};
        }
    };
    f64x2 vr[R][KC][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) load_tile(vr[m], L + m);
#pragma unroll
    for (int g = 0; g < L; g += G) {
        f64x2 v[G][KC][CPL];
#pragma unroll
        for (int m = 0; m < G; ++m) load_tile(v[m], g + m);
#pragma unroll
        for (int m = 0; m < G; ++m) {
            f64x2 r[CPL];
            finish(r, v[m]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((g + m) * CPL + c) * kBlock + threadIdx.x] = r[c];
        }
    }
    f64x2 res[R][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) finish(res[m], vr[m]);
#pragma unroll
    for (int m = 0; m < L + R; ++m) {
        const int64_t t = t_first + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T2 + threadIdx.x + c * kBlock;
                const f64x2 r = m < L ? staged[(m * CPL + c) * kBlock + threadIdx.x] : res[m < L ? 0 : m - L][c];
                if (i >= b2 && i < e2) __builtin_nontemporal_store(r, out + i);
            }
        }
    }
}

template <int OP, int FIN, int KC>
static hipError_t launch_f64_few(const RowTableGeneric& tab, int64_t ts2, f64x2* o, int64_t b2, int64_t e2,
                                 double fin_val, int grid, int form, hipStream_t s, uint64_t* nl) {
    constexpr int64_t T2 = (int64_t)kCpl64 * kBlock;
    const FewForm f = f64_few_form(KC, form);
#define FEDAVG_F64FEW(BB, RR, LL, GG)                                                                                    \
    if (f.bpc == BB && f.r == RR && f.l == LL && f.g == GG)                                                             \
        return burst_launches(b2 / T2, (e2 - 1) / T2 + 1, grid, RR + LL, nl, false,                                     \
                              [&](int nb, int64_t t0, int64_t t_end, uint32_t) {                                         \
                                  hipLaunchKernelGGL((fedavg_tiles_f64x2_few<OP, FIN, KC, RR, LL, GG, BB>), dim3(nb),   \
                                                     dim3(kBlock), 0, s, tab, ts2, o, b2, e2, fin_val, t0, t_end);       \
                              });
    if constexpr (KC == 1) {
        FEDAVG_F64FEW(2, 4, 2, 2)
        if constexpr (kABFew) {
            FEDAVG_F64FEW(2, 4, 2, 1)
            FEDAVG_F64FEW(1, 4, 4, 2)
            FEDAVG_F64FEW(2, 3, 2, 2)
            FEDAVG_F64FEW(1, 6, 4, 2)
        }
    } else if constexpr (KC == 2) {
        FEDAVG_F64FEW(1, 2, 5, 5)
        if constexpr (kABFew) {
            FEDAVG_F64FEW(1, 2, 5, 1)
            FEDAVG_F64FEW(1, 3, 4, 1)
            FEDAVG_F64FEW(1, 2, 4, 2)
            FEDAVG_F64FEW(2, 2, 2, 1)
        }
    } else {
        FEDAVG_F64FEW(1, 3, 4, 1)
        if constexpr (kABFew) {
            FEDAVG_F64FEW(1, 2, 5, 1)
            FEDAVG_F64FEW(1, 2, 4, 2)
            FEDAVG_F64FEW(2, 2, 2, 1)
            FEDAVG_F64FEW(1, 2, 5, 5)
        }
    }
#undef FEDAVG_F64FEW
    return hipErrorInvalidValue;
}

template <int OP, int FIN>
static hipError_t launch_t64_f(const RowTableGeneric& tab, int K, int64_t ts2, const void* acc_in, void* out, int64_t b2,
                               int64_t e2, double fin_val, int grid, int burst, hipStream_t s, uint64_t* nl) {
    const f64x2* ai = static_cast<const f64x2*>(acc_in);
    f64x2* o = static_cast<f64x2*>(out);
    constexpr int64_t T2 = (int64_t)kCpl64 * kBlock;
    if (burst >= 3) {  // the few-client form (1-3 reads, no chained sum); burst - 3 = its A/B form index (0: default)
        if (acc_in) return hipErrorInvalidValue;
        if (K == 1) return launch_f64_few<OP, FIN, 1>(tab, ts2, o, b2, e2, fin_val, grid, burst - 3, s, nl);
        if (K == 2) return launch_f64_few<OP, FIN, 2>(tab, ts2, o, b2, e2, fin_val, grid, burst - 3, s, nl);
        if (K == 3) return launch_f64_few<OP, FIN, 3>(tab, ts2, o, b2, e2, fin_val, grid, burst - 3, s, nl);
        return hipErrorInvalidValue;
    }
    if (burst == 2 || !kAB) {  // default: kBurstTiles64 in registers + kBurstLdsTiles64 in LDS per block and launch
        return burst_launches(b2 / T2, (e2 - 1) / T2 + 1, grid, kBurstTiles64 + kBurstLdsTiles64, nl, false,
                              [&](int nb, int64_t t0, int64_t t_end, uint32_t) {
            if (acc_in)
                hipLaunchKernelGGL((fedavg_tiles_f64x2_burst<OP, FIN, true, kBurstTiles64, kBurstLdsTiles64>), dim3(nb),
                                   dim3(kBlock), 0, s, tab, K, ts2, ai, o, b2, e2, fin_val, t0, t_end);
            else
                hipLaunchKernelGGL((fedavg_tiles_f64x2_burst<OP, FIN, false, kBurstTiles64, kBurstLdsTiles64>), dim3(nb),
                                   dim3(kBlock), 0, s, tab, K, ts2, ai, o, b2, e2, fin_val, t0, t_end);
        });
    }
    if constexpr (kAB) {  // A/B builds: the register-only burst form (variant bit 5) and the per-tile form (bit 3)
        if (burst) {
            return burst_launches(b2 / T2, (e2 - 1) / T2 + 1, grid, kBurstTiles64, nl, false, [&](int nb, int64_t t0, int64_t t_end, uint32_t) {
                if (acc_in)
                    hipLaunchKernelGGL((fedavg_tiles_f64x2_burst<OP, FIN, true, kBurstTiles64>), dim3(nb), dim3(kBlock), 0, s,
                                       tab, K, ts2, ai, o, b2, e2, fin_val, t0, t_end);
                else
                    hipLaunchKernelGGL((fedavg_tiles_f64x2_burst<OP, FIN, false, kBurstTiles64>), dim3(nb), dim3(kBlock), 0,
                                       s, tab, K, ts2, ai, o, b2, e2, fin_val, t0, t_end);
            });
        }
        if (acc_in) {
            hipLaunchKernelGGL((fedavg_tiles_f64x2<OP, FIN, true>), dim3(grid), dim3(kBlock), 0, s, tab, K, ts2, ai, o, b2, e2,
                               fin_val);
        } else {
            hipLaunchKernelGGL((fedavg_tiles_f64x2<OP, FIN, false>), dim3(grid), dim3(kBlock), 0, s, tab, K, ts2, ai, o, b2,
                               e2, fin_val);
        }
        if (nl) ++*nl;
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int OP>
static hipError_t launch_t64_o(const RowTableGeneric& tab, int K, int64_t ts2, const void* acc_in, void* out, int64_t b2,
                               int64_t e2, int fin, double fin_val, int grid, int burst, hipStream_t s, uint64_t* nl) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_t64_f<OP, FEDAVG_FIN_SCALE>(tab, K, ts2, acc_in, out, b2, e2, fin_val, grid, burst, s, nl);
        case FEDAVG_FIN_DIV:
            return launch_t64_f<OP, FEDAVG_FIN_DIV>(tab, K, ts2, acc_in, out, b2, e2, fin_val, grid, burst, s, nl);
        default:
            return launch_t64_f<OP, FEDAVG_FIN_NONE>(tab, K, ts2, acc_in, out, b2, e2, fin_val, grid, burst, s, nl);
    }
}

hipError_t launch_tiles_f64(const RowTableGeneric& tab, int K, int64_t tstride_elems, const void* acc_in, void* out,
                            int64_t begin, int64_t end, int op, int fin, double fin_val, int grid, int burst,
                            hipStream_t s, uint64_t* nl) {
    const int64_t ts2 = tstride_elems / 2, b2 = begin / 2, e2 = end / 2;
    switch (op) {
        case FEDAVG_OP_TORCH:
            return launch_t64_o<FEDAVG_OP_TORCH>(tab, K, ts2, acc_in, out, b2, e2, fin, fin_val, grid, burst, s, nl);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_t64_o<FEDAVG_OP_UNWEIGHTED>(tab, K, ts2, acc_in, out, b2, e2, fin, fin_val, grid, burst, s, nl);
        default:
            return launch_t64_o<FEDAVG_OP_NUMPY>(tab, K, ts2, acc_in, out, b2, e2, fin, fin_val, grid, burst, s, nl);
    }
}

// ---------------------------------------------------------------------------------------------
// integer / bool totals of numpy arrays with weigh_by_local_iter=False (weighted_aggregation_helper.py:195-199,
// :214-215): first T = v.copy(), step T = T + v in the array's own dtype -- two's-complement wraparound as
// numpy's integer add, logical OR for bool (numpy's add on bool arrays).  The caller finalises the sum as
// float64(T) * (1.0 / count) (:236) with a generic (int -> F64) launch.
// ---------------------------------------------------------------------------------------------
template <typename U, bool IS_BOOL, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_rows_intsum(const RowTableGeneric tab, const int K, const U* acc_in,
                                                              U* out, const int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        U acc;
        int k = 0;
        if constexpr (ACC_IN) {
            acc = acc_in[i];
        } else {
            acc = static_cast<const U*>(tab.rows[0])[i];
            k = 1;
        }
        for (; k < K; ++k) {
            const U v = static_cast<const U*>(tab.rows[k])[i];
            acc = IS_BOOL ? (U)(acc | v) : (U)(acc + v);  // unsigned arithmetic: defined wraparound
        }
        out[i] = acc;
    }
}

template <typename U, bool IS_BOOL>
static hipError_t launch_intsum_t(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int grid,
                                  hipStream_t s) {
    if (acc_in)
        hipLaunchKernelGGL((fedavg_rows_intsum<U, IS_BOOL, true>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const U*>(acc_in), static_cast<U*>(out), n);
    else
        hipLaunchKernelGGL((fedavg_rows_intsum<U, IS_BOOL, false>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const U*>(acc_in), static_cast<U*>(out), n);
    return hipGetLastError();
}

hipError_t launch_rows_intsum(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int dtype,
                              int grid, hipStream_t s) {
    switch (dtype) {
        case FEDAVG_I8:
        case FEDAVG_U8:
            return launch_intsum_t<uint8_t, false>(tab, K, acc_in, out, n, grid, s);
        case FEDAVG_BOOL:
            return launch_intsum_t<uint8_t, true>(tab, K, acc_in, out, n, grid, s);
        case FEDAVG_I16:
        case FEDAVG_U16:
            return launch_intsum_t<uint16_t, false>(tab, K, acc_in, out, n, grid, s);
        case FEDAVG_I32:
        case FEDAVG_U32:
            return launch_intsum_t<uint32_t, false>(tab, K, acc_in, out, n, grid, s);
        case FEDAVG_I64:
        case FEDAVG_U64:
            return launch_intsum_t<uint64_t, false>(tab, K, acc_in, out, n, grid, s);
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t launch_rows_generic(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n,
                               int in_dtype, int acc_dtype, int op, int fin, double fin_val, int grid,
                               hipStream_t s) {
    if (in_dtype == FEDAVG_F64 && acc_dtype == FEDAVG_F64) {
        const hipError_t e = launch_rows_f64x2(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
        if (e != hipErrorNotSupported) return e;
    }
    // integer / bool inputs are promoted to the accumulator type before the first operation, as numpy
    // (-> float64) and torch (-> float32, the default dtype) promote them
    if (acc_dtype == FEDAVG_F32) {
        switch (in_dtype) {
            case FEDAVG_F32:
                return launch_generic_t<float, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_F16:
                return launch_generic_t<_Float16, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I32:
                return launch_generic_t<int32_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I64:
                return launch_generic_t<int64_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_U8:
            case FEDAVG_BOOL:
                return launch_generic_t<uint8_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I8:
                return launch_generic_t<int8_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I16:
                return launch_generic_t<int16_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            default:
                return hipErrorInvalidValue;
        }
    } else if (acc_dtype == FEDAVG_F64) {
        switch (in_dtype) {
            case FEDAVG_F64:
                return launch_generic_t<double, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_F32:
                return launch_generic_t<float, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_F16:
                return launch_generic_t<_Float16, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I32:
                return launch_generic_t<int32_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I64:
                return launch_generic_t<int64_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_U8:
            case FEDAVG_BOOL:
                return launch_generic_t<uint8_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I8:
                return launch_generic_t<int8_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I16:
                return launch_generic_t<int16_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_U16:
                return launch_generic_t<uint16_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_U32:
                return launch_generic_t<uint32_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_U64:
                return launch_generic_t<uint64_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            default:
                return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_fill_synthetic_f32(float* dst, int64_t n, int64_t tile, int64_t tstride, uint64_t seed, uint64_t row,
                                     uint64_t col0, int grid, hipStream_t s) {
    hipLaunchKernelGGL(fedavg_fill_synthetic_f32, dim3(grid), dim3(kBlock), 0, s, dst, n, tile, tstride, seed, row,
                       col0);
    return hipGetLastError();
}

// test kernel: the epilogues' sqrt elementwise (torch_sqrt: FEDAVG_SQRT_* -- torch CPU's restated vsSqrt of the Intel
// or the AMD hosts, or the correctly rounded one; rsqrtps: the host's RSQRTPS table for FEDAVG_SQRT_TORCH_AMD)
__global__ void __launch_bounds__(kBlock) fedavg_sqrt_f32(const float* __restrict__ x, float* __restrict__ out, int64_t n,
                                                          int torch_sqrt, const uint32_t* __restrict__ rsqrtps) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    rsqrt14_stage();
    if (torch_sqrt == FEDAVG_SQRT_TORCH_AMD) rsqrtps_stage(rsqrtps);  // block-uniform: the barrier is safe
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = torch_sqrt == FEDAVG_SQRT_TORCH_AVX512 ? sqrt_torch_cpu(x[i])
                 : torch_sqrt == FEDAVG_SQRT_TORCH_AMD ? sqrt_mkl_rsqrtps(x[i])
                                                        : __builtin_sqrtf(x[i]);
}

hipError_t launch_sqrt_f32(const float* x, float* out, int64_t n, int torch_sqrt, const uint32_t* rsqrtps, int grid,
                           hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fedavg_sqrt_f32, dim3(grid), dim3(kBlock), 0, s, x, out, n, torch_sqrt, rsqrtps);
    return hipGetLastError();
}

hipError_t launch_gather_f32(const float* src, const uint64_t* idx, float* dst, int64_t m, hipStream_t s) {
    const int grid = (int)((m + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(fedavg_gather_f32, dim3(grid), dim3(kBlock), 0, s, src, idx, dst, m);
    return hipGetLastError();
}

}  // namespace fedavg
