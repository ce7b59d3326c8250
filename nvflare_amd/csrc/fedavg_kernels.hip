// fedavg_kernels.hip -- CDNA4 (gfx950) kernels for the FedAvg weighted accumulate-and-scale.
//
// Reference arithmetic (NVFlare nvflare/app_common/aggregators/weighted_aggregation_helper.py):
//   numpy branch  :188-193 (first T = v*w), :210-214 (T = T + v*w), :236 (T * (1.0/count))
//   torch branch  :181-187 (first T = v.mul(w)), :203-209 (T.add_(v, alpha=w) == one FMA), :233 (T.div_(count))
//   weigh_by_local_iter=False :186-199, :208-215 (T = v; T = T + v)
//
// Design:
//   * One pass over the stacked client rows: every element reads K client values once and writes its
//     result once -- 4*K + 4 bytes per fp32 parameter, no temporaries, HBM-bound (no MFMA: this is
//     elementwise, not a contraction).
//   * The per-element operation sequence is exactly the reference's, in arrival order, so the result
//     is bitwise equal to the reference (not merely within 1 ulp).  This file MUST be compiled with
//     -ffp-contract=off: the numpy mode's multiply and add round separately; the torch mode calls
//     __builtin_fmaf explicitly.  fp32 denormals are preserved (gfx950 default IEEE mode).
//   * Row pointers and fp32 weights travel in the kernel-argument segment: they are wave-uniform, so
//     the compiler keeps them in SGPRs (s_load from kernarg) and every client row is read with a
//     saddr-form global_load_dwordx4 (uniform 64-bit base + per-lane 32-bit offset).
//   * Each lane owns 4 consecutive floats (16 B); a wave reads 1 KiB contiguous per client row; loads
//     of UNROLL consecutive clients are issued before the dependent arithmetic (memory-level
//     parallelism), with nontemporal hints because every byte is read exactly once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fedavg_internal.h"

namespace fedavg {

// ---------------------------------------------------------------------------------------------
// per-element arithmetic
// ---------------------------------------------------------------------------------------------
template <int OP, typename T>
__device__ __forceinline__ T first_op(T v, T w) {
    if constexpr (OP == FEDAVG_OP_UNWEIGHTED) {
        return v;
    } else {
        return v * w;  // one rounding (fp-contract off)
    }
}

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <int OP, typename T>
__device__ __forceinline__ T step_op(T acc, T v, T w) {
    if constexpr (OP == FEDAVG_OP_TORCH) {
        return fma_t(v, w, acc);  // torch CPU add_(v, alpha=w): vec::fmadd, one rounding
    } else if constexpr (OP == FEDAVG_OP_NUMPY) {
        const T p = v * w;  // numpy: tmp = v * w (rounded) ...
        return acc + p;     // ... then total + tmp (rounded)
    } else {
        return acc + v;
    }
}

template <int FIN, typename T>
__device__ __forceinline__ T fin_op(T acc, T s) {
    if constexpr (FIN == FEDAVG_FIN_SCALE) {
        return acc * s;  // numpy: total * (1.0 / count), s = acc_t(1.0 / count)
    } else if constexpr (FIN == FEDAVG_FIN_DIV) {
        return acc / s;  // torch: total.div_(count), correctly rounded IEEE division
    } else {
        return acc;
    }
}

template <int OP>
__device__ __forceinline__ f32x4 first4(f32x4 v, float w) {
    return f32x4{first_op<OP>(v[0], w), first_op<OP>(v[1], w), first_op<OP>(v[2], w), first_op<OP>(v[3], w)};
}
template <int OP>
__device__ __forceinline__ f32x4 step4(f32x4 a, f32x4 v, float w) {
    return f32x4{step_op<OP>(a[0], v[0], w), step_op<OP>(a[1], v[1], w), step_op<OP>(a[2], v[2], w),
                 step_op<OP>(a[3], v[3], w)};
}
template <int FIN>
__device__ __forceinline__ f32x4 fin4(f32x4 a, float s) {
    return f32x4{fin_op<FIN>(a[0], s), fin_op<FIN>(a[1], s), fin_op<FIN>(a[2], s), fin_op<FIN>(a[3], s)};
}

template <bool NT>
__device__ __forceinline__ f32x4 load4(const f32x4* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void store4(f32x4* p, f32x4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 streaming kernel: out[i] = fin( fold_k step(acc, rows[k][i], w[k]) ), f32x4 per lane
//   VEC    float4 columns per lane per tile (tile = VEC * kBlock float4; lane j owns j, j+kBlock, ...)
//   UNROLL rows whose loads are issued before their arrival-ordered arithmetic
//   NT     nontemporal load hint (every client byte is read exactly once)
// ---------------------------------------------------------------------------------------------
template <int OP, int FIN, bool ACC_IN, int UNROLL, bool NT, int VEC, bool NTS = false>
__global__ void __launch_bounds__(kBlock) fedavg_rows_f32x4(const RowTableF32 tab, const int K,
                                                             const f32x4* acc_in, f32x4* out,
                                                             const int64_t n4, const float fin_val) {
    constexpr int64_t kTile = (int64_t)VEC * kBlock;
    const int64_t stride = (int64_t)gridDim.x * kTile;
    for (int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x; base < n4; base += stride) {
        if (VEC == 1 || base + (VEC - 1) * kBlock < n4) {
            f32x4 acc[VEC];
            int k = 0;
            if constexpr (ACC_IN) {
#pragma unroll
                for (int c = 0; c < VEC; ++c) acc[c] = load4<false>(acc_in + base + c * kBlock);
            } else {
#pragma unroll
                for (int c = 0; c < VEC; ++c) acc[c] = first4<OP>(load4<NT>(tab.rows[0] + base + c * kBlock), tab.w[0]);
                k = 1;
            }
            // groups of UNROLL clients: issue all loads, then the arrival-ordered arithmetic
            for (; k + UNROLL <= K; k += UNROLL) {
                f32x4 v[UNROLL][VEC];
#pragma unroll
                for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                    for (int c = 0; c < VEC; ++c) v[j][c] = load4<NT>(tab.rows[k + j] + base + c * kBlock);
#pragma unroll
                for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                    for (int c = 0; c < VEC; ++c) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[k + j]);
            }
            for (; k < K; ++k) {
#pragma unroll
                for (int c = 0; c < VEC; ++c)
                    acc[c] = step4<OP>(acc[c], load4<NT>(tab.rows[k] + base + c * kBlock), tab.w[k]);
            }
#pragma unroll
            for (int c = 0; c < VEC; ++c) store4<NTS>(out + base + c * kBlock, fin4<FIN>(acc[c], fin_val));
        } else {
            // ragged last tile (VEC > 1): column by column
            for (int c = 0; c < VEC; ++c) {
                const int64_t i = base + c * kBlock;
                if (i >= n4) break;
                f32x4 a;
                int k = 0;
                if constexpr (ACC_IN) {
                    a = load4<false>(acc_in + i);
                } else {
                    a = first4<OP>(load4<NT>(tab.rows[0] + i), tab.w[0]);
                    k = 1;
                }
                for (; k < K; ++k) a = step4<OP>(a, load4<NT>(tab.rows[k] + i), tab.w[k]);
                store4<false>(out + i, fin4<FIN>(a, fin_val));
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 tiled-slab kernel: clients interleaved per tile, slab[t][slot][T4] (f32x4 units).  The K rows of
// one tile are contiguous, so a block streams K*T4*16 contiguous bytes per tile.
// ---------------------------------------------------------------------------------------------
template <int OP, int FIN, bool ACC_IN, int UNROLL, bool NT, int CPL, bool NTS = false>
__global__ void __launch_bounds__(kBlock) fedavg_tiled_f32x4(const SlotTableF32 tab, const int K,
                                                              const f32x4* __restrict__ slab, const int64_t seg4,
                                                              const int64_t tstride4, const f32x4* acc_in, f32x4* out,
                                                              const int64_t n4, const float fin_val) {
    constexpr int64_t T4 = (int64_t)CPL * kBlock;  // tile width in f32x4 (CPL columns per lane)
    const int64_t n_tiles = (n4 + T4 - 1) / T4;
    for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const f32x4* tile = slab + t * tstride4;
        const int64_t col0 = t * T4 + threadIdx.x;
        f32x4 acc[CPL];
        int k = 0;
        if constexpr (ACC_IN) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = col0 + c * kBlock;
                acc[c] = i < n4 ? load4<false>(acc_in + i) : f32x4{0, 0, 0, 0};
            }
        } else {
            const f32x4* r = tile + (int64_t)tab.slot[0] * seg4 + threadIdx.x;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(load4<NT>(r + c * kBlock), tab.w[0]);
            k = 1;
        }
        for (; k + UNROLL <= K; k += UNROLL) {
            f32x4 v[UNROLL][CPL];
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                const f32x4* r = tile + (int64_t)tab.slot[k + j] * seg4 + threadIdx.x;
#pragma unroll
                for (int c = 0; c < CPL; ++c) v[j][c] = load4<NT>(r + c * kBlock);
            }
#pragma unroll
            for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[k + j]);
        }
        for (; k < K; ++k) {
            const f32x4* r = tile + (int64_t)tab.slot[k] * seg4 + threadIdx.x;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], load4<NT>(r + c * kBlock), tab.w[k]);
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col0 + c * kBlock;
            if (i < n4) store4<NTS>(out + i, fin4<FIN>(acc[c], fin_val));
        }
    }
}

// Software-pipelined form of the tiled kernel (K % UNROLL == 0): the loads of the next group of UNROLL
// clients -- possibly in the block's next tile -- are issued before the current group's arithmetic, so a
// wave keeps 2 * UNROLL * CPL 16-byte loads in flight instead of draining at every group boundary.
template <int OP, int FIN, bool ACC_IN, int UNROLL, bool NT, int CPL>
__global__ void __launch_bounds__(kBlock) fedavg_tiled_pipe_f32x4(const SlotTableF32 tab, const int K,
                                                                   const f32x4* __restrict__ slab, const int64_t seg4,
                                                                   const int64_t tstride4, const f32x4* acc_in,
                                                                   f32x4* out, const int64_t n4, const float fin_val) {
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    const int64_t n_tiles = (n4 + T4 - 1) / T4;
    const int G = K / UNROLL;  // groups per tile
    int64_t t = blockIdx.x;
    if (t >= n_tiles) return;
    f32x4 bufA[UNROLL][CPL], bufB[UNROLL][CPL];
    auto issue = [&](f32x4 (&b)[UNROLL][CPL], int64_t tt, int g) {
        const f32x4* tile = slab + tt * tstride4 + threadIdx.x;
#pragma unroll
        for (int j = 0; j < UNROLL; ++j) {
            const f32x4* r = tile + (int64_t)tab.slot[g * UNROLL + j] * seg4;
#pragma unroll
            for (int c = 0; c < CPL; ++c) b[j][c] = load4<NT>(r + c * kBlock);
        }
    };
    // consume one group from `cur` after issuing the next group into `nxt`; returns false when done
    f32x4 acc[CPL];
    int g = 0;
    auto stage = [&](f32x4 (&cur)[UNROLL][CPL], f32x4 (&nxt)[UNROLL][CPL]) -> bool {
        int64_t tn = t;
        int gn = g + 1;
        if (gn == G) {
            gn = 0;
            tn = t + gridDim.x;
        }
        const bool more = tn < n_tiles;
        // always issue (the last prefetch re-reads the current tile): a conditional issue would make
        // the compiler's vmcnt bookkeeping fall back to vmcnt(0) at the join and drain the pipeline
        issue(nxt, more ? tn : t, gn);
        if (g == 0) {
            if constexpr (ACC_IN) {
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                    acc[c] = i < n4 ? load4<false>(acc_in + i) : f32x4{0, 0, 0, 0};
                }
#pragma unroll
                for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], cur[j][c], tab.w[j]);
            } else {
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(cur[0][c], tab.w[0]);
#pragma unroll
                for (int j = 1; j < UNROLL; ++j)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], cur[j][c], tab.w[j]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], cur[j][c], tab.w[g * UNROLL + j]);
        }
        if (g == G - 1) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                if (i < n4) store4<false>(out + i, fin4<FIN>(acc[c], fin_val));
            }
        }
        t = tn;
        g = gn;
        return more;
    };
    issue(bufA, t, 0);
    // ping-pong between the two register buffers: no register copies, so no wait on in-flight loads
    while (stage(bufA, bufB) && stage(bufB, bufA)) {
    }
}

// synthetic fill of a tiled slab: element (tile t, slot k, j) = synth(seed, k, col0 + t*T + j)
__global__ void __launch_bounds__(kBlock) fedavg_fill_synthetic_tiled_f32(float* slab, const int64_t k_max,
                                                                           const int64_t tile_elems, const int64_t seg,
                                                                           const int64_t tstride, const int64_t n,
                                                                           const uint64_t seed, const uint64_t col0);

// ---------------------------------------------------------------------------------------------
// generic scalar kernel: any (Tin, Tacc) pair, any alignment (tails, small keys, fp64, ints)
// ---------------------------------------------------------------------------------------------
template <typename Tin, typename Tacc, int OP, int FIN, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_rows_generic(const RowTableGeneric tab, const int K,
                                                               const Tacc* acc_in, Tacc* out, const int64_t n,
                                                               const double fin_val_d) {
    const Tacc fin_val = (Tacc)fin_val_d;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        Tacc acc;
        int k = 0;
        if constexpr (ACC_IN) {
            acc = acc_in[i];
        } else {
            acc = first_op<OP>((Tacc)(static_cast<const Tin*>(tab.rows[0])[i]), (Tacc)tab.w[0]);
            k = 1;
        }
        for (; k < K; ++k) {
            const Tacc v = (Tacc)(static_cast<const Tin*>(tab.rows[k])[i]);
            acc = step_op<OP>(acc, v, (Tacc)tab.w[k]);
        }
        out[i] = fin_op<FIN>(acc, fin_val);
    }
}

// ---------------------------------------------------------------------------------------------
// synthetic inputs (bit-identical host twin: oracle/fedavg_oracle.c oracle_synth_value)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void __launch_bounds__(kBlock) fedavg_fill_synthetic_f32(float* dst, const int64_t n, const uint64_t seed,
                                                                     const uint64_t row, const uint64_t col0) {
    const uint64_t base = (seed * 0x9E3779B97F4A7C15ULL) ^ (row * 0xD1B54A32D192ED03ULL);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t col = col0 + (uint64_t)i;
        int32_t s = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) s += (int32_t)(mix32(base + col * 4ULL + (uint64_t)j) >> 8);
        s -= (int32_t)(1 << 25);
        dst[i] = (float)s * 1.0323827e-07f;
    }
}

__global__ void __launch_bounds__(kBlock) fedavg_fill_synthetic_tiled_f32(float* slab, const int64_t k_max,
                                                                           const int64_t tile_elems, const int64_t seg,
                                                                           const int64_t tstride, const int64_t n,
                                                                           const uint64_t seed, const uint64_t col0) {
    // logical element (row, i) of every slot row k < k_max, i < n_tiles * tile_elems
    const int64_t n_tiles = (n + tile_elems - 1) / tile_elems;
    const int64_t total = n_tiles * k_max * tile_elems;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += stride) {
        const int64_t t = e / (k_max * tile_elems);
        const int64_t rem = e - t * k_max * tile_elems;
        const int64_t row = rem / tile_elems;
        const int64_t j = rem - row * tile_elems;
        const uint64_t col = col0 + (uint64_t)(t * tile_elems + j);
        const uint64_t base = (seed * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)row * 0xD1B54A32D192ED03ULL);
        int32_t s = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) s += (int32_t)(mix32(base + col * 4ULL + (uint64_t)q) >> 8);
        s -= (int32_t)(1 << 25);
        slab[t * tstride + row * seg + j] = (float)s * 1.0323827e-07f;
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
template <int OP, int FIN, bool ACC_IN, int UNROLL, bool NT, int VEC>
static hipError_t launch_f32x4_v(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4,
                                 float fin_val, int grid, int variant, hipStream_t s) {
    if (variant & 8) {
        hipLaunchKernelGGL((fedavg_rows_f32x4<OP, FIN, ACC_IN, UNROLL, NT, VEC, true>), dim3(grid), dim3(kBlock), 0, s,
                           tab, K, reinterpret_cast<const f32x4*>(acc_in), reinterpret_cast<f32x4*>(out), n4, fin_val);
    } else {
        hipLaunchKernelGGL((fedavg_rows_f32x4<OP, FIN, ACC_IN, UNROLL, NT, VEC>), dim3(grid), dim3(kBlock), 0, s, tab,
                           K, reinterpret_cast<const f32x4*>(acc_in), reinterpret_cast<f32x4*>(out), n4, fin_val);
    }
    return hipGetLastError();
}

// variant bit 0: VEC=2 columns per lane; bit 1: plain (temporal) loads instead of nontemporal
template <int OP, int FIN, bool ACC_IN, int UNROLL>
static hipError_t launch_f32x4_u(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4,
                                 float fin_val, int grid, int variant, hipStream_t s) {
    switch (variant & 3) {
        case 1:
            return launch_f32x4_v<OP, FIN, ACC_IN, UNROLL, true, 2>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
        case 2:
            return launch_f32x4_v<OP, FIN, ACC_IN, UNROLL, false, 1>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
        case 3:
            return launch_f32x4_v<OP, FIN, ACC_IN, UNROLL, false, 2>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
        default:
            return launch_f32x4_v<OP, FIN, ACC_IN, UNROLL, true, 1>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
    }
}

template <int OP, int FIN, bool ACC_IN>
static hipError_t launch_f32x4_a(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4,
                                 float fin_val, int grid, int unroll, int variant, hipStream_t s) {
    switch (unroll) {
        case 4:
            return launch_f32x4_u<OP, FIN, ACC_IN, 4>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
        case 16:
            return launch_f32x4_u<OP, FIN, ACC_IN, 16>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
        default:
            return launch_f32x4_u<OP, FIN, ACC_IN, 8>(tab, K, acc_in, out, n4, fin_val, grid, variant, s);
    }
}

template <int OP, int FIN>
static hipError_t launch_f32x4_f(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4,
                                 float fin_val, int grid, int unroll, int variant, hipStream_t s) {
    if (acc_in) return launch_f32x4_a<OP, FIN, true>(tab, K, acc_in, out, n4, fin_val, grid, unroll, variant, s);
    return launch_f32x4_a<OP, FIN, false>(tab, K, acc_in, out, n4, fin_val, grid, unroll, variant, s);
}

template <int OP>
static hipError_t launch_f32x4_o(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4, int fin,
                                 float fin_val, int grid, int unroll, int variant, hipStream_t s) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_f32x4_f<OP, FEDAVG_FIN_SCALE>(tab, K, acc_in, out, n4, fin_val, grid, unroll, variant, s);
        case FEDAVG_FIN_DIV:
            return launch_f32x4_f<OP, FEDAVG_FIN_DIV>(tab, K, acc_in, out, n4, fin_val, grid, unroll, variant, s);
        default:
            return launch_f32x4_f<OP, FEDAVG_FIN_NONE>(tab, K, acc_in, out, n4, fin_val, grid, unroll, variant, s);
    }
}

hipError_t launch_rows_f32x4(const RowTableF32& tab, int K, const float* acc_in, float* out, int64_t n4, int op,
                             int fin, float fin_val, int grid, int unroll, int variant, hipStream_t s) {
    switch (op) {
        case FEDAVG_OP_TORCH:
            return launch_f32x4_o<FEDAVG_OP_TORCH>(tab, K, acc_in, out, n4, fin, fin_val, grid, unroll, variant, s);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_f32x4_o<FEDAVG_OP_UNWEIGHTED>(tab, K, acc_in, out, n4, fin, fin_val, grid, unroll, variant, s);
        default:
            return launch_f32x4_o<FEDAVG_OP_NUMPY>(tab, K, acc_in, out, n4, fin, fin_val, grid, unroll, variant, s);
    }
}

template <typename Tin, typename Tacc, int OP, int FIN>
static hipError_t launch_generic_f(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n,
                                   double fin_val, int grid, hipStream_t s) {
    if (acc_in) {
        hipLaunchKernelGGL((fedavg_rows_generic<Tin, Tacc, OP, FIN, true>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const Tacc*>(acc_in), static_cast<Tacc*>(out), n, fin_val);
    } else {
        hipLaunchKernelGGL((fedavg_rows_generic<Tin, Tacc, OP, FIN, false>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const Tacc*>(acc_in), static_cast<Tacc*>(out), n, fin_val);
    }
    return hipGetLastError();
}

template <typename Tin, typename Tacc, int OP>
static hipError_t launch_generic_o(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int fin,
                                   double fin_val, int grid, hipStream_t s) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_generic_f<Tin, Tacc, OP, FEDAVG_FIN_SCALE>(tab, K, acc_in, out, n, fin_val, grid, s);
        case FEDAVG_FIN_DIV:
            return launch_generic_f<Tin, Tacc, OP, FEDAVG_FIN_DIV>(tab, K, acc_in, out, n, fin_val, grid, s);
        default:
            return launch_generic_f<Tin, Tacc, OP, FEDAVG_FIN_NONE>(tab, K, acc_in, out, n, fin_val, grid, s);
    }
}

template <typename Tin, typename Tacc>
static hipError_t launch_generic_t(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int op,
                                   int fin, double fin_val, int grid, hipStream_t s) {
    switch (op) {
        case FEDAVG_OP_TORCH:
            return launch_generic_o<Tin, Tacc, FEDAVG_OP_TORCH>(tab, K, acc_in, out, n, fin, fin_val, grid, s);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_generic_o<Tin, Tacc, FEDAVG_OP_UNWEIGHTED>(tab, K, acc_in, out, n, fin, fin_val, grid, s);
        default:
            return launch_generic_o<Tin, Tacc, FEDAVG_OP_NUMPY>(tab, K, acc_in, out, n, fin, fin_val, grid, s);
    }
}

hipError_t launch_rows_generic(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n,
                               int in_dtype, int acc_dtype, int op, int fin, double fin_val, int grid,
                               hipStream_t s) {
    if (acc_dtype == FEDAVG_F32) {
        switch (in_dtype) {
            case FEDAVG_F32:
                return launch_generic_t<float, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I32:
                return launch_generic_t<int32_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I64:
                return launch_generic_t<int64_t, float>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            default:
                return hipErrorInvalidValue;
        }
    } else if (acc_dtype == FEDAVG_F64) {
        switch (in_dtype) {
            case FEDAVG_F64:
                return launch_generic_t<double, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_F32:
                return launch_generic_t<float, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I32:
                return launch_generic_t<int32_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            case FEDAVG_I64:
                return launch_generic_t<int64_t, double>(tab, K, acc_in, out, n, op, fin, fin_val, grid, s);
            default:
                return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_fill_synthetic_f32(float* dst, int64_t n, uint64_t seed, uint64_t row, uint64_t col0, int grid,
                                     hipStream_t s) {
    hipLaunchKernelGGL(fedavg_fill_synthetic_f32, dim3(grid), dim3(kBlock), 0, s, dst, n, seed, row, col0);
    return hipGetLastError();
}

hipError_t launch_gather_f32(const float* src, const uint64_t* idx, float* dst, int64_t m, hipStream_t s) {
    const int grid = (int)((m + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(fedavg_gather_f32, dim3(grid), dim3(kBlock), 0, s, src, idx, dst, m);
    return hipGetLastError();
}

template <int OP, int FIN, bool ACC_IN, int CPL, int UNROLL>
static hipError_t launch_tiled_u(const SlotTableF32& tab, int K, const float* slab, int64_t seg4, int64_t tstride4,
                                 const float* acc_in, float* out, int64_t n4, float fin_val, int grid, int variant,
                                 hipStream_t s) {
    const f32x4* sl = reinterpret_cast<const f32x4*>(slab);
    const f32x4* ai = reinterpret_cast<const f32x4*>(acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(out);
    if ((variant & 4) && K >= UNROLL && K % UNROLL == 0) {
        if (variant & 2) {
            hipLaunchKernelGGL((fedavg_tiled_pipe_f32x4<OP, FIN, ACC_IN, UNROLL, false, CPL>), dim3(grid), dim3(kBlock),
                               0, s, tab, K, sl, seg4, tstride4, ai, o, n4, fin_val);
        } else {
            hipLaunchKernelGGL((fedavg_tiled_pipe_f32x4<OP, FIN, ACC_IN, UNROLL, true, CPL>), dim3(grid), dim3(kBlock),
                               0, s, tab, K, sl, seg4, tstride4, ai, o, n4, fin_val);
        }
    } else if (variant & 8) {
        hipLaunchKernelGGL((fedavg_tiled_f32x4<OP, FIN, ACC_IN, UNROLL, true, CPL, true>), dim3(grid), dim3(kBlock), 0,
                           s, tab, K, sl, seg4, tstride4, ai, o, n4, fin_val);
    } else if (variant & 2) {
        hipLaunchKernelGGL((fedavg_tiled_f32x4<OP, FIN, ACC_IN, UNROLL, false, CPL>), dim3(grid), dim3(kBlock), 0, s,
                           tab, K, sl, seg4, tstride4, ai, o, n4, fin_val);
    } else {
        hipLaunchKernelGGL((fedavg_tiled_f32x4<OP, FIN, ACC_IN, UNROLL, true, CPL>), dim3(grid), dim3(kBlock), 0, s,
                           tab, K, sl, seg4, tstride4, ai, o, n4, fin_val);
    }
    return hipGetLastError();
}

template <int OP, int FIN, bool ACC_IN, int CPL>
static hipError_t launch_tiled_c(const SlotTableF32& tab, int K, const float* slab, int64_t seg4, int64_t tstride4,
                                 const float* acc_in, float* out, int64_t n4, float fin_val, int grid, int unroll,
                                 int variant, hipStream_t s) {
    if (unroll == 4)
        return launch_tiled_u<OP, FIN, ACC_IN, CPL, 4>(tab, K, slab, seg4, tstride4, acc_in, out, n4, fin_val, grid,
                                                       variant, s);
    return launch_tiled_u<OP, FIN, ACC_IN, CPL, 8>(tab, K, slab, seg4, tstride4, acc_in, out, n4, fin_val, grid,
                                                   variant, s);
}

template <int OP, int FIN>
static hipError_t launch_tiled_f(const SlotTableF32& tab, int K, const float* slab, int64_t seg4, int64_t tstride4,
                                 int64_t tile4,
                                 const float* acc_in, float* out, int64_t n4, float fin_val, int grid, int unroll,
                                 int variant, hipStream_t s) {
#define FEDAVG_TILED_CPL(C)                                                                                        \
    return acc_in ? launch_tiled_c<OP, FIN, true, C>(tab, K, slab, seg4, tstride4, acc_in, out, n4, fin_val, grid, unroll,  \
                                                     variant, s)                                                   \
                  : launch_tiled_c<OP, FIN, false, C>(tab, K, slab, seg4, tstride4, acc_in, out, n4, fin_val, grid, unroll, \
                                                      variant, s);
    switch (tile4 / kBlock) {
        case 1:
            FEDAVG_TILED_CPL(1)
        case 2:
            FEDAVG_TILED_CPL(2)
        case 4:
            FEDAVG_TILED_CPL(4)
        case 8:
            FEDAVG_TILED_CPL(8)
        default:
            return hipErrorInvalidValue;
    }
#undef FEDAVG_TILED_CPL
}

hipError_t launch_tiled_f32x4(const SlotTableF32& tab, int K, const float* slab, int64_t seg4, int64_t tstride4,
                              int64_t tile4,
                              const float* acc_in, float* out, int64_t n4, int op, int fin, float fin_val, int grid,
                              int unroll, int variant, hipStream_t s) {
#define FEDAVG_TILED_FIN(OPV)                                                                                   \
    switch (fin) {                                                                                              \
        case FEDAVG_FIN_SCALE:                                                                                  \
            return launch_tiled_f<OPV, FEDAVG_FIN_SCALE>(tab, K, slab, seg4, tstride4, tile4, acc_in, out, n4, fin_val, grid, \
                                                         unroll, variant, s);                                           \
        case FEDAVG_FIN_DIV:                                                                                    \
            return launch_tiled_f<OPV, FEDAVG_FIN_DIV>(tab, K, slab, seg4, tstride4, tile4, acc_in, out, n4, fin_val, grid,   \
                                                       unroll, variant, s);                                             \
        default:                                                                                                \
            return launch_tiled_f<OPV, FEDAVG_FIN_NONE>(tab, K, slab, seg4, tstride4, tile4, acc_in, out, n4, fin_val, grid,  \
                                                        unroll, variant, s);                                            \
    }
    switch (op) {
        case FEDAVG_OP_TORCH:
            FEDAVG_TILED_FIN(FEDAVG_OP_TORCH)
        case FEDAVG_OP_UNWEIGHTED:
            FEDAVG_TILED_FIN(FEDAVG_OP_UNWEIGHTED)
        default:
            FEDAVG_TILED_FIN(FEDAVG_OP_NUMPY)
    }
#undef FEDAVG_TILED_FIN
}

hipError_t launch_fill_synthetic_tiled_f32(float* slab, int64_t k_max, int64_t tile_elems, int64_t seg, int64_t tstride,
                                           int64_t n, uint64_t seed, uint64_t col0, int grid, hipStream_t s) {
    hipLaunchKernelGGL(fedavg_fill_synthetic_tiled_f32, dim3(grid), dim3(kBlock), 0, s, slab, k_max, tile_elems, seg,
                       tstride, n, seed, col0);
    return hipGetLastError();
}

}  // namespace fedavg
