// fedavg_tiles.h -- the fp32 tiled aggregation kernels (the hot path) and their launch templates; included by
// one translation unit per arithmetic mode (fedavg_tiles_{numpy,torch,unweighted}.hip) so the instantiations
// compile in parallel.  Design notes: fedavg_kernels.hip header, DESIGN.md section 3.
#pragma once

#include "fedavg_arith.h"

namespace fedavg {

constexpr int kVariantRuntimeK = 128;  // burst kernels: round 3's runtime-K tile loop (tile_sum GROUPED) instead of the
                                       // built-in client count (1-6) or remainder (7+) forms (tile_sum_kc / _rem, round 4)

// ---------------------------------------------------------------------------------------------
// THE HOT KERNEL.  Global f32x4 index range [b4, e4); tiles t = b4/T4 .. (e4-1)/T4 are dealt to blocks
// round-robin.  For every column of a tile:
//     acc = ACC_IN ? acc_in[i] : first(client 0);  acc = step(acc, client k) for k = 1..K-1 in order;
//     out[i] = fin(acc)                  (only for i in [b4, e4): partial edge tiles are masked at store)
// Client loads are unconditional: the caller guarantees every client's tiled storage covers whole
// tiles (slabs are allocated in whole tiles; the pointer-list entry point sends ragged tails elsewhere).
// ---------------------------------------------------------------------------------------------
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL, bool NTL, bool NTS>
__global__ void __launch_bounds__(kBlock) fedavg_tiles_f32x4(const RowTableF32 tab, const int K,
                                                              const int64_t tstride4, const f32x4* acc_in,
                                                              f32x4* out, const int64_t b4, const int64_t e4,
                                                              const float fin_val) {
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    const int64_t t_last = (e4 - 1) / T4;
    const FinConst fc = fin_const<FIN>(fin_val);
    for (int64_t t = b4 / T4 + blockIdx.x; t <= t_last; t += gridDim.x) {
        const int64_t off = t * tstride4 + threadIdx.x;  // offset inside each client's tiled storage
        const int64_t col = t * T4 + threadIdx.x;        // global f32x4 index of column group 0
        f32x4 acc[CPL];
        int k = 0;
        if constexpr (ACC_IN) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = col + c * kBlock;
                acc[c] = (i >= b4 && i < e4) ? load4<false>(acc_in + i) : f32x4{0, 0, 0, 0};
            }
        } else {
            const f32x4* r = tab.rows[0] + off;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(load4<NTL>(r + c * kBlock), tab.w[0]);
            k = 1;
        }
        // groups of UNROLL clients: issue all their loads, then the arrival-ordered arithmetic
        for (; k + UNROLL <= K; k += UNROLL) {
            f32x4 v[UNROLL][CPL];
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                const f32x4* r = tab.rows[k + j] + off;
#pragma unroll
                for (int c = 0; c < CPL; ++c) v[j][c] = load4<NTL>(r + c * kBlock);
            }
#pragma unroll
            for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[k + j]);
        }
        for (; k < K; ++k) {
            const f32x4* r = tab.rows[k] + off;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], load4<NTL>(r + c * kBlock), tab.w[k]);
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            if (i >= b4 && i < e4) store4<NTS>(out + i, fin4c<FIN>(acc[c], fc));
        }
    }
}

// tile_sum with the launch's client count KC known at build time (round 4; fedavg_arith.h tile_sum is the runtime-K
// form): groups of min(KC - g, 4) clients -- exactly the launch's rows, where the runtime form's last group re-loads
// its last client in the missing slots (at K = 2 half of a tile's loads were such repeats) -- and every row pointer
// and weight at a fixed kernarg offset, loaded once per kernel into SGPRs instead of per group and tile.
// SHAPE: -1 (default) -- from 4 clients on the full group's loads as two pairs (fedavg_arith.h client_group4; plain
// burst at 4 / 5 / 6 / 7 clients 71.9 / 73.7 / 73.7 / 77.0 % -> 76.9 / 75.7 / 75.1 / 83.3 %, profiles/r04/s15/, s16/),
// together at 1-3; A/B only: 0 -- four together, 2 -- pairs (3 clients: a pair, then the third).
template <int OP, bool ACC_IN, int KC, int CPL, int SHAPE = -1>
__device__ __forceinline__ void tile_sum_kc(f32x4 (&acc)[CPL], const RowTableF32& tab, const int64_t off, const int64_t col,
                                            const f32x4* acc_in, const int64_t b4, const int64_t e4) {
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            acc[c] = (i >= b4 && i < e4) ? __builtin_nontemporal_load(acc_in + i) : f32x4{0, 0, 0, 0};
        }
    }
#pragma unroll
    for (int g = 0; g < KC; g += 4) {
        if constexpr (SHAPE == 2 || (SHAPE < 0 && KC >= 4)) {
            if (g + 4 <= KC) {
                client_group4<OP, ACC_IN, 2, CPL>(acc, tab, g, off);
                continue;
            }
        }
        if constexpr (SHAPE == 2 && KC == 3) {
            client_group<OP, ACC_IN, 2, CPL>(acc, tab, 0, off);
            fence_on(acc);
            client_group<OP, ACC_IN, 1, CPL>(acc, tab, 2, off);
            continue;
        }
        f32x4 v[4][CPL];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (g + j < KC)
#pragma unroll
                for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(tab.rows[g + j] + off + c * kBlock);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (g + j < KC) {
                const float w = tab.w[g + j];
                if (!ACC_IN && g + j == 0) {
#pragma unroll
                    for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(v[j][c], w);
                } else {
#pragma unroll
                    for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], w);
                }
            }
        }
    }
}

// The runtime-K form with the remainder REM = K mod 4 built in: full groups of 4 clients in a loop, then one group of
// exactly REM clients -- no repeated loads for any K (fedavg_arith.h tile_sum's GROUPED form re-loads the last client
// 4 - K mod 4 times per tile).  SHAPE: how a full group's loads are issued (fedavg_arith.h client_group4).  -1, the
// default: as two pairs, the second pair's loads after the first pair's arithmetic (at 7 clients, one group plus 3:
// 76.5 -> 82.8 %, profiles/r04/s15/).  0: four together (round 4 until session 7); 2-4: the other shapes (A/B,
// launch variant bits 9-11).  Plain
// burst, % of 8 TB/s, four together / round 3's GROUPED loop / pairs, one process each (profiles/r04/s7/plain_k*):
// 64 clients 87.8 / 90.3 / 90.0, 32: 86.9 / 89.0 / 88.2, 16: 80.7 / 84.9 / 84.9, 8: 77.0 / 79.9 / 83.9 -- fewer
// loads in flight per wave (one wave per SIMD) stream better.
template <int OP, bool ACC_IN, int REM, int CPL, int SHAPE = -1>
__device__ __forceinline__ void tile_sum_rem(f32x4 (&acc)[CPL], const RowTableF32& tab, const int K, const int64_t off,
                                             const int64_t col, const f32x4* acc_in, const int64_t b4, const int64_t e4) {
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            acc[c] = (i >= b4 && i < e4) ? __builtin_nontemporal_load(acc_in + i) : f32x4{0, 0, 0, 0};
        }
    }
    const int k_full = K - REM;
    if constexpr (SHAPE > 0) {
        for (int k = 0; k < k_full; k += 4) client_group4<OP, ACC_IN, SHAPE, CPL>(acc, tab, k, off);
    } else if constexpr (SHAPE < 0) {  // the default: pairs (these forms run from 7 clients on)
        for (int k = 0; k < k_full; k += 4) client_group4<OP, ACC_IN, 2, CPL>(acc, tab, k, off);
    } else {
    for (int k = 0; k < k_full; k += 4) {
        f32x4 v[4][CPL];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(tab.rows[k + j] + off + c * kBlock);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float w = tab.w[k + j];
            if (!ACC_IN && k + j == 0) {
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(v[j][c], w);
            } else {
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], w);
            }
        }
    }
    }
    if constexpr (REM > 0) {
        f32x4 v[REM][CPL];
#pragma unroll
        for (int j = 0; j < REM; ++j)
#pragma unroll
            for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(tab.rows[k_full + j] + off + c * kBlock);
#pragma unroll
        for (int j = 0; j < REM; ++j) {
            const float w = tab.w[k_full + j];
            if (!ACC_IN && k_full + j == 0) {
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(v[j][c], w);
            } else {
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], w);
            }
        }
    }
}

// one tile's sum: KC > 0 -- the client count built in (tile_sum_kc); KC = -1 - REM -- the runtime count with its
// remainder mod 4 built in (tile_sum_rem); KC = 0 -- fedavg_arith.h tile_sum's GROUPED form (variant bit 7, for A/Bs)
// SHAPE (remainder forms): -1 -- tile_sum_rem's default; A/B only (launch variant bits 9-11): 1 -- tile_sum's GROUPED
// loop with round 3's repeats; 0, 2-4 -- tile_sum_rem with that shape
template <int OP, bool ACC_IN, int UNROLL, int CPL, int KC, int SHAPE = -1>
__device__ __forceinline__ void tile_sum_any(f32x4 (&acc)[CPL], const RowTableF32& tab, const int K, const int64_t off,
                                             const int64_t col, const f32x4* acc_in, const int64_t b4, const int64_t e4) {
    if constexpr (KC > 0) {
        tile_sum_kc<OP, ACC_IN, KC, CPL, SHAPE>(acc, tab, off, col, acc_in, b4, e4);
    } else if constexpr (KC < 0 && SHAPE == 1) {
        tile_sum<OP, ACC_IN, UNROLL, CPL, 2>(acc, tab, K, off, col, acc_in, b4, e4);
    } else if constexpr (KC < 0) {
        tile_sum_rem<OP, ACC_IN, -1 - KC, CPL, SHAPE>(acc, tab, K, off, col, acc_in, b4, e4);
    } else {
        tile_sum<OP, ACC_IN, UNROLL, CPL, true>(acc, tab, K, off, col, acc_in, b4, e4);
    }
}

// ---------------------------------------------------------------------------------------------
// BURST form of the hot kernel (launch variant bit 5).  Measured on MI355X (profiles/r02/pattern_probe):
// a 1 MiB-chunk read stream reaches 88 % of spec alone, but adding the result stream (1/64 of the bytes,
// 16 KiB per tile, written as each tile finishes) drops it to 74-81 % whatever the store cache policy --
// small writes scattered in time through a read stream are expensive.  Written as chip-wide bursts
// instead (every block holds its results and all blocks store at about the same moment, at the end of a
// short launch whose start re-aligns them) the same stream ran at 88.6 %.  So: each launch gives every
// block TPB tiles (dealt round-robin, so the concurrently-read tiles stay adjacent), the results stay in
// registers (TPB x CPL float4 per lane), and the stores are issued after the block's last tile; the host
// issues one launch per grid x TPB tiles.  One block per CU (one wave per SIMD, registers for the staged
// results and a whole client group's loads in flight).
// ---------------------------------------------------------------------------------------------
// TPB_LDS > 0 (the default; launch variant bit 5 turns it off): TPB_LDS more tiles per block whose results wait in LDS (each lane
// reads back only what it wrote, so no barrier), making each launch (TPB + TPB_LDS) / TPB times longer.
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL, int TPB, int TPB_LDS = 0, int KC = 0, int SHAPE = -1>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
fedavg_tiles_burst_f32x4(const RowTableF32 tab, const int K, const int64_t tstride4, const f32x4* acc_in, f32x4* out,
                         const int64_t b4, const int64_t e4, const float fin_val, const int64_t t0, const int64_t t_end) {
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    const FinConst fc = fin_const<FIN>(fin_val);
    f32x4 res[TPB][CPL];
    __shared__ f32x4 staged[TPB_LDS > 0 ? TPB_LDS * CPL * kBlock : 1];
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f32x4 acc[CPL];
            tile_sum_any<OP, ACC_IN, UNROLL, CPL, KC, SHAPE>(acc, tab, K, t * tstride4 + threadIdx.x, t * T4 + threadIdx.x,
                                                      acc_in, b4, e4);
#pragma unroll
            for (int c = 0; c < CPL; ++c) res[m][c] = fin4c<FIN>(acc[c], fc);
        }
    }
    // the LDS-held tiles in a rolled loop: one more copy of the tile body, not TPB_LDS of them
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f32x4 acc[CPL];
            tile_sum_any<OP, ACC_IN, UNROLL, CPL, KC, SHAPE>(acc, tab, K, t * tstride4 + threadIdx.x, t * T4 + threadIdx.x,
                                                      acc_in, b4, e4);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((m - TPB) * CPL + c) * kBlock + threadIdx.x] = fin4c<FIN>(acc[c], fc);
        }
    }
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                if (i >= b4 && i < e4)
                    __builtin_nontemporal_store(staged[((m - TPB) * CPL + c) * kBlock + threadIdx.x], out + i);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                if (i >= b4 && i < e4) __builtin_nontemporal_store(res[m][c], out + i);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
// one launch per grid x (TPB + TPB_LDS) tiles (fedavg_tiles_burst_f32x4)
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL, int TPB, int TPB_LDS, int KC, int SHAPE = -1>
inline hipError_t launch_burst_kc(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const f32x4* ai = reinterpret_cast<const f32x4*>(L.acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, TPB + TPB_LDS, nl,
                          L.variant & kVariantAnyOrder, [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                              hipExtLaunchKernelGGL(
                                  (fedavg_tiles_burst_f32x4<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, KC, SHAPE>), dim3(nb),
                                  dim3(kBlock), 0, s, nullptr, nullptr, flags, L.tab, L.k, L.tstride4, ai, o, L.b4, L.e4,
                                  L.fin_val, t0, t_end);
                          });
}

// the burst kernel with the launch's client count built in (1-6 clients: every row pointer and weight in SGPRs, every
// load a real client's; from 7 on -- 7 with a chained partial sum, 8 -- both groups' loads are hoisted together past
// 256 VGPRs, one wave per SIMD), or from 7 clients on the runtime count with its remainder mod 4 built in; variant bit
// 7 takes the round-3 runtime form everywhere (A/Bs)
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL, int TPB, int TPB_LDS = 0>
inline hipError_t launch_burst(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    if constexpr (CPL == 4 && UNROLL == 4) {
        if constexpr (OP == FEDAVG_OP_TORCH && FIN == FEDAVG_FIN_DIV && !ACC_IN) {  // A/B: client-loop shapes, K % 4 == 0
            const int shape = (L.variant >> kVariantLoopShift) & 7;
            if (shape == 2 && L.k == 3) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 3, 2>(L, s, nl);
            if (shape == 5 && L.k == 4) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 4, 0>(L, s, nl);
            if (shape == 5 && L.k >= 5 && L.k <= 7) {  // one group plus a remainder, four together (before session 16)
                if (L.k == 5) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 5, 0>(L, s, nl);
                if (L.k == 6) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 6, 0>(L, s, nl);
                return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -4, 0>(L, s, nl);
            }
            if (L.k >= 8 && L.k % 4 == 0) {
                switch ((L.variant >> kVariantLoopShift) & 7) {
                    case 1: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1, 1>(L, s, nl);
                    case 2: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1, 2>(L, s, nl);
                    case 3: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1, 3>(L, s, nl);
                    case 4: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1, 4>(L, s, nl);
                    case 5: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1, 0>(L, s, nl);
                    default: break;
                }
            }
        }
        if (!(L.variant & kVariantRuntimeK)) {
            switch (L.k) {
#define FEDAVG_KC(N) \
    case N:          \
        return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, N>(L, s, nl);
                FEDAVG_KC(1)
                FEDAVG_KC(2)
                FEDAVG_KC(3)
                FEDAVG_KC(4)
                FEDAVG_KC(5)
                FEDAVG_KC(6)
#undef FEDAVG_KC
                default:
                    break;
            }
            switch (L.k % 4) {
                case 1:
                    return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -2>(L, s, nl);
                case 2:
                    return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -3>(L, s, nl);
                case 3:
                    return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -4>(L, s, nl);
                default:
                    return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1>(L, s, nl);
            }
        }
    }
    return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 0>(L, s, nl);
}

template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL>
inline hipError_t launch_tiles_v(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const f32x4* ai = reinterpret_cast<const f32x4*>(L.acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    if constexpr (CPL * (UNROLL + kBurstTiles) <= 64) {  // staged results + a group's loads within 256 VGPRs
        if (!(L.variant & (kVariantTileStores | kVariantTemporalLoads | kVariantTemporalStores))) {
            if constexpr (CPL == 4 && UNROLL == 4) {  // the default geometry only (build time)
                if (L.variant & kVariantWideLds)
                    return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles, kBurstLdsTilesWide>(L, s, nl);
                if (!(L.variant & kVariantRegisterTiles))
                    return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles, kBurstLdsTiles>(L, s, nl);
            }
            return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles>(L, s, nl);
        }
    }
    const bool ntl = !(L.variant & kVariantTemporalLoads);
    const bool nts = !(L.variant & kVariantTemporalStores);
#define FEDAVG_LAUNCH_TILES(NTL, NTS)                                                                                \
    hipLaunchKernelGGL((fedavg_tiles_f32x4<OP, FIN, ACC_IN, UNROLL, CPL, NTL, NTS>), dim3(L.grid), dim3(kBlock), 0, \
                       s, L.tab, L.k, L.tstride4, ai, o, L.b4, L.e4, L.fin_val)
    if (ntl && nts) {
        FEDAVG_LAUNCH_TILES(true, true);
    } else if (ntl) {
        FEDAVG_LAUNCH_TILES(true, false);
    } else if (nts) {
        FEDAVG_LAUNCH_TILES(false, true);
    } else {
        FEDAVG_LAUNCH_TILES(false, false);
    }
#undef FEDAVG_LAUNCH_TILES
    if (nl) ++*nl;
    return hipGetLastError();
}

template <int OP, int FIN, bool ACC_IN>
inline hipError_t launch_tiles_a(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const int64_t cpl = L.tile4 / kBlock;
#define FEDAVG_TILES_CPL(C) \
    return L.unroll == 8 ? launch_tiles_v<OP, FIN, ACC_IN, 8, C>(L, s, nl) : launch_tiles_v<OP, FIN, ACC_IN, 4, C>(L, s, nl);
    switch (cpl) {
        case 1:
            FEDAVG_TILES_CPL(1)
        case 2:
            FEDAVG_TILES_CPL(2)
        case 4:
            FEDAVG_TILES_CPL(4)
        case 8:
            FEDAVG_TILES_CPL(8)
        default:
            return hipErrorInvalidValue;
    }
#undef FEDAVG_TILES_CPL
}

template <int OP, int FIN>
inline hipError_t launch_tiles_f(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    return L.acc_in ? launch_tiles_a<OP, FIN, true>(L, s, nl) : launch_tiles_a<OP, FIN, false>(L, s, nl);
}

template <int OP>
inline hipError_t launch_tiles_o(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    switch (L.fin) {
        case FEDAVG_FIN_SCALE:
            return launch_tiles_f<OP, FEDAVG_FIN_SCALE>(L, s, nl);
        case FEDAVG_FIN_DIV:
            return launch_tiles_f<OP, FEDAVG_FIN_DIV>(L, s, nl);
        default:
            return launch_tiles_f<OP, FEDAVG_FIN_NONE>(L, s, nl);
    }
}

}  // namespace fedavg
