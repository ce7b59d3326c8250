// fedavg_tiles.h -- the fp32 tiled aggregation kernels (the hot path) and their launch templates; included by
// one translation unit per arithmetic mode (fedavg_tiles_{numpy,torch,unweighted}.hip) so the instantiations
// compile in parallel.  Design notes: fedavg_kernels.hip header, DESIGN.md section 3.
#pragma once

#include "fedavg_arith.h"

namespace fedavg {

constexpr int kVariantRuntimeK = 128;  // A/B: burst kernels on round 3's runtime-K tile loop (tile_sum GROUPED = 2, the
                                       // last group re-loading its last client) instead of the built-in client count
                                       // (3-6) or remainder (7+) forms (tile_sum_kc / _rem, round 4)

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
        f32x4 r[CPL];
        fin_tile<FIN, CPL>(r, acc, fc);
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            if (i >= b4 && i < e4) store4<NTS>(out + i, r[c]);
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
// remainder mod 4 built in (tile_sum_rem); KC = 0 -- fedavg_arith.h tile_sum's GROUPED = 2 form, round 3's loop with
// its repeated loads (A/B builds only: variant bit 7, and every launch of a non-default tile width or unroll)
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
    } else {  // A/B builds: round 3's loop (variant bit 7, and the non-default tile widths and unrolls)
        tile_sum<OP, ACC_IN, UNROLL, CPL, 2>(acc, tab, K, off, col, acc_in, b4, e4);
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
            fin_tile<FIN, CPL>(res[m], acc, fc);
        }
    }
    // the LDS-held tiles in a rolled loop: one more copy of the tile body, not TPB_LDS of them
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f32x4 acc[CPL], r[CPL];
            tile_sum_any<OP, ACC_IN, UNROLL, CPL, KC, SHAPE>(acc, tab, K, t * tstride4 + threadIdx.x, t * T4 + threadIdx.x,
                                                      acc_in, b4, e4);
            fin_tile<FIN, CPL>(r, acc, fc);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((m - TPB) * CPL + c) * kBlock + threadIdx.x] = r[c];
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
// FEW-CLIENT burst form (round 5): launches with 1 or 2 row reads and no chained sum.  With one or
// two reads per result the burst kernel above spends its launch in round trips: each register-held tile's loads sit
// behind a guard (`t < t_end`) and the finalisation's rare-case branches, basic-block boundaries the scheduler does
// not hoist loads across, so a wave has one tile's 4-8 KiB in flight where HBM wants ~64 KiB per CU.  Here every load
// is unconditional (a slot past the launch's last tile re-reads that tile; only real tiles are stored), the
// finalisation has one rare-case branch per tile (fin_tile), and the R register-held tiles' loads all go out first:
//   1. R tiles' loads (KC x 4 float4 per lane each) issued together -- in flight while step 2 runs;
//   2. the L LDS-held tiles in groups of G (a group's loads together), summed, finalised, written to LDS;
//   3. the R register-held tiles summed and finalised;
//   4. every result stored: the LDS-held tiles', then the register-held tiles' -- the launch's write burst.
// Per-element sequence as tile_sum_kc's (first4, then step4 for client 1), so the bits are the burst kernel's.
// ---------------------------------------------------------------------------------------------
// P = 2 (the 1-read default since session 20): a unit is a pair of consecutive tiles, K x 32 KiB of contiguous slab;
// the pair's second tile past the range's last tile re-reads that tile (never stored).
template <int OP, int FIN, int KC, int R, int L, int G, int P = 1>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 2)))
fedavg_tiles_few_f32x4(const RowTableF32 tab, const int64_t tstride4, f32x4* out, const int64_t b4, const int64_t e4,
                       const float fin_val, const int64_t t0, const int64_t t_end) {
    static_assert(KC >= 1 && KC <= 4, "one to four row reads (3-4: A/B builds only)");
    static_assert(L % G == 0 || L == 0, "whole LDS groups");
    static_assert(P == 1 || P == 2, "single tiles or pairs");
    constexpr int CPT = 4;  // float4 columns per lane per tile
    constexpr int CPL = CPT * P;
    constexpr int64_t T4 = (int64_t)CPL * kBlock;  // float4 per unit
    const int64_t last_tile = (e4 - 1) / ((int64_t)CPT * kBlock);
    // a pair unit starting before begin's tile (begin's tile index odd) re-reads begin's tile instead of the one before
    // it: the C-ABI only requires storage for the tiles [begin, end) touches
    const int64_t first_tile = b4 / ((int64_t)CPT * kBlock);
    const FinConst fc = fin_const<FIN>(fin_val);
    __shared__ f32x4 staged[L > 0 ? L * CPL * kBlock : 1];
    const int64_t t_first = t0 + blockIdx.x;
    auto tile_of = [&](const int m) __attribute__((always_inline)) {
        const int64_t t = t_first + (int64_t)m * gridDim.x;
        return t < t_end ? t : t_end - 1;  // unconditional loads: a slot past the end re-reads the last tile
    };
    auto sum = [&](f32x4 (&acc)[CPL], const f32x4 (&v)[KC][CPL]) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            acc[c] = first4<OP>(v[0][c], tab.w[0]);
#pragma unroll
            for (int j = 1; j < KC; ++j) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[j]);
        }
    };
    auto load_unit = [&](f32x4 (&v)[KC][CPL], const int m) __attribute__((always_inline)) {
        const int64_t u = tile_of(m);
#pragma unroll
        for (int h = 0; h < P; ++h) {
            int64_t tile = u * P + h;
            tile = tile <= last_tile ? tile : last_tile;
            tile = tile >= first_tile ? tile : first_tile;
            const int64_t off = tile * tstride4 + threadIdx.x;
#pragma unroll
            for (int j = 0; j < KC; ++j)
#pragma unroll
                for (int c = 0; c < CPT; ++c)
                    v[j][h * CPT + c] = __builtin_nontemporal_load(tab.rows[j] + off + c * kBlock);
        }
    };
    // 1. the register-held tiles' loads
    f32x4 vr[R][KC][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) load_unit(vr[m], L + m);
    // 2. the LDS-held tiles (slots 0 .. L-1), G at a time
#pragma unroll
    for (int g = 0; g < L; g += G) {
        f32x4 v[G][KC][CPL];
#pragma unroll
        for (int m = 0; m < G; ++m) load_unit(v[m], g + m);
#pragma unroll
        for (int m = 0; m < G; ++m) {
            f32x4 acc[CPL], r[CPL];
            sum(acc, v[m]);
            fin_tile<FIN, CPL>(r, acc, fc);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((g + m) * CPL + c) * kBlock + threadIdx.x] = r[c];
        }
    }
    // 3. the register-held tiles (slots L .. L+R-1)
    f32x4 res[R][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) {
        f32x4 acc[CPL];
        sum(acc, vr[m]);
        fin_tile<FIN, CPL>(res[m], acc, fc);
    }
    // 4. the write burst
#pragma unroll
    for (int m = 0; m < L + R; ++m) {
        const int64_t t = t_first + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                const f32x4 r = m < L ? staged[(m * CPL + c) * kBlock + threadIdx.x] : res[m < L ? 0 : m - L][c];
                if (i >= b4 && i < e4) __builtin_nontemporal_store(r, out + i);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
template <int OP, int FIN, int KC, int R, int L, int G, int P = 1>
inline hipError_t launch_few_form(const TileLaunch& L_, hipStream_t s, uint64_t* nl) {
    f32x4* o = reinterpret_cast<f32x4*>(L_.out);
    const int64_t u4 = L_.tile4 * P;
    return burst_launches(L_.b4 / u4, (L_.e4 - 1) / u4 + 1, L_.grid, R + L, nl,
                          L_.variant & kVariantAnyOrder, [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                              hipExtLaunchKernelGGL((fedavg_tiles_few_f32x4<OP, FIN, KC, R, L, G, P>), dim3(nb),
                                                    dim3(kBlock), 0, s, nullptr, nullptr, flags, L_.tab, L_.tstride4, o,
                                                    L_.b4, L_.e4, L_.fin_val, t0, t_end);
                          });
}

// the few-client burst kernel (1-2 client reads, no chained sum): the host sets L.grid from few_form().bpc
template <int OP, int FIN, int KC>
inline hipError_t launch_few(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const FewForm f = few_form(KC, L.variant);
#define FEDAVG_FEW(R, LL, G)                                                       \
    if (f.r == R && f.l == LL && f.g == G && f.p <= 1) return launch_few_form<OP, FIN, KC, R, LL, G>(L, s, nl);
#define FEDAVG_FEW2(R, LL, G)                                                      \
    if (f.r == R && f.l == LL && f.g == G && f.p == 2) return launch_few_form<OP, FIN, KC, R, LL, G, 2>(L, s, nl);
    if constexpr (KC == 1) {
        FEDAVG_FEW2(4, 2, 2)
        if constexpr (kABFew) {
            FEDAVG_FEW(8, 4, 2)
            FEDAVG_FEW(12, 10, 2)
            FEDAVG_FEW(8, 10, 1)
            FEDAVG_FEW(10, 4, 2)
            FEDAVG_FEW2(4, 2, 1)
            FEDAVG_FEW2(3, 2, 2)
        }
    } else if constexpr (KC == 2) {
        FEDAVG_FEW(4, 10, 1)
        if constexpr (kABFew) {
            FEDAVG_FEW(6, 10, 1)
            FEDAVG_FEW(5, 10, 1)
            FEDAVG_FEW(4, 9, 1)
            FEDAVG_FEW2(2, 5, 1)
            FEDAVG_FEW2(2, 2, 1)
        }
    } else if constexpr (KC == 3) {
        FEDAVG_FEW(4, 10, 1)
        if constexpr (kABFew) {
            FEDAVG_FEW(2, 10, 1)
            FEDAVG_FEW(3, 10, 1)
            FEDAVG_FEW2(2, 5, 1)
            FEDAVG_FEW2(1, 5, 1)
        }
    } else if constexpr (kABFew && KC == 4) {
        FEDAVG_FEW(2, 10, 1)
        FEDAVG_FEW(3, 10, 1)
        FEDAVG_FEW(1, 10, 1)
        FEDAVG_FEW(2, 4, 1)
        FEDAVG_FEW(2, 8, 1)
        FEDAVG_FEW(2, 10, 2)
    }
#undef FEDAVG_FEW
#undef FEDAVG_FEW2
    return hipErrorInvalidValue;
}
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

// The burst kernel's client loop per launch: the client count built in for 3-6 clients (tile_sum_kc: every row pointer
// and weight in SGPRs, every load a real client's), from 7 on the runtime count with its remainder mod 4 built in
// (tile_sum_rem; 7 with a chained partial sum and 8 built in would hoist both groups' 32 loads past 256 VGPRs at one wave
// per SIMD).  The built-in counts are instantiated only where the router sends them -- no chained sum, two blocks per
// CU (fewer than kBurstOneBlockMinK clients); a chained sum or a one-block-per-CU grid takes the remainder forms, which
// run the same per-element sequence.  A/B builds (kAB) add the built-in 1-2 client forms (public variant bit 8), the
// round-3 runtime loop (bit 7: tile_sum's GROUPED form with its repeated loads) and the loop shapes (bits 9-11).
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL, int TPB, int TPB_LDS = 0>
inline hipError_t launch_burst(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    if constexpr (CPL == 4 && UNROLL == 4) {
        if constexpr (kAB && OP == FEDAVG_OP_TORCH && FIN == FEDAVG_FIN_DIV && !ACC_IN) {  // A/B: client-loop shapes
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
        if constexpr (kAB) {
            if (L.variant & kVariantRuntimeK) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 0>(L, s, nl);
        }
        // A/B: bits 9-11 = 7 -- 3-6 clients on the remainder forms, 6 -- on a built-in count (1-2 with bit 8)
        if constexpr (kABFew) {
            if (((L.variant >> kVariantLoopShift) & 7) == 6 && L.k >= 3 && L.k <= 6) {
                switch (L.k) {
                    case 3: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 3>(L, s, nl);
                    case 4: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 4>(L, s, nl);
                    case 5: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 5>(L, s, nl);
                    default: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 6>(L, s, nl);
                }
            }
            if (((L.variant >> kVariantLoopShift) & 7) == 7) {
                switch (L.k % 4) {
                    case 1: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -2>(L, s, nl);
                    case 2: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -3>(L, s, nl);
                    case 3: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -4>(L, s, nl);
                    default: return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, -1>(L, s, nl);
                }
            }
        }
        // the product's built-in count: 5 clients only (session 6, profiles/r05/s6/rem_k*.jsonl, 1e9, % of 8 TB/s: 5
        // clients 79.8 built in against 76.6 on the remainder form; 6 clients 76.7 against 84.3, 4: 74.8 against 76.2
        // -- those take the remainder forms; 3 clients take the few-client kernel, fedavg_capi.cpp run_tiles)
        if constexpr (kAB || (!ACC_IN && TPB_LDS != kBurstLdsTilesWide)) {
            switch (L.k) {
#define FEDAVG_KC(N) \
    case N:          \
        return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, N>(L, s, nl);
                FEDAVG_KC(5)
                default:
                    break;
            }
            if constexpr (kAB) {
                switch (L.k) {
                    FEDAVG_KC(1)
                    FEDAVG_KC(2)
                    default:
                        break;
                }
            }
#undef FEDAVG_KC
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
    if constexpr (kAB) return launch_burst_kc<OP, FIN, ACC_IN, UNROLL, CPL, TPB, TPB_LDS, 0>(L, s, nl);
    return hipErrorInvalidValue;  // product builds: the default geometry only (launch_tiles_a)
}

// the per-tile-store kernel (each tile's results stored as it finishes) or the burst kernel; product builds carry the
// default geometry's nontemporal per-tile form and the burst forms with LDS-held tiles (4 on two-block grids, 10 on
// one-block grids)
template <int OP, int FIN, bool ACC_IN, int UNROLL, int CPL>
inline hipError_t launch_tiles_v(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const f32x4* ai = reinterpret_cast<const f32x4*>(L.acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    if (L.variant & kVariantFew) {  // 1-2 client reads, no chained sum (fedavg_capi.cpp run_tiles); A/B: 3-4 too
        if constexpr (!ACC_IN && CPL == 4 && UNROLL == 4) {
            if (L.k == 1) return launch_few<OP, FIN, 1>(L, s, nl);
            if (L.k == 2) return launch_few<OP, FIN, 2>(L, s, nl);
            if (L.k == 3) return launch_few<OP, FIN, 3>(L, s, nl);
            if constexpr (kABFew) {
                if (L.k == 4) return launch_few<OP, FIN, 4>(L, s, nl);
            }
        }
        return hipErrorInvalidValue;
    }
    if constexpr (CPL * (UNROLL + kBurstTiles) <= 64) {  // staged results + a group's loads within 256 VGPRs
        if (!(L.variant & (kVariantTileStores | kVariantTemporalLoads | kVariantTemporalStores))) {
            if constexpr (CPL == 4 && UNROLL == 4) {  // the default geometry only (build time)
                if (L.variant & kVariantWideLds)
                    return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles, kBurstLdsTilesWide>(L, s, nl);
                if (!kAB || !(L.variant & kVariantRegisterTiles))
                    return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles, kBurstLdsTiles>(L, s, nl);
            }
            if constexpr (kAB) return launch_burst<OP, FIN, ACC_IN, UNROLL, CPL, kBurstTiles>(L, s, nl);
        }
    }
    const bool ntl = !(L.variant & kVariantTemporalLoads);
    const bool nts = !(L.variant & kVariantTemporalStores);
#define FEDAVG_LAUNCH_TILES(NTL, NTS)                                                                                \
    hipLaunchKernelGGL((fedavg_tiles_f32x4<OP, FIN, ACC_IN, UNROLL, CPL, NTL, NTS>), dim3(L.grid), dim3(kBlock), 0, \
                       s, L.tab, L.k, L.tstride4, ai, o, L.b4, L.e4, L.fin_val)
    if (!kAB || (ntl && nts)) {
        FEDAVG_LAUNCH_TILES(true, true);
    } else if constexpr (kAB) {
        if (ntl) {
            FEDAVG_LAUNCH_TILES(true, false);
        } else if (nts) {
            FEDAVG_LAUNCH_TILES(false, true);
        } else {
            FEDAVG_LAUNCH_TILES(false, false);
        }
    }
#undef FEDAVG_LAUNCH_TILES
    if (nl) ++*nl;
    return hipGetLastError();
}

template <int OP, int FIN, bool ACC_IN>
inline hipError_t launch_tiles_a(const TileLaunch& L, hipStream_t s, uint64_t* nl) {
    const int64_t cpl = L.tile4 / kBlock;
    if constexpr (!kAB) {  // product builds: the default tile (4096 elements) and unroll only (fedavg_set_tile / _launch)
        if (cpl != 4 || L.unroll != 4) return hipErrorInvalidValue;
        return launch_tiles_v<OP, FIN, ACC_IN, 4, 4>(L, s, nl);
    } else {
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
