// fedavg_narrow.hip -- weighted FedAvg over float16 / bfloat16 client values with a 16-bit running sum.
//
// Reference: weighted_aggregation_helper.py:181-236 when the client arrays are float16 (numpy) or
// float16 / bfloat16 tensors (torch): the total keeps the input's 16-bit dtype and every library
// operation rounds to it.  The library sequence, restated per element:
//
//   numpy float16 (NEP 50: the python weight becomes half(w), computed on the host from fp64):
//       first  T = h(v * w)                   numpy half loops compute in fp32 and round once
//       step   T = h(T + h(v * w))            (:210-214, two library operations)
//       SCALE  T = h(T * half(1.0 / count))   (:236)
//   torch CPU float16 / bfloat16 (vectorised kernels, fp32 "opmath"):
//       first  T = r(v * float(w))            mul with a CPU scalar keeps the scalar as float
//       step   T = r(fma(v, r(w), T))         add_(v, alpha=w): alpha cast to the tensor dtype, vec::fmadd
//       DIV    T = r(T / float(count))        div_ with a CPU scalar, fp32 division
//   weigh_by_local_iter=False: first T = v, step T = r(T + v).
//
// The running value lives in an fp32 register but always holds a representable 16-bit value, so partial
// sums chain through 16-bit acc_in / out buffers without changing a bit.  Bytes per element: 2K + 2;
// HBM-bound like the fp32 kernel.  Each lane handles 8 consecutive elements with 16-byte loads when every
// pointer is 16-byte aligned; the remainder and unaligned rows take the per-element loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fedavg_arith.h"  // FinConst / div_const_fast (the few-client form's FIN_DIV)
#include "fedavg_internal.h"

namespace fedavg {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int FMT>
__device__ __forceinline__ float load16(uint16_t b) {
    if constexpr (FMT == FEDAVG_BF16) {
        return __uint_as_float((uint32_t)b << 16);
    } else {
        _Float16 h;
        __builtin_memcpy(&h, &b, 2);
        return (float)h;
    }
}

template <int FMT>
__device__ __forceinline__ uint16_t bits16(float x) {
    if constexpr (FMT == FEDAVG_BF16) {
        // c10::BFloat16 round_to_nearest_even (add the rounding bias, truncate; NaN -> a quiet NaN) is what
        // gfx950's v_cvt_pk_bf16_f32 does in one instruction: equal bits for every non-NaN fp32 input,
        // denormals included (exhaustive check over all 2^32 inputs: tools/bf16_cvt_probe.hip).
        asm volatile("" : "+v"(x));
        const __bf16 h = (__bf16)x;
        uint16_t b;
        __builtin_memcpy(&b, &h, 2);
        return b;
    } else {
        // The fp32 value must exist before it is narrowed: without this barrier LLVM folds
        // fptrunc(fma(a, b, c)) into v_fma_mixlo_f16, which rounds the exact result to fp16 ONCE -- torch
        // rounds to fp32 first and then to fp16 (a different result when the fp32 rounding makes a tie).
        asm volatile("" : "+v"(x));
        const _Float16 h = (_Float16)x;  // v_cvt_f16_f32: round to nearest even, fp16 denormals kept
        uint16_t b;
        __builtin_memcpy(&b, &h, 2);
        return b;
    }
}

template <int FMT>
__device__ __forceinline__ float rnd(float x) {
    return load16<FMT>(bits16<FMT>(x));
}

template <int FMT, int OP>
__device__ __forceinline__ float first16(float v, float w) {
    if constexpr (OP == FEDAVG_OP_UNWEIGHTED) {
        return v;
    } else {
        return rnd<FMT>(v * w);
    }
}

// torch-ROCm's float16 add_(v, alpha) on device-resident tensors (FEDAVG_OP_TORCH_DEVICE) in its unrolled
// (non-vector) path: the exact fma rounded once, straight to fp16 (v_fma_mixlo_f16; established against torch
// on the GPU: tools/debug_fp16_device.py), where its vector path and the CPU kernel round to fp32 first.
// Explicit, so that no compiler choice decides it; all three sources are fp32 (op_sel_hi 0), result in the low
// half.
__device__ __forceinline__ float fma_f16_once(float a, float b, float c) {
    uint32_t d = 0;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, %3" : "+v"(d) : "v"(a), "v"(b), "v"(c));
    return load16<FEDAVG_F16>((uint16_t)(d & 0xffffu));
}

template <int FMT, int OP>
__device__ __forceinline__ float step16(float t, float v, float w) {
    if constexpr (OP == FEDAVG_OP_TORCH) {
        return rnd<FMT>(__builtin_fmaf(v, w, t));
    } else if constexpr (OP == FEDAVG_OP_NUMPY) {
        return rnd<FMT>(t + rnd<FMT>(v * w));
    } else {
        return rnd<FMT>(t + v);
    }
}

template <int FMT, int FIN>
__device__ __forceinline__ float fin16(float t, float s) {
    if constexpr (FIN == FEDAVG_FIN_SCALE) {
        return rnd<FMT>(t * s);
    } else if constexpr (FIN == FEDAVG_FIN_DIV) {
        return rnd<FMT>(t / s);
    } else {
        return t;
    }
}

template <int FMT, int OP, int FIN, bool ACC_IN>
__device__ __forceinline__ float elem16(const RowTableNarrow& tab, int K, const uint16_t* acc_in, int64_t i, float fv) {
    float t;
    int k = 0;
    if constexpr (ACC_IN) {
        t = load16<FMT>(acc_in[i]);
    } else {
        t = first16<FMT, OP>(load16<FMT>(static_cast<const uint16_t*>(tab.rows[0])[i]), tab.w_first[0]);
        k = 1;
    }
    for (; k < K; ++k) t = step16<FMT, OP>(t, load16<FMT>(static_cast<const uint16_t*>(tab.rows[k])[i]), tab.w_step[k]);
    return fin16<FMT, FIN>(t, fv);
}

__device__ __forceinline__ uint16_t half_of(const u32x4& v, int j) {
    return (uint16_t)((v[j >> 1] >> ((j & 1) * 16)) & 0xffffu);
}

// Packed forms of the steps above, two elements per 32-bit word (element 0 in the low half): the fp32 arithmetic on
// f32x2 compiles to gfx950's packed v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32 (each lane computes both elements
// with the per-element roundings of the scalar ops -- the same bits), and pack2 rounds both to the format in one
// v_cvt_pk_{bf16,f16}_f32 (round to nearest even; bit-equal to bits16 per element for every fp32 input, NaN to a
// NaN: tools/cvt_pk_probe.hip, exhaustive).  The opaque asm operands also keep fptrunc(fma) from folding into a
// single-rounding mixed fma (see bits16).  Used by the few-client kernel below only: there it beat the per-element
// form (bf16 1 client 68.0 against 62.6 % of 8 TB/s, profiles/r05/s9/, s10/), while in tile_sum16 (the burst and
// per-tile forms) it lost badly (bf16 8 / 64 clients 71.7 / 64.5 % against 81.1 / 89.2 %, profiles/r05/s11/).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

template <int FMT>
__device__ __forceinline__ f32x2 unpack2(const uint32_t d) {
    if constexpr (FMT == FEDAVG_BF16) {
        return f32x2{__uint_as_float(d << 16), __uint_as_float(d & 0xffff0000u)};
    } else {
        return f32x2{load16<FEDAVG_F16>((uint16_t)(d & 0xffffu)), load16<FEDAVG_F16>((uint16_t)(d >> 16))};
    }
}

template <int FMT>
__device__ __forceinline__ uint32_t pack2(const f32x2 x) {
    uint32_t d;
    if constexpr (FMT == FEDAVG_BF16) {
        asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(d) : "v"(x[0]), "v"(x[1]));
    } else {
        asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(d) : "v"(x[0]), "v"(x[1]));
    }
    return d;
}

// first16 / step16 on a word: returns the rounded running values' word; t their fp32 values
template <int FMT, int OP>
__device__ __forceinline__ uint32_t first2(const uint32_t d, const float w, f32x2& t) {
    if constexpr (OP == FEDAVG_OP_UNWEIGHTED) {
        t = unpack2<FMT>(d);
        return d;
    } else {
        const uint32_t r = pack2<FMT>(unpack2<FMT>(d) * w);
        t = unpack2<FMT>(r);
        return r;
    }
}

template <int FMT, int OP>
__device__ __forceinline__ uint32_t step2(const uint32_t d, const float w, f32x2& t) {
    const f32x2 v = unpack2<FMT>(d);
    uint32_t r;
    if constexpr (OP == FEDAVG_OP_TORCH) {
        r = pack2<FMT>(__builtin_elementwise_fma(v, f32x2{w, w}, t));
    } else if constexpr (OP == FEDAVG_OP_NUMPY) {
        r = pack2<FMT>(t + unpack2<FMT>(pack2<FMT>(v * w)));
    } else {
        r = pack2<FMT>(t + v);
    }
    t = unpack2<FMT>(r);
    return r;
}

// The finalisation on packed running values (CPL 8-element groups of a lane: words and their fp32 values), to the
// output words.  FIN_DIV: rnd(T / float(count)), the exact fp32 quotient (div_const_fast's Markstein correction,
// packed), then the rounding.  Its range condition on the dividends -- fp32 exponent 27..226, which a 16-bit T
// meets unless it is zero, infinite or NaN, or a bfloat16 beyond 2^+-100 -- is checked on the words' magnitudes,
// their packed 16-bit maximum and minimum over the tile (bit order = magnitude order); else the IEEE quotient.
template <int FMT, int FIN, int CPL>
__device__ __forceinline__ void fin_words(u32x4 (&res)[CPL], const uint32_t (&word)[CPL][4], const f32x2 (&t)[CPL][4],
                                          const FinConst& fc, const float fv) {
    if constexpr (FIN == FEDAVG_FIN_DIV) {
        u16x2 mx = {0, 0}, mn = {0xffff, 0xffff};
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t a = word[c][e] & 0x7fff7fffu;
                u16x2 h;
                __builtin_memcpy(&h, &a, 4);
                mx = __builtin_elementwise_max(mx, h);
                mn = __builtin_elementwise_min(mn, h);
            }
        constexpr uint16_t lo = FMT == FEDAVG_BF16 ? 27u << 7 : 1u;          // bf16: exponent >= 27; f16: nonzero
        constexpr uint16_t hi = FMT == FEDAVG_BF16 ? 227u << 7 : 0x7c00u;    // bf16: exponent <= 226; f16: finite
        const bool slow = !fc.fast || mx[0] >= hi || mx[1] >= hi || mn[0] < lo || mn[1] < lo;
        if (__builtin_expect(!slow, 1)) {
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const f32x2 q = t[c][e] * fc.r;
                    const f32x2 er = __builtin_elementwise_fma(-q, f32x2{fc.v, fc.v}, t[c][e]);
                    res[c][e] = pack2<FMT>(__builtin_elementwise_fma(er, f32x2{fc.r, fc.r}, q));
                }
        } else {
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) res[c][e] = pack2<FMT>(t[c][e] / fc.v);
        }
    } else if constexpr (FIN == FEDAVG_FIN_SCALE) {
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) res[c][e] = pack2<FMT>(t[c][e] * fv);
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) res[c][e] = word[c][e];
    }
}

template <int FMT, int OP, int FIN, bool ACC_IN, bool VEC>
__global__ void __launch_bounds__(kBlock) fedavg_rows_narrow(const RowTableNarrow tab, const int K,
                                                              const uint16_t* acc_in, uint16_t* out, const int64_t n,
                                                              const float fv) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    int64_t done = 0;
    if constexpr (VEC) {
        const int64_t n8 = n / 8;
        for (int64_t g = tid; g < n8; g += stride) {
            float t[8];
            int k = 0;
            if constexpr (ACC_IN) {
                const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(acc_in) + g);
#pragma unroll
                for (int j = 0; j < 8; ++j) t[j] = load16<FMT>(half_of(a, j));
            } else {
                const u32x4 a = __builtin_nontemporal_load(static_cast<const u32x4*>(tab.rows[0]) + g);
#pragma unroll
                for (int j = 0; j < 8; ++j) t[j] = first16<FMT, OP>(load16<FMT>(half_of(a, j)), tab.w_first[0]);
                k = 1;
            }
            // four clients' loads in flight before their arrival-ordered arithmetic (as the fp32 kernel)
            for (; k + 4 <= K; k += 4) {
                u32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(static_cast<const u32x4*>(tab.rows[k + u]) + g);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float w = tab.w_step[k + u];
#pragma unroll
                    for (int j = 0; j < 8; ++j) t[j] = step16<FMT, OP>(t[j], load16<FMT>(half_of(v[u], j)), w);
                }
            }
            for (; k < K; ++k) {
                const u32x4 v = __builtin_nontemporal_load(static_cast<const u32x4*>(tab.rows[k]) + g);
                const float w = tab.w_step[k];
#pragma unroll
                for (int j = 0; j < 8; ++j) t[j] = step16<FMT, OP>(t[j], load16<FMT>(half_of(v, j)), w);
            }
            u32x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[j] = (uint32_t)bits16<FMT>(fin16<FMT, FIN>(t[2 * j], fv)) |
                       ((uint32_t)bits16<FMT>(fin16<FMT, FIN>(t[2 * j + 1], fv)) << 16);
            }
            __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(out) + g);
        }
        done = n8 * 8;
    }
    for (int64_t i = done + tid; i < n; i += stride) out[i] = bits16<FMT>(elem16<FMT, OP, FIN, ACC_IN>(tab, K, acc_in, i, fv));
}

// ---------------------------------------------------------------------------------------------
// TILED storage (the engine's slab layout for 16-bit keys): element i of client k lives at
//   bases[k] + (i / 4096) * tile_stride + i % 4096      (16-bit elements)
// A block owns a tile (4096 elements = 8 KiB per client); each lane owns two 8-element groups, so a wave
// reads 1 KiB contiguous per client and group, and one tile's K client segments form one sequential run
// (S * 8 KiB) when the slots are interleaved.  Units below are 8-element groups (u32x4).
// ---------------------------------------------------------------------------------------------
constexpr int kTile16 = 4096;
constexpr int kCpl16 = kTile16 / (8 * kBlock);  // 2
#ifndef FEDAVG_NARROW_BURST_WAVES
#define FEDAVG_NARROW_BURST_WAVES 2  // waves per SIMD the burst kernel is compiled for (register budget)
#endif
#ifndef FEDAVG_NARROW_UNROLL
#define FEDAVG_NARROW_UNROLL 6  // clients whose loads are in flight together (A/B: profiles/r01/narrow_unroll_ab.jsonl)
#endif
// Burst launches under this many clients take groups of 4 (round 4, bf16, groups of 4 against 6: 8 / 12 / 16 clients
// 79.8 / 80.6 / 84.2 % against 77.8 / 77.5 / 82.0 %, but 64 clients 71.0 % against 89.4 %; profiles/r04/s13/)
constexpr int kNarrowUnroll4MaxK = 32;

// One tile's arrival-ordered sum for this lane's kCpl16 8-element groups, packed to the output format.
// GROUPED (the burst form): load groups of UNROLL clients from client 0 on, as fedavg_arith.h tile_sum.
template <int FMT, int OP, int FIN, bool ACC_IN, bool GROUPED = false, int UNROLL = FEDAVG_NARROW_UNROLL>
__device__ __forceinline__ void tile_sum16(u32x4 (&res)[kCpl16], const RowTableNarrow& tab, const int K,
                                           const int64_t off, const int64_t col, const u32x4* acc_in, const int64_t b8,
                                           const int64_t e8, const float fv) {
    float acc[kCpl16][8];
    int k = 0;
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < kCpl16; ++c) {
            const int64_t i = col + c * kBlock;
            const u32x4 a = (i >= b8 && i < e8) ? acc_in[i] : u32x4{0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[c][j] = load16<FMT>(half_of(a, j));
        }
    }
    if constexpr (GROUPED) {
        for (; k < K; k += UNROLL) {
            u32x4 v[UNROLL][kCpl16];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const u32x4* r = static_cast<const u32x4*>(tab.rows[k + u < K ? k + u : K - 1]) + off;
#pragma unroll
                for (int c = 0; c < kCpl16; ++c) v[u][c] = __builtin_nontemporal_load(r + c * kBlock);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                if (k + u < K) {
                    if (!ACC_IN && k + u == 0) {
                        const float w = tab.w_first[0];
#pragma unroll
                        for (int c = 0; c < kCpl16; ++c)
#pragma unroll
                            for (int j = 0; j < 8; ++j) acc[c][j] = first16<FMT, OP>(load16<FMT>(half_of(v[u][c], j)), w);
                    } else {
                        const float w = tab.w_step[k + u];
#pragma unroll
                        for (int c = 0; c < kCpl16; ++c)
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                acc[c][j] = step16<FMT, OP>(acc[c][j], load16<FMT>(half_of(v[u][c], j)), w);
                    }
                }
            }
        }
        k = K;
    } else if constexpr (!ACC_IN) {
        const u32x4* r = static_cast<const u32x4*>(tab.rows[0]) + off;
#pragma unroll
        for (int c = 0; c < kCpl16; ++c) {
            const u32x4 a = __builtin_nontemporal_load(r + c * kBlock);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[c][j] = first16<FMT, OP>(load16<FMT>(half_of(a, j)), tab.w_first[0]);
        }
        k = 1;
    }
    for (; k + UNROLL <= K; k += UNROLL) {
        u32x4 v[UNROLL][kCpl16];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const u32x4* r = static_cast<const u32x4*>(tab.rows[k + u]) + off;
#pragma unroll
            for (int c = 0; c < kCpl16; ++c) v[u][c] = __builtin_nontemporal_load(r + c * kBlock);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const float w = tab.w_step[k + u];
#pragma unroll
            for (int c = 0; c < kCpl16; ++c)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[c][j] = step16<FMT, OP>(acc[c][j], load16<FMT>(half_of(v[u][c], j)), w);
        }
    }
    for (; k < K; ++k) {
        const u32x4* r = static_cast<const u32x4*>(tab.rows[k]) + off;
        const float w = tab.w_step[k];
#pragma unroll
        for (int c = 0; c < kCpl16; ++c) {
            const u32x4 v = __builtin_nontemporal_load(r + c * kBlock);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[c][j] = step16<FMT, OP>(acc[c][j], load16<FMT>(half_of(v, j)), w);
        }
    }
#pragma unroll
    for (int c = 0; c < kCpl16; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            res[c][j] = (uint32_t)bits16<FMT>(fin16<FMT, FIN>(acc[c][2 * j], fv)) |
                        ((uint32_t)bits16<FMT>(fin16<FMT, FIN>(acc[c][2 * j + 1], fv)) << 16);
}

// per-tile-store form (launch variant bit 3): each tile's results stored as it finishes
template <int FMT, int OP, int FIN, bool ACC_IN>
__global__ void __launch_bounds__(kBlock) fedavg_tiles_narrow(const RowTableNarrow tab, const int K,
                                                               const int64_t tstride8, const u32x4* acc_in,
                                                               u32x4* out, const int64_t b8, const int64_t e8,
                                                               const float fv) {
    constexpr int64_t T8 = (int64_t)kCpl16 * kBlock;
    const int64_t t_last = (e8 - 1) / T8;
    for (int64_t t = b8 / T8 + blockIdx.x; t <= t_last; t += gridDim.x) {
        u32x4 res[kCpl16];
        tile_sum16<FMT, OP, FIN, ACC_IN>(res, tab, K, t * tstride8 + threadIdx.x, t * T8 + threadIdx.x, acc_in, b8, e8, fv);
#pragma unroll
        for (int c = 0; c < kCpl16; ++c) {
            const int64_t i = t * T8 + threadIdx.x + c * kBlock;
            if (i >= b8 && i < e8) __builtin_nontemporal_store(res[c], out + i);
        }
    }
}

// BURST form (the default; fedavg_tiles.h fedavg_tiles_burst_f32x4 has the measurements): TPB tiles per
// block per launch, their packed results held in registers and stored after the block's last tile; client
// loads grouped from client 0 on (bf16 64 x 1e9: 85.6 % against 84.4 % ungrouped and 82.0 % for the per-tile
// form, profiles/r02/ab/narrow_burst_grouped.jsonl).
// TPB_LDS > 0 (the default; burst mode 2): that many more tiles per block, their packed results held in LDS
// (8 KiB per tile; each lane reads back only what it wrote) -- launches (TPB + TPB_LDS) / TPB times longer.
template <int FMT, int OP, int FIN, bool ACC_IN, int TPB, int TPB_LDS = 0, int UNROLL = FEDAVG_NARROW_UNROLL>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(FEDAVG_NARROW_BURST_WAVES, FEDAVG_NARROW_BURST_WAVES))) fedavg_tiles_narrow_burst(const RowTableNarrow tab, const int K, const int64_t tstride8, const u32x4* acc_in, u32x4* out,
                          const int64_t b8, const int64_t e8, const float fv, const int64_t t0, const int64_t t_end) {
    constexpr int64_t T8 = (int64_t)kCpl16 * kBlock;
    u32x4 res[TPB][kCpl16];
    __shared__ u32x4 staged[TPB_LDS > 0 ? TPB_LDS * kCpl16 * kBlock : 1];
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end)
            tile_sum16<FMT, OP, FIN, ACC_IN, true, UNROLL>(res[m], tab, K, t * tstride8 + threadIdx.x, t * T8 + threadIdx.x,
                                                   acc_in, b8, e8, fv);
    }
    // the LDS-held tiles in a rolled loop: one more copy of the (long) tile body, not TPB_LDS of them
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            u32x4 r[kCpl16];
            tile_sum16<FMT, OP, FIN, ACC_IN, true, UNROLL>(r, tab, K, t * tstride8 + threadIdx.x, t * T8 + threadIdx.x, acc_in,
                                                   b8, e8, fv);
#pragma unroll
            for (int c = 0; c < kCpl16; ++c) staged[((m - TPB) * kCpl16 + c) * kBlock + threadIdx.x] = r[c];
        }
    }
#pragma unroll 1
    for (int m = TPB; m < TPB + TPB_LDS; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < kCpl16; ++c) {
                const int64_t i = t * T8 + threadIdx.x + c * kBlock;
                if (i >= b8 && i < e8)
                    __builtin_nontemporal_store(staged[((m - TPB) * kCpl16 + c) * kBlock + threadIdx.x], out + i);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < kCpl16; ++c) {
                const int64_t i = t * T8 + threadIdx.x + c * kBlock;
                if (i >= b8 && i < e8) __builtin_nontemporal_store(res[m][c], out + i);
            }
        }
    }
}

// FEW-CLIENT 16-bit burst form (round 5): 1-3 client reads, no chained sum -- the 16-bit twin of fedavg_tiles.h
// fedavg_tiles_few_f32x4.  The burst form above loads its clients in groups of 4 or 6 from client 0 on, so at one or
// two clients most of its loads re-read a row (bf16 x 1e9: 38 / 56 % of 8 TB/s at 1 / 2 clients, profiles/r05/s8/), and
// its tile guard and per-element FIN_DIV keep one tile's loads in flight per wave.  Here every load is a real client's
// and unconditional (a slot past the launch's last tile re-reads that tile; only real tiles are stored), the R
// register-held tiles' loads go out first, the L LDS-held tiles stream through in groups of G, the arithmetic is the
// packed form (pack2 / step2: two elements per instruction), and FIN_DIV is the exact fp32 quotient by Markstein's
// correction with one rare-case branch per tile (fedavg_arith.h div_const_fast), rounded to the format as torch's
// div_ rounds it.  Per-element sequence as tile_sum16's: the same bits.
// P = 2 (the 1- and 3-read defaults): a unit is a pair of consecutive tiles -- K x 16 KiB of contiguous slab per
// unit, the fp32 forms' shape in bytes; the pair's second tile past the range's last tile re-reads that tile (never
// stored).
template <int FMT, int OP, int FIN, int KC, int R, int L, int G, int B, int P = 1>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(B, 2)))  // B blocks per CU must co-reside
fedavg_tiles_narrow_few(const RowTableNarrow tab, const int64_t tstride8, u32x4* out, const int64_t b8, const int64_t e8,
                        const float fv, const int64_t t0, const int64_t t_end) {
    static_assert(KC >= 1 && KC <= 3, "one to three row reads");
    static_assert(L == 0 || L % G == 0, "whole LDS groups");
    static_assert(P == 1 || P == 2 || P == 4, "single tiles, pairs or quads");
    constexpr int CPL = kCpl16 * P;                      // u32x4 per lane per unit
    constexpr int64_t T8 = (int64_t)CPL * kBlock;        // u32x4 per unit
    const int64_t last_tile = (e8 - 1) / ((int64_t)kCpl16 * kBlock);
    const int64_t first_tile = b8 / ((int64_t)kCpl16 * kBlock);  // a unit's tiles before begin's are not read
    const FinConst fc = fin_const<FIN>(fv);
    __shared__ u32x4 staged[L > 0 ? L * CPL * kBlock : 1];
    const int64_t t_first = t0 + blockIdx.x;
    auto tile_of = [&](const int m) __attribute__((always_inline)) {
        const int64_t t = t_first + (int64_t)m * gridDim.x;
        return t < t_end ? t : t_end - 1;
    };
    auto load_tile = [&](u32x4 (&v)[KC][CPL], const int m) __attribute__((always_inline)) {
        const int64_t u = tile_of(m);
#pragma unroll
        for (int h = 0; h < P; ++h) {
            int64_t tile = u * P + h;
            tile = tile <= last_tile ? tile : last_tile;
            tile = tile >= first_tile ? tile : first_tile;
            const int64_t off = tile * tstride8 + threadIdx.x;
#pragma unroll
            for (int j = 0; j < KC; ++j)
#pragma unroll
                for (int c = 0; c < kCpl16; ++c)
                    v[j][h * kCpl16 + c] =
                        __builtin_nontemporal_load(static_cast<const u32x4*>(tab.rows[j]) + off + c * kBlock);
        }
    };
    auto finish = [&](u32x4 (&res)[CPL], const u32x4 (&v)[KC][CPL]) __attribute__((always_inline)) {
        uint32_t word[CPL][4];  // the running values, rounded to the format, two per word
        f32x2 t[CPL][4];        // and as fp32
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                word[c][e] = first2<FMT, OP>(v[0][c][e], tab.w_first[0], t[c][e]);
#pragma unroll
                for (int j = 1; j < KC; ++j) word[c][e] = step2<FMT, OP>(v[j][c][e], tab.w_step[j], t[c][e]);
            }
        fin_words<FMT, FIN, CPL>(res, word, t, fc, fv);
    };
    // 1. the register-held tiles' loads (slots L .. L+R-1)
    u32x4 vr[R][KC][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) load_tile(vr[m], L + m);
    // 2. the LDS-held tiles (slots 0 .. L-1), G at a time
#pragma unroll
    for (int g = 0; g < L; g += G) {
        u32x4 v[G][KC][CPL];
#pragma unroll
        for (int m = 0; m < G; ++m) load_tile(v[m], g + m);
#pragma unroll
        for (int m = 0; m < G; ++m) {
            u32x4 r[CPL];
            finish(r, v[m]);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((g + m) * CPL + c) * kBlock + threadIdx.x] = r[c];
        }
    }
    // 3. the register-held tiles
    u32x4 res[R][CPL];
#pragma unroll
    for (int m = 0; m < R; ++m) finish(res[m], vr[m]);
    // 4. the write burst
#pragma unroll
    for (int m = 0; m < L + R; ++m) {
        const int64_t t = t_first + (int64_t)m * gridDim.x;
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T8 + threadIdx.x + c * kBlock;
                const u32x4 r = m < L ? staged[(m * CPL + c) * kBlock + threadIdx.x] : res[m < L ? 0 : m - L][c];
                if (i >= b8 && i < e8) __builtin_nontemporal_store(r, out + i);
            }
        }
    }
}

template <int FMT, int OP, int FIN, int KC, int R, int L, int G, int B, int P = 1>
static hipError_t launch_narrow_few_form(const RowTableNarrow& tab, int64_t tstride8, void* out, int64_t b8, int64_t e8,
                                         float fv, int grid, hipStream_t s, uint64_t* nl) {
    constexpr int64_t U8 = (int64_t)kCpl16 * kBlock * P;
    u32x4* o = static_cast<u32x4*>(out);
    return burst_launches(b8 / U8, (e8 - 1) / U8 + 1, grid, R + L, nl, false, [&](int nb, int64_t t0, int64_t t_end, uint32_t) {
        hipLaunchKernelGGL((fedavg_tiles_narrow_few<FMT, OP, FIN, KC, R, L, G, B, P>), dim3(nb), dim3(kBlock), 0, s, tab,
                           tstride8, o, b8, e8, fv, t0, t_end);
    });
}

template <int FMT, int OP, int FIN, int KC>
static hipError_t launch_narrow_few(const RowTableNarrow& tab, int64_t tstride8, void* out, int64_t b8, int64_t e8,
                                    float fv, int grid, int form, hipStream_t s, uint64_t* nl) {
    const FewForm f = narrow_few_form(KC, form);
#define FEDAVG_NFEW(B, R, LL, G)                                      \
    if (f.bpc == B && f.r == R && f.l == LL && f.g == G && f.p <= 1)  \
        return launch_narrow_few_form<FMT, OP, FIN, KC, R, LL, G, B>(tab, tstride8, out, b8, e8, fv, grid, s, nl);
#define FEDAVG_NFEW2(B, R, LL, G)                                     \
    if (f.bpc == B && f.r == R && f.l == LL && f.g == G && f.p == 2)  \
        return launch_narrow_few_form<FMT, OP, FIN, KC, R, LL, G, B, 2>(tab, tstride8, out, b8, e8, fv, grid, s, nl);
#define FEDAVG_NFEW4(B, R, LL, G)                                     \
    if (f.bpc == B && f.r == R && f.l == LL && f.g == G && f.p == 4)  \
        return launch_narrow_few_form<FMT, OP, FIN, KC, R, LL, G, B, 4>(tab, tstride8, out, b8, e8, fv, grid, s, nl);
    if constexpr (KC == 1) {
        FEDAVG_NFEW2(2, 8, 4, 4)
        if constexpr (kABFew) {
            FEDAVG_NFEW(2, 8, 8, 4)
            FEDAVG_NFEW2(2, 8, 4, 2)
            FEDAVG_NFEW4(2, 4, 2, 2)
            FEDAVG_NFEW4(2, 4, 2, 1)
        }
    } else if constexpr (KC == 2) {
        FEDAVG_NFEW(2, 8, 8, 4)
        if constexpr (kABFew) {
            FEDAVG_NFEW2(1, 4, 10, 1)
            FEDAVG_NFEW2(1, 4, 10, 2)
            FEDAVG_NFEW(1, 8, 20, 2)
            FEDAVG_NFEW(1, 6, 20, 4)
        }
    } else {
        FEDAVG_NFEW2(1, 4, 10, 2)
        if constexpr (kABFew) {
            FEDAVG_NFEW(1, 8, 20, 4)
            FEDAVG_NFEW2(1, 4, 10, 1)
            FEDAVG_NFEW(1, 8, 20, 2)
            FEDAVG_NFEW(1, 6, 20, 2)
        }
    }
#undef FEDAVG_NFEW
#undef FEDAVG_NFEW2
#undef FEDAVG_NFEW4
    return hipErrorInvalidValue;
}

template <int FMT, int OP, int FIN>
static hipError_t launch_t16_a(const RowTableNarrow& tab, int K, int64_t tstride8, const void* acc_in, void* out,
                               int64_t b8, int64_t e8, float fv, int grid, int burst, hipStream_t s, uint64_t* nl) {
    const u32x4* ai = static_cast<const u32x4*>(acc_in);
    u32x4* o = static_cast<u32x4*>(out);
    constexpr int64_t T8 = (int64_t)kCpl16 * kBlock;
    if (burst >= 3) {  // the few-client form (1-3 reads, no chained sum); burst - 3 = its A/B form index (0: default)
        if (acc_in) return hipErrorInvalidValue;
        if (K == 1) return launch_narrow_few<FMT, OP, FIN, 1>(tab, tstride8, out, b8, e8, fv, grid, burst - 3, s, nl);
        if (K == 2) return launch_narrow_few<FMT, OP, FIN, 2>(tab, tstride8, out, b8, e8, fv, grid, burst - 3, s, nl);
        if (K == 3) return launch_narrow_few<FMT, OP, FIN, 3>(tab, tstride8, out, b8, e8, fv, grid, burst - 3, s, nl);
        return hipErrorInvalidValue;
    }
    if (burst == 2 || !kAB) {  // default: kBurstTiles in registers + kBurstLdsTiles16 in LDS per block and launch
        // client groups of 4 under kNarrowUnroll4MaxK clients, of FEDAVG_NARROW_UNROLL (6) from there on
        const bool u4 = K < kNarrowUnroll4MaxK;
        return burst_launches(b8 / T8, (e8 - 1) / T8 + 1, grid, kBurstTiles + kBurstLdsTiles16, nl, false,
                              [&](int nb, int64_t t0, int64_t t_end, uint32_t) {
#define FEDAVG_T16_BURST(AI, U)                                                                                        \
    hipLaunchKernelGGL((fedavg_tiles_narrow_burst<FMT, OP, FIN, AI, kBurstTiles, kBurstLdsTiles16, U>), dim3(nb),      \
                       dim3(kBlock), 0, s, tab, K, tstride8, ai, o, b8, e8, fv, t0, t_end)
            if (acc_in && u4) FEDAVG_T16_BURST(true, 4);
            else if (acc_in) FEDAVG_T16_BURST(true, FEDAVG_NARROW_UNROLL);
            else if (u4) FEDAVG_T16_BURST(false, 4);
            else FEDAVG_T16_BURST(false, FEDAVG_NARROW_UNROLL);
#undef FEDAVG_T16_BURST
        });
    }
    if constexpr (kAB) {  // A/B builds: the register-only burst form (variant bit 5) and the per-tile form (bit 3)
        if (burst) {
            return burst_launches(b8 / T8, (e8 - 1) / T8 + 1, grid, kBurstTiles, nl, false, [&](int nb, int64_t t0, int64_t t_end, uint32_t) {
                if (acc_in)
                    hipLaunchKernelGGL((fedavg_tiles_narrow_burst<FMT, OP, FIN, true, kBurstTiles>), dim3(nb), dim3(kBlock), 0,
                                       s, tab, K, tstride8, ai, o, b8, e8, fv, t0, t_end);
                else
                    hipLaunchKernelGGL((fedavg_tiles_narrow_burst<FMT, OP, FIN, false, kBurstTiles>), dim3(nb), dim3(kBlock),
                                       0, s, tab, K, tstride8, ai, o, b8, e8, fv, t0, t_end);
            });
        }
        if (acc_in) {
            hipLaunchKernelGGL((fedavg_tiles_narrow<FMT, OP, FIN, true>), dim3(grid), dim3(kBlock), 0, s, tab, K, tstride8, ai,
                               o, b8, e8, fv);
        } else {
            hipLaunchKernelGGL((fedavg_tiles_narrow<FMT, OP, FIN, false>), dim3(grid), dim3(kBlock), 0, s, tab, K, tstride8,
                               ai, o, b8, e8, fv);
        }
        if (nl) ++*nl;
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int FMT, int OP>
static hipError_t launch_t16_f(const RowTableNarrow& tab, int K, int64_t tstride8, const void* acc_in, void* out,
                               int64_t b8, int64_t e8, int fin, float fv, int grid, int burst, hipStream_t s,
                               uint64_t* nl) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_t16_a<FMT, OP, FEDAVG_FIN_SCALE>(tab, K, tstride8, acc_in, out, b8, e8, fv, grid, burst, s, nl);
        case FEDAVG_FIN_DIV:
            return launch_t16_a<FMT, OP, FEDAVG_FIN_DIV>(tab, K, tstride8, acc_in, out, b8, e8, fv, grid, burst, s, nl);
        default:
            return launch_t16_a<FMT, OP, FEDAVG_FIN_NONE>(tab, K, tstride8, acc_in, out, b8, e8, fv, grid, burst, s, nl);
    }
}

template <int FMT>
static hipError_t launch_t16_o(const RowTableNarrow& tab, int K, int64_t tstride8, const void* acc_in, void* out,
                               int64_t b8, int64_t e8, int op, int fin, float fv, int grid, int burst, hipStream_t s,
                               uint64_t* nl) {
    switch (op) {
        case FEDAVG_OP_TORCH_DEVICE:  // same steps; the host keeps alpha in fp32 in the table
        case FEDAVG_OP_TORCH:
            return launch_t16_f<FMT, FEDAVG_OP_TORCH>(tab, K, tstride8, acc_in, out, b8, e8, fin, fv, grid, burst, s, nl);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_t16_f<FMT, FEDAVG_OP_UNWEIGHTED>(tab, K, tstride8, acc_in, out, b8, e8, fin, fv, grid, burst, s,
                                                            nl);
        default:
            return launch_t16_f<FMT, FEDAVG_OP_NUMPY>(tab, K, tstride8, acc_in, out, b8, e8, fin, fv, grid, burst, s, nl);
    }
}

// ---------------------------------------------------------------------------------------------
// The build compiles this file twice (nvflare_amd/_build.py): FEDAVG_NARROW_PART=1 holds the bfloat16 kernels and the
// dispatchers below, =2 the float16 kernels -- each format's entry points (tiles16_fmt, rows16_fmt, tails16_fmt) are
// instantiated in its own unit, halving what was the build's longest translation unit.  Without the macro (a tool
// compiling this file alone) one unit holds both.
// ---------------------------------------------------------------------------------------------
#if !defined(FEDAVG_NARROW_PART)
#define FEDAVG_NARROW_PART 0
#endif

template <int FMT>
hipError_t tiles16_fmt(const RowTableNarrow& tab, int K, int64_t ts8, const void* acc_in, void* out, int64_t b8,
                       int64_t e8, int op, int fin, float fv, int grid, int burst, hipStream_t s, uint64_t* nl) {
    return launch_t16_o<FMT>(tab, K, ts8, acc_in, out, b8, e8, op, fin, fv, grid, burst, s, nl);
}

// ---------------------------------------------------------------------------------------------
// torch's scalar remainder.  torch CPU runs T.add_(v, alpha=w) on float16 / bfloat16 tensors
// (weighted_aggregation_helper.py:207) over the ranges at::parallel_for gives its threads (one range below
// 32768 elements), each through cpu_kernel_vec's vectorized loop -- one fp32 fma, the TORCH step above --
// and, for the last (range length mod 32) elements of the range, through the scalar remainder loop, whose
// c10::Half / c10::BFloat16 operators round the product and the sum separately:  p = r(v * r(w)), T = r(T + p).
// (The first v.mul(w) and the final div_ compute the same in both loops.)  The engine lists those elements;
// fedavg_torch16_tails recomputes them from the same inputs into a side buffer before the tile kernel runs
// (acc_in may alias out), and fedavg_scatter16 writes them over the tile kernel's results after it.
// ---------------------------------------------------------------------------------------------
// DEVICE: the listed elements are those torch-ROCm's float16 add_ runs through its unrolled path (the last
// partial block of its vectorized kernel): one rounding of the exact fma, fma_f16_once.
template <int FMT, int FIN, bool ACC_IN, bool DEVICE>
__global__ void __launch_bounds__(kBlock) fedavg_torch16_tails(const RowTableNarrow tab, const int K, const int64_t tile,
                                                                const int64_t tstride, const int64_t* idx,
                                                                const int64_t m, const uint16_t* acc_in,
                                                                uint16_t* vals, const float fv) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= m) return;
    const int64_t i = idx[j];
    const int64_t off = (i / tile) * tstride + i % tile;
    float t;
    int k = 0;
    if constexpr (ACC_IN) {
        t = load16<FMT>(acc_in[i]);
    } else {
        t = first16<FMT, FEDAVG_OP_TORCH>(load16<FMT>(static_cast<const uint16_t*>(tab.rows[0])[off]), tab.w_first[0]);
        k = 1;
    }
    for (; k < K; ++k) {
        const float v = load16<FMT>(static_cast<const uint16_t*>(tab.rows[k])[off]);
        if constexpr (DEVICE)
            t = fma_f16_once(v, tab.w_step[k], t);  // tab.w_step[k] = float(w): torch-ROCm's fp32 opmath alpha
        else
            t = rnd<FMT>(t + rnd<FMT>(v * tab.w_step[k]));  // tab.w_step[k] = r(w): c10 casts alpha to the dtype
    }
    vals[j] = bits16<FMT>(fin16<FMT, FIN>(t, fv));
}


template <int FMT, int FIN, bool DEVICE>
static hipError_t launch_tails_a(const RowTableNarrow& tab, int K, int64_t tile, int64_t tstride, const int64_t* idx,
                                 int64_t m, const void* acc_in, void* vals, float fv, int grid, hipStream_t s) {
    const uint16_t* ai = static_cast<const uint16_t*>(acc_in);
    uint16_t* v = static_cast<uint16_t*>(vals);
    if (acc_in)
        hipLaunchKernelGGL((fedavg_torch16_tails<FMT, FIN, true, DEVICE>), dim3(grid), dim3(kBlock), 0, s, tab, K, tile,
                           tstride, idx, m, ai, v, fv);
    else
        hipLaunchKernelGGL((fedavg_torch16_tails<FMT, FIN, false, DEVICE>), dim3(grid), dim3(kBlock), 0, s, tab, K, tile,
                           tstride, idx, m, ai, v, fv);
    return hipGetLastError();
}

template <int FMT, bool DEVICE>
static hipError_t launch_tails_f(const RowTableNarrow& tab, int K, int64_t tile, int64_t tstride, const int64_t* idx,
                                 int64_t m, const void* acc_in, void* vals, int fin, float fv, int grid, hipStream_t s) {
    switch (fin) {  // (FEDAVG_FIN_RECIP arrives as its SCALE form)
        case FEDAVG_FIN_SCALE:
            return launch_tails_a<FMT, FEDAVG_FIN_SCALE, DEVICE>(tab, K, tile, tstride, idx, m, acc_in, vals, fv, grid, s);
        case FEDAVG_FIN_DIV:
            return launch_tails_a<FMT, FEDAVG_FIN_DIV, DEVICE>(tab, K, tile, tstride, idx, m, acc_in, vals, fv, grid, s);
        default:
            return launch_tails_a<FMT, FEDAVG_FIN_NONE, DEVICE>(tab, K, tile, tstride, idx, m, acc_in, vals, fv, grid, s);
    }
}

template <int FMT>
hipError_t tails16_fmt(const RowTableNarrow& tab, int K, int64_t tile, int64_t tstride, const int64_t* idx, int64_t m,
                       const void* acc_in, void* vals, bool device, int fin, float fv, int grid, hipStream_t s) {
    if (device) {  // float16 only: bfloat16 has no single-rounding path in torch-ROCm
        if constexpr (FMT == FEDAVG_F16)
            return launch_tails_f<FMT, true>(tab, K, tile, tstride, idx, m, acc_in, vals, fin, fv, grid, s);
        else
            return hipErrorInvalidValue;
    }
    return launch_tails_f<FMT, false>(tab, K, tile, tstride, idx, m, acc_in, vals, fin, fv, grid, s);
}

template <int FMT, int OP, int FIN, bool ACC_IN>
static hipError_t launch_n_v(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, float fv,
                             int grid, bool vec, hipStream_t s) {
    if (vec) {
        hipLaunchKernelGGL((fedavg_rows_narrow<FMT, OP, FIN, ACC_IN, true>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const uint16_t*>(acc_in), static_cast<uint16_t*>(out), n, fv);
    } else {
        hipLaunchKernelGGL((fedavg_rows_narrow<FMT, OP, FIN, ACC_IN, false>), dim3(grid), dim3(kBlock), 0, s, tab, K,
                           static_cast<const uint16_t*>(acc_in), static_cast<uint16_t*>(out), n, fv);
    }
    return hipGetLastError();
}

template <int FMT, int OP, int FIN>
static hipError_t launch_n_a(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, float fv,
                             int grid, bool vec, hipStream_t s) {
    return acc_in ? launch_n_v<FMT, OP, FIN, true>(tab, K, acc_in, out, n, fv, grid, vec, s)
                  : launch_n_v<FMT, OP, FIN, false>(tab, K, acc_in, out, n, fv, grid, vec, s);
}

template <int FMT, int OP>
static hipError_t launch_n_f(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, int fin,
                             float fv, int grid, bool vec, hipStream_t s) {
    switch (fin) {
        case FEDAVG_FIN_SCALE:
            return launch_n_a<FMT, OP, FEDAVG_FIN_SCALE>(tab, K, acc_in, out, n, fv, grid, vec, s);
        case FEDAVG_FIN_DIV:
            return launch_n_a<FMT, OP, FEDAVG_FIN_DIV>(tab, K, acc_in, out, n, fv, grid, vec, s);
        default:
            return launch_n_a<FMT, OP, FEDAVG_FIN_NONE>(tab, K, acc_in, out, n, fv, grid, vec, s);
    }
}

template <int FMT>
static hipError_t launch_n_o(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, int op, int fin,
                             float fv, int grid, bool vec, hipStream_t s) {
    switch (op) {
        case FEDAVG_OP_TORCH_DEVICE:
        case FEDAVG_OP_TORCH:
            return launch_n_f<FMT, FEDAVG_OP_TORCH>(tab, K, acc_in, out, n, fin, fv, grid, vec, s);
        case FEDAVG_OP_UNWEIGHTED:
            return launch_n_f<FMT, FEDAVG_OP_UNWEIGHTED>(tab, K, acc_in, out, n, fin, fv, grid, vec, s);
        default:
            return launch_n_f<FMT, FEDAVG_OP_NUMPY>(tab, K, acc_in, out, n, fin, fv, grid, vec, s);
    }
}

template <int FMT>
hipError_t rows16_fmt(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, int op, int fin,
                      float fv, int grid, bool vec, hipStream_t s) {
    return launch_n_o<FMT>(tab, K, acc_in, out, n, op, fin, fv, grid, vec, s);
}

#define FEDAVG_NARROW_ENTRIES(PREFIX, FMT)                                                                             \
    PREFIX hipError_t tiles16_fmt<FMT>(const RowTableNarrow&, int, int64_t, const void*, void*, int64_t, int64_t, int, \
                                       int, float, int, int, hipStream_t, uint64_t*);                                 \
    PREFIX hipError_t rows16_fmt<FMT>(const RowTableNarrow&, int, const void*, void*, int64_t, int, int, float, int,   \
                                      bool, hipStream_t);                                                              \
    PREFIX hipError_t tails16_fmt<FMT>(const RowTableNarrow&, int, int64_t, int64_t, const int64_t*, int64_t,          \
                                       const void*, void*, bool, int, float, int, hipStream_t);
#if FEDAVG_NARROW_PART == 1
FEDAVG_NARROW_ENTRIES(extern template, FEDAVG_F16)  // in the float16 unit
#elif FEDAVG_NARROW_PART == 2
FEDAVG_NARROW_ENTRIES(template, FEDAVG_F16)
#endif
#undef FEDAVG_NARROW_ENTRIES

#if FEDAVG_NARROW_PART != 2  // the dispatchers, and the format-free scatter
hipError_t launch_tiles_narrow(const RowTableNarrow& tab, int K, int64_t tstride_elems, const void* acc_in, void* out,
                               int64_t begin, int64_t end, int fmt, int op, int fin, float fin_val, int grid,
                               int burst, hipStream_t s, uint64_t* nl) {
    const int64_t ts8 = tstride_elems / 8, b8 = begin / 8, e8 = end / 8;
    if (fmt == FEDAVG_BF16)
        return tiles16_fmt<FEDAVG_BF16>(tab, K, ts8, acc_in, out, b8, e8, op, fin, fin_val, grid, burst, s, nl);
    if (fmt == FEDAVG_F16)
        return tiles16_fmt<FEDAVG_F16>(tab, K, ts8, acc_in, out, b8, e8, op, fin, fin_val, grid, burst, s, nl);
    return hipErrorInvalidValue;
}

hipError_t launch_rows_narrow(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, int fmt,
                              int op, int fin, float fin_val, int grid, hipStream_t s) {
    bool vec = reinterpret_cast<uintptr_t>(out) % 16 == 0 && reinterpret_cast<uintptr_t>(acc_in) % 16 == 0;
    for (int k = 0; vec && k < K; ++k) vec = reinterpret_cast<uintptr_t>(tab.rows[k]) % 16 == 0;
    if (fmt == FEDAVG_BF16) return rows16_fmt<FEDAVG_BF16>(tab, K, acc_in, out, n, op, fin, fin_val, grid, vec, s);
    if (fmt == FEDAVG_F16) return rows16_fmt<FEDAVG_F16>(tab, K, acc_in, out, n, op, fin, fin_val, grid, vec, s);
    return hipErrorInvalidValue;
}

hipError_t launch_torch16_tails(const RowTableNarrow& tab, int K, int64_t tile, int64_t tstride, const int64_t* idx,
                                int64_t m, const void* acc_in, void* vals, int fmt, int op, int fin, float fin_val,
                                hipStream_t s) {
    const int grid = (int)((m + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    const bool device = op == FEDAVG_OP_TORCH_DEVICE;
    if (fmt == FEDAVG_BF16)
        return tails16_fmt<FEDAVG_BF16>(tab, K, tile, tstride, idx, m, acc_in, vals, device, fin, fin_val, grid, s);
    if (fmt == FEDAVG_F16)
        return tails16_fmt<FEDAVG_F16>(tab, K, tile, tstride, idx, m, acc_in, vals, device, fin, fin_val, grid, s);
    return hipErrorInvalidValue;
}

__global__ void __launch_bounds__(kBlock) fedavg_scatter16(const int64_t* idx, const uint16_t* vals, const int64_t m,
                                                            uint16_t* out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < m) out[idx[j]] = vals[j];
}

hipError_t launch_scatter16(const int64_t* idx, const void* vals, int64_t m, void* out, hipStream_t s) {
    const int grid = (int)((m + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(fedavg_scatter16, dim3(grid), dim3(kBlock), 0, s, idx, static_cast<const uint16_t*>(vals), m,
                       static_cast<uint16_t*>(out));
    return hipGetLastError();
}
#endif

}  // namespace fedavg
