// fedavg_arith.h -- per-element arithmetic of the reference, shared by the fp32 kernels (not installed).
// numpy / torch / unweighted steps and finalisations of weighted_aggregation_helper.py:181-236, the
// f32x4 forms, and the cache-policy load / store helpers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fedavg_internal.h"
#include "fedavg_rsqrt14.h"

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
// Division by a launch constant b: the plain and fused kernels' FIN_DIV (torch's total.div_(count), the correctly
// rounded quotient by the weight sum) and the fused optimizers' divisions by a bias correction (Adam's
// sqrt(v) / sqrt(bc2), NAdam's v / bc2, RAdam's m / bc1).  Instead of the IEEE division sequence per element (v_div_scale x 2, v_rcp, four FMAs,
// v_div_fmas, v_div_fixup) it takes Markstein's correction from the correctly rounded reciprocal, computed once per
// thread:  r = RN(1 / b);  q = RN(a r);  e = fma(-q, b, a) (exact);  a / b = RN(q + e r).  Checked against the IEEE
// division for every pair of significands (2^23 dividends x 2^23 divisors, tools/div_const_probe.py); away from
// underflow and overflow the result depends on the significands only, so the fast path runs where 2^-20 <= b <= 2^20
// (every weight sum of a FedAvg round in practice; a uniform flag) and |a| in [2^-100, 2^100) (exponent field 27..226),
// which keeps q, e r and every intermediate normal; zeros, subnormals, huge values, inf and NaN take the IEEE division,
// a branch the waves skip unless one of their lanes needs it.
// ---------------------------------------------------------------------------------------------
struct FinConst {
    float v;     // the finalisation scalar (FIN_SCALE: 1 / count as the reference rounds it; FIN_DIV: count), or divisor
    float r;     // divisor: RN(1 / v)
    bool fast;   // divisor in [2^-20, 2^20]
};

__device__ __forceinline__ FinConst div_const_init(const float v) {
    return FinConst{v, 1.0f / v, v >= 0x1p-20f && v <= 0x1p20f};
}

template <int FIN>
__device__ __forceinline__ FinConst fin_const(const float v) {
    if constexpr (FIN == FEDAVG_FIN_DIV) return div_const_init(v);
    return FinConst{v, 0.0f, false};
}

__device__ __forceinline__ float div_const(const float a, const FinConst& f) {
#if defined(FEDAVG_AB_IEEE_DIV)  // A/B builds only (tools/build_rev_lib.py -D): the IEEE division everywhere
    return a / f.v;
#endif
    const float q = a * f.r;
    const float e = __builtin_fmaf(-q, f.v, a);
    float res = __builtin_fmaf(e, f.r, q);
    const uint32_t ea = (__float_as_uint(a) >> 23) & 0xFFu;
    if (__builtin_expect(!f.fast || ea - 27u >= 200u, 0)) res = a / f.v;
    return res;
}

template <int FIN>
__device__ __forceinline__ f32x4 fin4c(const f32x4 a, const FinConst& f) {
    if constexpr (FIN == FEDAVG_FIN_DIV) {
        return f32x4{div_const(a[0], f), div_const(a[1], f), div_const(a[2], f), div_const(a[3], f)};
    } else {
        return fin4<FIN>(a, f.v);
    }
}

// div_const's fast path with its range check folded into `slow` (non-zero: some input left [2^-100, 2^100) or the
// divisor is not fast); the caller recomputes a whole group with the exact form when it is set, so a group of
// quotients is straight-line code with one branch after it instead of one per element (round 5: a branch is a
// basic-block boundary the scheduler does not hoist loads across)
__device__ __forceinline__ float div_const_fast(const float a, const FinConst& f, uint32_t& slow) {
#if defined(FEDAVG_AB_IEEE_DIV)
    return a / f.v;
#endif
    const float q = a * f.r;
    const float e = __builtin_fmaf(-q, f.v, a);
    slow |= (uint32_t)(((__float_as_uint(a) >> 23) & 0xFFu) - 27u >= 200u);
    return __builtin_fmaf(e, f.r, q);
}

// div_const_fast with +0 on the fast form -- the epilogues' quotients (fedavg_epi.h div_x): q = +-0, e = +0 and the
// result 0 with the divisor's sign, as a / v (-0 stays rare: the form returns +0 for -0 / v, v > 0).  A frozen
// parameter (every client's update exactly 0) keeps Adam's exp_avg at 0, and its unit would otherwise recompute per
// element on every step (round 6: the LDS-DMA form at 1 / 2 / 3 clients with half the parameters frozen 61.5 / 66.8 /
// 55.9 % of HBM, live 75.3 / 73.9 / 78.7 %; profiles/r06/s20/).  The aggregation's own FIN_DIV (fin_tile) keeps the
// one-compare form: a zero sum there costs only its group's IEEE divisions, and the plain few-client kernel lost 3
// points to the extra compare (79.3 -> 76.2 % at 2 clients, s20).
__device__ __forceinline__ float div_const_fast_z(const float a, const FinConst& f, uint32_t& slow) {
#if defined(FEDAVG_AB_IEEE_DIV)
    return a / f.v;
#endif
    const float q = a * f.r;
    const float e = __builtin_fmaf(-q, f.v, a);
    const uint32_t ab = __float_as_uint(a);
    slow |= (uint32_t)(((ab >> 23) & 0xFFu) - 27u >= 200u && ab != 0u);
    return __builtin_fmaf(e, f.r, q);
}

// A lane's rare-case flag made wave-uniform: the recompute then runs on every lane of the wave (each rare-case form is
// bit-identical to its fast form) behind a scalar branch, with no exec mask to restore at the join.  With the branch
// divergent, hipcc placed the register allocator's copy of a held result (a VGPR -> AGPR move) in the join block BEFORE
// its exec restore, behind SGPR-spill writelanes: the lanes that had skipped the branch never got the value (round 6,
// session 22: the LDS-DMA Adam form at 3 clients lost unit 14's parameter in every wave, tools/r06/diag_u14.py).
__device__ __forceinline__ bool wave_any(const uint32_t slow) { return __builtin_amdgcn_ballot_w64(slow != 0u) != 0; }

// fin4c over a lane's CPL columns of one tile, with one rare-case branch for all of them (div_const_fast)
template <int FIN, int CPL>
__device__ __forceinline__ void fin_tile(f32x4 (&r)[CPL], const f32x4 (&a)[CPL], const FinConst& f) {
    if constexpr (FIN == FEDAVG_FIN_DIV) {
        uint32_t slow = f.fast ? 0u : 1u;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) r[c][j] = div_const_fast(a[c][j], f, slow);
        if (__builtin_expect(wave_any(slow), 0)) {
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j) r[c][j] = a[c][j] / f.v;
        }
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) r[c] = fin4<FIN>(a[c], f.v);
    }
}

// One tile's arrival-ordered sum for the CPL float4 columns this lane owns: acc = ACC_IN ? acc_in : first(client
// 0), then step(client k) for every later client, UNROLL clients' loads issued before their arithmetic.  Client
// rows are tiled (row + off is this lane's first column of the tile); acc_in is indexed by global column and
// masked to [b4, e4).
// GROUPED (1 or 2): every load group holds UNROLL clients from client 0 on (the first client's operation applied in
// the first group), so a tile takes ceil(K / UNROLL) load round trips instead of 1 + (K-1) / UNROLL + the
// remainder.  GROUPED = 1: a partial last group loads only its real clients (wave-uniform branches per slot);
// GROUPED = 2 (round 3): the missing slots re-load the last client, branch-free (at 5 or 6 clients a third of a
// tile's loads are such repeats).
template <int OP, bool ACC_IN, int UNROLL, int CPL, int GROUPED = 0>
__device__ __forceinline__ void tile_sum(f32x4 (&acc)[CPL], const RowTableF32& tab, const int K, const int64_t off,
                                         const int64_t col, const f32x4* acc_in, const int64_t b4, const int64_t e4) {
    if constexpr (GROUPED != 0) {
        if constexpr (ACC_IN) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = col + c * kBlock;
                acc[c] = (i >= b4 && i < e4) ? acc_in[i] : f32x4{0, 0, 0, 0};
            }
        }
        for (int k = 0; k < K; k += UNROLL) {
            f32x4 v[UNROLL][CPL];
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                if constexpr (GROUPED == 2) {
                    const f32x4* r = tab.rows[k + j < K ? k + j : K - 1] + off;
#pragma unroll
                    for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(r + c * kBlock);
                } else if (j == 0 || k + j < K) {  // uniform: only a partial last group skips slots
                    const f32x4* r = tab.rows[k + j] + off;
#pragma unroll
                    for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(r + c * kBlock);
                }
            }
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                if (k + j < K) {
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
        return;
    }
    int k = 0;
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            acc[c] = (i >= b4 && i < e4) ? acc_in[i] : f32x4{0, 0, 0, 0};
        }
    } else {
        const f32x4* r = tab.rows[0] + off;
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(__builtin_nontemporal_load(r + c * kBlock), tab.w[0]);
        k = 1;
    }
    for (; k + UNROLL <= K; k += UNROLL) {
        f32x4 v[UNROLL][CPL];
#pragma unroll
        for (int j = 0; j < UNROLL; ++j) {
            const f32x4* r = tab.rows[k + j] + off;
#pragma unroll
            for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(r + c * kBlock);
        }
#pragma unroll
        for (int j = 0; j < UNROLL; ++j)
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[k + j]);
    }
    for (; k < K; ++k) {
        const f32x4* r = tab.rows[k] + off;
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], __builtin_nontemporal_load(r + c * kBlock), tab.w[k]);
    }
}

// a chained partial sum's column i, or zero outside [b4, e4): the load is unconditional (an in-range clamped address),
// so it adds no control flow to the tile loop
__device__ __forceinline__ f32x4 load_acc_in(const f32x4* acc_in, const int64_t i, const int64_t b4, const int64_t e4) {
    const int64_t j = i < b4 ? b4 : (i >= e4 ? e4 - 1 : i);
    const f32x4 v = __builtin_nontemporal_load(acc_in + j);
    return (i >= b4 && i < e4) ? v : f32x4{0, 0, 0, 0};
}

// client k's operation on this lane's columns: first4 for client 0 unless ACC_IN, step4 otherwise
template <int OP, bool ACC_IN, int CPL>
__device__ __forceinline__ void client_apply(f32x4 (&acc)[CPL], const RowTableF32& tab, const int k, const f32x4 (&v)[CPL]) {
    const float w = tab.w[k];
    if (!ACC_IN && k == 0) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(v[c], w);
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[c], w);
    }
}

// N clients from client k on: the N rows' loads issued together, then their arithmetic in arrival order (client 0's
// operation is first4 unless ACC_IN)
template <int OP, bool ACC_IN, int N, int CPL>
__device__ __forceinline__ void client_group(f32x4 (&acc)[CPL], const RowTableF32& tab, const int k, const int64_t off) {
    f32x4 v[N][CPL];
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
        for (int c = 0; c < CPL; ++c) v[j][c] = __builtin_nontemporal_load(tab.rows[k + j] + off + c * kBlock);
#pragma unroll
    for (int j = 0; j < N; ++j) client_apply<OP, ACC_IN>(acc, tab, k + j, v[j]);
}

// Shapes of the fused kernels' four-client group (A/B only: launch variant bits 9-11, fedavg_epi.h): 0 -- the four
// clients' loads together (client_group<4>, the default); 2 -- two pairs, the second pair's loads issued after the
// first pair's arithmetic; 3 -- clients 0, 2 and 3 of the group, then client 1 after client 0's arithmetic (the order
// round 3's GROUPED loop compiled to); 4 -- one client at a time.  fence(): a value the next loads must wait for.
template <int CPL>
__device__ __forceinline__ void fence_on(const f32x4 (&acc)[CPL]) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) asm volatile("" ::"v"(acc[c]) : "memory");  // every column: no arithmetic deferred past it
}

template <int OP, bool ACC_IN, int SHAPE, int CPL>
__device__ __forceinline__ void client_group4(f32x4 (&acc)[CPL], const RowTableF32& tab, const int k, const int64_t off) {
    if constexpr (SHAPE == 2) {
        client_group<OP, ACC_IN, 2, CPL>(acc, tab, k, off);
        fence_on(acc);
        client_group<OP, ACC_IN, 2, CPL>(acc, tab, k + 2, off);
    } else if constexpr (SHAPE == 3) {
        f32x4 v0[CPL], v1[CPL], v2[CPL], v3[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            v0[c] = __builtin_nontemporal_load(tab.rows[k] + off + c * kBlock);
            v2[c] = __builtin_nontemporal_load(tab.rows[k + 2] + off + c * kBlock);
            v3[c] = __builtin_nontemporal_load(tab.rows[k + 3] + off + c * kBlock);
        }
        client_apply<OP, ACC_IN>(acc, tab, k, v0);
        fence_on(acc);
#pragma unroll
        for (int c = 0; c < CPL; ++c) v1[c] = __builtin_nontemporal_load(tab.rows[k + 1] + off + c * kBlock);
        client_apply<OP, ACC_IN>(acc, tab, k + 1, v1);
        client_apply<OP, ACC_IN>(acc, tab, k + 2, v2);
        client_apply<OP, ACC_IN>(acc, tab, k + 3, v3);
    } else if constexpr (SHAPE == 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            client_group<OP, ACC_IN, 1, CPL>(acc, tab, k + j, off);
            if (j < 3) fence_on(acc);
        }
    } else {
        client_group<OP, ACC_IN, 4, CPL>(acc, tab, k, off);
    }
}

// The fused kernels' tile sum (round 4): groups of 4 clients in a loop with unconditional loads, then the K mod 4
// remainder as one group of exactly that many clients, chosen by a wave-uniform branch per tile -- no repeated loads
// for any K, in one instantiation (the plain kernels build the client count or its remainder into the kernel
// instead: fedavg_tiles.h tile_sum_kc / tile_sum_rem).  SHAPE -1 (default): the groups' loads as two pairs from two
// full groups on, four together below (fedavg_tiles.h tile_sum_rem has the measurements); SHAPE >= 0 forces
// client_group4's shape (A/B).
template <int OP, bool ACC_IN, int CPL, int SHAPE = -1>
__device__ __forceinline__ void tile_sum_rrem(f32x4 (&acc)[CPL], const RowTableF32& tab, const int K, const int64_t off,
                                              const int64_t col, const f32x4* acc_in, const int64_t b4, const int64_t e4) {
    if constexpr (ACC_IN) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] = load_acc_in(acc_in, col + c * kBlock, b4, e4);
    }
    const int rem = K & 3;
    const int k_full = K - rem;
    if constexpr (SHAPE >= 0) {
        for (int k = 0; k < k_full; k += 4) client_group4<OP, ACC_IN, SHAPE, CPL>(acc, tab, k, off);
    } else if (k_full >= 8) {  // uniform
        for (int k = 0; k < k_full; k += 4) client_group4<OP, ACC_IN, 2, CPL>(acc, tab, k, off);
    } else {
        for (int k = 0; k < k_full; k += 4) client_group4<OP, ACC_IN, 0, CPL>(acc, tab, k, off);
    }
    if (rem == 3) {
        client_group<OP, ACC_IN, 3, CPL>(acc, tab, k_full, off);
    } else if (rem == 2) {
        client_group<OP, ACC_IN, 2, CPL>(acc, tab, k_full, off);
    } else if (rem == 1) {
        client_group<OP, ACC_IN, 1, CPL>(acc, tab, k_full, off);
    }
}

// torch CPU's fp32 Tensor.sqrt (the epilogues' sqrt when EpiParams.torch_sqrt is set, fedavg_epi.h sqrt_e): MKL VML
// vsSqrt on AVX-512 (ATen vml.h IMPLEMENT_VML_MKL(sqrt, Sqrt), VML_HA), which is not correctly rounded but one Newton
// step from the VRSQRT14PS estimate (measured bit-exact against torch over every mantissa of [1, 4), every subnormal
// and a sample of every binade: tools/sqrt_probe.py; restated in oracle_sqrt_torch_cpu):
//     y = rsqrt14(x);  s = x * y;  r = fma(-s, s, x);  sqrt = fma(r, 0.5 * y, s)
// rsqrt14 depends on the exponent parity and the top 15 mantissa bits; mantissa bits 22..7 of the estimate for x in
// [1, 4) are 32 exact fixed-point lines per parity (fedavg_rsqrt14.h, generated from the captured instruction table
// nvflare_amd/data/rsqrt14_avx512.bin), a power of four giving its exact root.  Inputs below 2^-96 run at x * 2^64
// and are scaled back by 2^-32 (no subnormal residual); 0, inf, NaN and negatives take the correctly rounded sqrt
// (a branch the waves skip unless a lane needs it: the raw v_sqrt_f32 it replaced flushed negative subnormals to -0
// where torch returns NaN -- tools/sqrt_device_exhaustive.py over all 2^32 inputs).  Per sqrt one 8-byte LDS read of
// the staged segment table (rsqrt14_stage) and one integer multiply-add.  (The first form gathered 2 bytes per sqrt from a 128 KiB device table: fused Adam at config 5 ran
// 81.3 % of HBM peak against 87.3 % with the correctly rounded sqrt; the same segments read from global memory,
// 83.3 %: profiles/r03/s4, s5.)
__shared__ uint2 g_rsqrt14_lds[64];  // {kRsqrt14Base, kRsqrt14Slope}[segment]

// every kernel that computes sqrt_torch_cpu calls this first, with the whole block (one barrier)
__device__ __forceinline__ void rsqrt14_stage() {
    if (threadIdx.x < 64) g_rsqrt14_lds[threadIdx.x] = uint2{kRsqrt14Base[threadIdx.x], kRsqrt14Slope[threadIdx.x]};
    __syncthreads();
}

__device__ __forceinline__ float sqrt_torch_cpu(const float x) {
    const bool special = !(x > 0.0f) || x == __builtin_inff();
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p64f : x;
    const uint32_t b = __float_as_uint(xs);
    const int e = (int)(b >> 23) - 127;
    const uint32_t m = b & 0x7FFFFFu;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint2 ab = g_rsqrt14_lds[(((uint32_t)p << 5) | (m >> 18)) & 63u];
    const uint32_t y16 = (ab.x - ab.y * ((m >> 8) & 1023u)) >> 10;
    const uint32_t yb = (p == 0 && m == 0) ? 0x3F800000u : (0x3F000000u | (y16 << 7));
    const float y = __uint_as_float((uint32_t)((int32_t)yb - k * 8388608));
    const float s = xs * y;
    const float r = __builtin_fmaf(-s, s, xs);
    const float res = __builtin_fmaf(r, 0.5f * y, s);
    float out = tiny ? res * 0x1p-32f : res;
    if (__builtin_expect(special, 0)) out = __builtin_sqrtf(x);
    return out;
}

// sqrt_torch_cpu without its special-input branch: `slow` set where it would have taken the callout (the caller then
// recomputes the group with sqrt_torch_cpu)
__device__ __forceinline__ float sqrt_torch_cpu_fast(const float x, uint32_t& slow) {
    // the callout for -0, negatives, inf and NaN; +0 runs the refinement (xs = 0, a finite estimate: s = r = res = +0)
    slow |= (uint32_t)(__float_as_uint(x) >= 0x7F800000u);
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p64f : x;
    const uint32_t b = __float_as_uint(xs);
    const int e = (int)(b >> 23) - 127;
    const uint32_t m = b & 0x7FFFFFu;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint2 ab = g_rsqrt14_lds[(((uint32_t)p << 5) | (m >> 18)) & 63u];
    const uint32_t y16 = (ab.x - ab.y * ((m >> 8) & 1023u)) >> 10;
    const uint32_t yb = (p == 0 && m == 0) ? 0x3F800000u : (0x3F000000u | (y16 << 7));
    const float y = __uint_as_float((uint32_t)((int32_t)yb - k * 8388608));
    const float s = xs * y;
    const float r = __builtin_fmaf(-s, s, xs);
    const float res = __builtin_fmaf(r, 0.5f * y, s);
    return tiny ? res * 0x1p-32f : res;
}

// torch CPU's fp32 Tensor.sqrt on hosts where MKL takes vsSqrt's SSE4.2 / AVX kernel -- the GPU pool's AMD EPYC hosts
// (EpiParams.torch_sqrt == FEDAVG_SQRT_TORCH_AMD; mkl_vml_kernel_sSqrt_EXHAynn, equal to torch.sqrt on all 59.8 M probe
// inputs on the box, tools/sqrt_box_kernels.py), which starts a coupled Newton step in plain fp32 -- every operation
// rounds, no FMA (-ffp-contract=off) -- from the RSQRTPS estimate:
//     y = rsqrtps(x);  s = x * y;  h = y * 0.5;  r = 0.5 - s * h;  s1 = s * r + s;  h1 = h * r + h;
//     sqrt = (x - s1 * s1) * h1 + s1
// on positive normals up to 0x7f7ff000; every other input takes the kernel's correctly rounded scalar callout.
// RSQRTPS is vendor-specific: the HOST CPU's estimates (12 bits, a function of the exponent parity and the top 12
// mantissa bits), captured at run time by fedavg_host_rsqrtps_table and uploaded by fedavg_set_rsqrtps_table (8192
// entries, two per word, EpiParams.rsqrtps), are staged in LDS once per block (rsqrtps_stage, 16 KiB); each sqrt reads
// one 16-bit entry.  Restated in oracle_sqrt_mkl_rsqrtps: with this container's RSQRTPS it equals MKL's EX kernel on
// all 2^32 inputs, with the box's table the box's torch.sqrt on all 2^32 inputs (tools/sqrt_mkl_sse_check.py,
// profiles/r03/final/sqrt_check_torch_all.log).
__shared__ uint32_t g_rsqrtps_lds[4096];  // two 12-bit estimates per word (low half first)

// every kernel that computes sqrt_mkl_rsqrtps calls this first, with the whole block (one barrier)
__device__ __forceinline__ void rsqrtps_stage(const uint32_t* table) {
    const uint4* src = reinterpret_cast<const uint4*>(table);
    uint4* dst = reinterpret_cast<uint4*>(g_rsqrtps_lds);
    for (int i = threadIdx.x; i < 1024; i += kBlock) dst[i] = src[i];
    __syncthreads();
}

__device__ __forceinline__ float sqrt_mkl_rsqrtps(const float x) {
    const uint32_t b = __float_as_uint(x);
    const int e = (int)((b >> 23) & 0xFFu) - 127;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint32_t t = reinterpret_cast<const uint16_t*>(g_rsqrtps_lds)[((uint32_t)p << 12) | ((b & 0x7FFFFFu) >> 11)];
    const float y = __uint_as_float((0x3F000000u | (t << 11)) - (uint32_t)(k * 8388608));
    const float s = x * y;
    const float h = y * 0.5f;
    const float r = 0.5f - s * h;
    const float s1 = s * r + s;
    const float h1 = h * r + h;
    float res = (x - s1 * s1) * h1 + s1;
    // the callout (zero, subnormals, the top 4095 finite values, inf, NaN, negatives) as a branch the waves skip
    // unless one of their lanes needs it: the correctly rounded sqrt is more instructions than the refinement
    if (__builtin_expect(b - 0x00800000u > 0x7F7FF000u - 0x00800000u, 0)) res = __builtin_sqrtf(x);
    return res;
}

// sqrt_mkl_rsqrtps without its callout branch: `slow` set where it would have been taken (the caller then recomputes
// the group with sqrt_mkl_rsqrtps)
__device__ __forceinline__ float sqrt_mkl_rsqrtps_fast(const float x, uint32_t& slow) {
    const uint32_t b = __float_as_uint(x);
    // the callout for subnormals, the top finite values, inf, NaN, negatives and -0; +0 runs the refinement (a finite
    // estimate for exponent -127: s = s1 = res = +0), so a frozen parameter's zero exp_avg_sq stays on the fast form
    // (v_cmp_class for +subnormals (class bit 7), one unsigned compare for the top finite values, +inf, NaN and every
    // negative -0 included: as many VALU compares as the range test that also sent +0 to the callout)
    slow |= (uint32_t)(__builtin_amdgcn_class(x, 0x080) || b > 0x7F7FF000u);
    const int e = (int)((b >> 23) & 0xFFu) - 127;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint32_t t = reinterpret_cast<const uint16_t*>(g_rsqrtps_lds)[((uint32_t)p << 12) | ((b & 0x7FFFFFu) >> 11)];
    const float y = __uint_as_float((0x3F000000u | (t << 11)) - (uint32_t)(k * 8388608));
    const float s = x * y;
    const float h = y * 0.5f;
    const float r = 0.5f - s * h;
    const float s1 = s * r + s;
    const float h1 = h * r + h;
    return (x - s1 * s1) * h1 + s1;
}

}  // namespace fedavg
