// fedavg_internal.h -- shared between the HIP kernels and the C-ABI layer (not installed).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nvflare_amd_fedavg.h"

namespace fedavg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;             // 4 waves of 64 lanes
constexpr int kMaxRowsPerLaunch = 128;  // clients per launch carried in the kernel-argument segment

// launch defaults, from the MI355X sweeps recorded in profiles/r01
constexpr int kDefaultTile = 4096;      // elements per client segment per tile (16 KiB)
constexpr int kDefaultBlocksPerCu = 2;  // 8 waves per CU (per-tile-store, epilogue, fp64 and 16-bit kernels)
constexpr int kDefaultUnroll = 4;       // clients whose loads are in flight together per lane

// The product library carries only the kernel forms the launchers route to (round 5); the A/B
// forms -- other tile widths and unrolls, temporal loads / stores, register-only burst forms, the round-3 client loop,
// client-loop shapes, the per-tile forms of the 16-bit and fp64 kernels -- are compiled only with -DFEDAVG_AB
// (tools/build_rev_lib.py), where fedavg_set_variant / set_launch / set_tile accept them.
#if defined(FEDAVG_AB)
constexpr bool kAB = true;
#else
constexpr bool kAB = false;
#endif
// -DFEDAVG_AB_FEW: a product library plus the few-client forms' geometry sweep only (launch variant bits 9-11 for 1-2
// client reads, kFewAB) -- a product-sized A/B build (tools/build_rev_lib.py --product -D FEDAVG_AB_FEW)
#if defined(FEDAVG_AB) || defined(FEDAVG_AB_FEW)
constexpr bool kABFew = true;
#else
constexpr bool kABFew = false;
#endif

// variant bits (fedavg_set_variant).  Default (0): the plain aggregation runs fedavg_tiles_burst_f32x4.
constexpr int kVariantTemporalLoads = 1;   // per-tile-store kernel with temporal (cached) client loads
constexpr int kVariantTemporalStores = 2;  // per-tile-store kernel with temporal result stores
constexpr int kVariantEpiPrefetch = 4;     // epilogue kernel: software-pipelined across tiles (see fedavg_tiles_epi_f32x4)
constexpr int kVariantTileStores = 8;      // plain aggregation on fedavg_tiles_f32x4 (each tile's results stored
                                           // when it finishes; implied by bits 0 and 1)
constexpr int kVariantAnyOrder = 16;       // burst launches after an aggregation's first go without the AQL barrier
                                           // bit (hipExtAnyOrderLaunch): launch i+1's blocks fill CUs as launch i
                                           // drains; they touch disjoint tiles, and the next ordinary packet waits
constexpr int kVariantRegisterTiles = 32;  // plain burst kernel without its kBurstLdsTiles LDS-held tiles (by default
                                           // each block also holds 4 tiles' results in LDS: 1.5x longer launches,
                                           // +0.3 to +1.5 points at 8-64 clients, profiles/r02/ab/lds_tiles/)
constexpr int kVariantWideLds = 64;       // inside TileLaunch: plain burst kernel with kBurstLdsTilesWide LDS-held tiles
                                           // (160 KiB, one block per CU); run_tiles sets it for one-block-per-CU grids
                                           // unless the public variant has bit 6, which keeps the 4-tile form there
                                           // (32 clients 88.4 -> 88.9 %, 64: 89.7 -> 89.9 %, profiles/r02/ab/wide_lds/)
constexpr int kVariantLoopShift = 9;       // bits 9-11: A/B shapes of the burst kernels' client loop
                                           // (fedavg_epi.h launch_epi_loop_ab, fedavg_tiles.h launch_burst)
constexpr int kVariantFew = 1 << 12;      // inside TileLaunch: the few-client burst kernel (fedavg_tiles.h
                                           // fedavg_tiles_few_f32x4), set by run_tiles for 1-2 reads, no chained sum
constexpr int kVariantEpiDma = 1 << 14;   // inside TileLaunch: the LDS-DMA few-client fused form (fedavg_epi.h
                                           // fedavg_tiles_epi_dma_f32x4), set by the C-ABI for 1-3 reads, no chained
                                           // sum, every kind (RMSprop centered only with momentum); public bit 2 (the
                                           // per-tile pipelined form) keeps the round-5 route for same-process A/Bs
constexpr int kVariantEpiNoSplit = 1 << 15;  // fused Adam at one block per CU (64+ clients) on round 5's burst form
                                              // instead of the split-epilogue form (fedavg_epi.h
                                              // fedavg_tiles_epi_split_f32x4): a product-build A/B switch
// public variant bits a product build accepts (fedavg_set_variant): the fused per-tile pipelined form (2), burst
// launches without the barrier bit (16), the 4-LDS-tile form on one-block-per-CU grids (64), the fused burst form
// without the split epilogue (1 << 15) -- each a routed form
constexpr int kVariantProductMask = kVariantEpiPrefetch | kVariantAnyOrder | kVariantWideLds | kVariantEpiNoSplit;
// epilogue template value: the optimizer kind | kEpiTorchSqrt when the step's sqrt is torch CPU's restated AVX-512
// vsSqrt (EpiParams.torch_sqrt == FEDAVG_SQRT_TORCH_AVX512; fedavg_arith.h sqrt_torch_cpu) | kEpiTorchSqrtAmd for the
// AMD hosts' path (FEDAVG_SQRT_TORCH_AMD; sqrt_mkl_rsqrtps) -- a compile-time choice, so the correctly rounded path
// keeps its own code (a runtime branch cost the fused Adam kernel 9 points, profiles/r03/s3/)
constexpr int kEpiTorchSqrt = 0x100;
constexpr int kEpiTorchSqrtAmd = 0x200;
constexpr int kEpiSqrtMask = kEpiTorchSqrt | kEpiTorchSqrtAmd;
constexpr int kBurstLdsTilesWide = 10;     // 10 x 16 KiB = all of a CU's LDS
constexpr int kBurstEpiLdsTilesWide = 9;   // fused form at one block per CU: 9 x 16 KiB (+ a sqrt table: 512 B / 16 KiB)
constexpr int kBurstTiles = 8;             // tiles per block per burst launch (results held in registers)
constexpr int kBurstLdsTiles = 4;          // 4 x 16 KiB of LDS per block (2 blocks fit a CU)

// Per-launch client table passed BY VALUE in the kernarg segment: wave-uniform base pointers and
// weights are loaded with s_load into SGPRs.
struct RowTableF32 {
    const f32x4* rows[kMaxRowsPerLaunch];
    float w[kMaxRowsPerLaunch];
};

struct RowTableGeneric {
    const void* rows[kMaxRowsPerLaunch];
    double w[kMaxRowsPerLaunch];
};

// 16-bit accumulators (fedavg_narrow.hip): per-client weight of the first operation and of the later
// steps, both already rounded on the host the way the reference library rounds them (fp32 values).
struct RowTableNarrow {
    const void* rows[kMaxRowsPerLaunch];
    float w_first[kMaxRowsPerLaunch];
    float w_step[kMaxRowsPerLaunch];
};

struct TileLaunch {
    RowTableF32 tab;
    int k;
    int op, fin;
    int unroll, variant;
    int grid;
    int64_t tile4;     // tile width, f32x4 units
    int64_t tstride4;  // tile stride of every client's storage, f32x4 units
    int64_t b4, e4;    // global f32x4 range
    const float* acc_in;
    float* out;
    float fin_val;
};

// Epilogue scalars, precomputed on the host exactly as torch computes them (python fp64, cast to fp32
// where they meet a tensor) -- see fedavg_capi.cpp make_epi().
struct EpiParams {
    int kind;
    int first_step, nesterov, maximize, decoupled_weight_decay, has_weight_decay, has_momentum;
    float weight_decay, momentum, one_minus_dampening, neg_lr;                  // SGD
    float decoupled_scale, one_minus_beta1, one_minus_beta1_m1, one_minus_beta2; // Adam
    float beta2, step_size_neg, bias_correction2_sqrt, eps;
    float* param;
    float* state1;  // SGD momentum buffer / Adam exp_avg
    float* state2;  // Adam exp_avg_sq
    const float* base;
    int amsgrad;
    float* state3;  // Adam amsgrad: max_exp_avg_sq | RMSprop centered: grad_avg
    int centered;   // RMSprop (alpha in beta2 / one_minus_beta2 / one_minus_beta1)
    float bias_correction2, coef_grad, coef_avg;  // NAdam: the two addcdiv values
    float bias_correction1, lr, rect;             // RAdam
    int rectified;                                // RAdam: rho_t > 5
    float etaminus, etaplus, ss_min, ss_max;      // Rprop
    float decay, neg_eta, mu;                     // ASGD: 1 - lambd * eta, -eta, mu (averaging when != 1)
    int torch_sqrt;                               // FEDAVG_SQRT_*: torch CPU's sqrt (Intel / AMD host), or IEEE
    const uint32_t* rsqrtps;                      // FEDAVG_SQRT_TORCH_AMD: this host's RSQRTPS table (device, 16 KiB)
};

// operand streams the LDS-DMA few-client fused form (fedavg_epi.h fedavg_tiles_epi_dma_f32x4) reads for this kind and
// step, or 0 when it does not take them (the C-ABI then routes the per-tile form)
// k: client reads.  Adam with amsgrad takes the form at 3 reads only: 65.7 / 72.2 / 76.2 % of HBM at 1 / 2 / 3 clients
// against the per-tile form's 72.0 / 72.9 / 70.2 % (profiles/r06/s26/; 4 waves x 24 units, not swept)
inline int epi_dma_nin(const EpiParams& E, const int k) {
    switch (E.kind) {
        case FEDAVG_EPI_ADD_BASE: return 1;
        case FEDAVG_EPI_SGD: return (E.has_momentum && !E.first_step) ? 2 : 1;
        case FEDAVG_EPI_ADAM: return E.amsgrad ? (k == 3 ? 4 : 0) : 3;  // p, exp_avg, exp_avg_sq (, max_exp_avg_sq)
        case FEDAVG_EPI_NADAM:
        case FEDAVG_EPI_RADAM:
        case FEDAVG_EPI_ADAMAX:
        case FEDAVG_EPI_RPROP: return 3;  // p and two states
        case FEDAVG_EPI_ADAGRAD:
        case FEDAVG_EPI_ASGD: return 2;  // p and one state
        // RMSprop: p, square_avg (, momentum buffer (, grad_avg)); centered without momentum would read state3 as the
        // third stream: the per-tile form
        case FEDAVG_EPI_RMSPROP: return E.centered ? (E.has_momentum ? 4 : 0) : E.has_momentum ? 3 : 2;
        default: return 0;
    }
}

struct DequantLaunch {
    int qtype;
    const void* q;
    int64_t n;
    const float* absmax;
    const float* code;
    int64_t blocksize;
    double norm, level, offset;
    int has_norm;
    float* out;
    int64_t tile, tstride, elem0;
    int grid;
};

// launch_count (optional): incremented by the number of kernel launches issued
hipError_t launch_tiles_f32x4(const TileLaunch& L, hipStream_t s, uint64_t* launch_count = nullptr);

// Host loop of a BURST kernel (fedavg_tiles.h): one launch per grid x tpb tiles of [t_first, t_stop), every
// block holding its tpb tiles' results until the end of its launch; launch(blocks, t0, t_end, flags) issues
// one with hipExtLaunchKernel flags: 0 for the first, hipExtAnyOrderLaunch for the rest when any_order (the
// first keeps the barrier bit, so it waits for the staging copies; the launches of one call touch disjoint tiles).
template <typename Launch>
inline hipError_t burst_launches(int64_t t_first, int64_t t_stop, int grid, int tpb, uint64_t* launch_count,
                                 bool any_order, Launch&& launch) {
    const int64_t per = (int64_t)grid * tpb;
    for (int64_t t0 = t_first; t0 < t_stop; t0 += per) {
        const int64_t t_end = t0 + per < t_stop ? t0 + per : t_stop;
        launch((int)(t_end - t0 < grid ? t_end - t0 : grid), t0, t_end,
               (any_order && t0 != t_first) ? (uint32_t)hipExtAnyOrderLaunch : 0u);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (launch_count) ++*launch_count;
    }
    return hipSuccess;
}
// per-mode instantiations (fedavg_tiles_*.hip, fedavg_epi_*.hip), dispatched on L.op by the two above
hipError_t launch_tiles_f32x4_numpy(const TileLaunch& L, hipStream_t s, uint64_t* launch_count);
hipError_t launch_tiles_f32x4_torch(const TileLaunch& L, hipStream_t s, uint64_t* launch_count);
hipError_t launch_tiles_f32x4_unweighted(const TileLaunch& L, hipStream_t s, uint64_t* launch_count);
// fused kernels, one entry per (mode, finalisation): fedavg_epi_inst.hip compiled once per pair (nine A/B builds, the
// five of epi_direct in product builds, plus launch_epi_step there: the server step alone, no clients, FIN_NONE)
#define FEDAVG_EPI_DECL(name) \
    hipError_t name(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl);
FEDAVG_EPI_DECL(launch_epi_step)
FEDAVG_EPI_DECL(launch_epi_numpy_none)
FEDAVG_EPI_DECL(launch_epi_numpy_scale)
FEDAVG_EPI_DECL(launch_epi_numpy_div)
FEDAVG_EPI_DECL(launch_epi_torch_none)
FEDAVG_EPI_DECL(launch_epi_torch_scale)
FEDAVG_EPI_DECL(launch_epi_torch_div)
FEDAVG_EPI_DECL(launch_epi_unweighted_none)
FEDAVG_EPI_DECL(launch_epi_unweighted_scale)
FEDAVG_EPI_DECL(launch_epi_unweighted_div)
#undef FEDAVG_EPI_DECL
// Whether a fused launch (clients + epilogue in one kernel) is in this build.  Product builds carry, per optimizer kind
// and sqrt, the forms without a chained sum for the (mode, finalisation) pairs the drop-in's callers produce -- numpy
// * SCALE, torch * DIV, torch device tensors * SCALE (FEDAVG_FIN_RECIP), unweighted * SCALE | DIV -- and the server step
// alone (no clients, the aggregate as the chained sum, FIN_NONE: the FedOpt generator's step, fedopt.py:157-182).
// Anything else (a chained sum with clients, more than 128 clients, numpy with FIN_DIV, FIN_NONE with clients) runs as
// the plain aggregation into a scratch followed by that server step (fedavg_capi.cpp): the same per-element sequence.
inline bool epi_direct(int op, int fin, int k, bool acc_in) {
    if (kAB) return true;
    if (acc_in || k == 0) return acc_in && k == 0 && fin == FEDAVG_FIN_NONE;
    if (k > kMaxRowsPerLaunch) return false;
    if (fin == FEDAVG_FIN_SCALE) return true;
    return fin == FEDAVG_FIN_DIV && op != FEDAVG_OP_NUMPY;
}
// the few-client forms' geometry: blocks per CU, register-held tiles R, LDS-held tiles L, LDS tiles per load group G
struct FewForm {
    int bpc, r, l, g;
    int p = 0;  // 16-bit form only: tiles per unit (0 / 1: one; 2: a pair of consecutive tiles, K x 16 KiB contiguous)
};
// the product's form per read count: the best of two sweeps (profiles/r05/s2/few_k*.jsonl, s3/few_k*.jsonl; 1e9
// params, interleaved in one process, outputs bit-equal, % of 8 TB/s): 1 read -- two blocks per CU, 8 register- + 4
// LDS-held tiles, LDS tiles loaded two at a time (75.2 / 74.6, against 74.4 / 73.8 four at a time, 72.2 one at a time,
// 71.5 / 73.5 with 10 LDS tiles at one block per CU); 2 reads -- one block per CU, 4 register- + 10 LDS-held tiles, one
// LDS tile's loads at a time (78.9, against 77.2 two at a time, 75.3 five, 77.5 with 6 register tiles, 74.1 / 73.8 at
// two blocks per CU).  The same box's 1 : 1 and 2 : 1 burst patterns: 74.5 / 77.2 % (s3/mix_r*.jsonl).
// 3 reads (round 5, session 6, profiles/r05/s6/few34_k3.jsonl): the same kernel at one block per CU, 4 + 10 tiles, 79.2
// against 76.3 % for the burst form with the count built in (78.9 / 78.2 with 3 / 2 register-held tiles, 73.9 at two
// blocks per CU); 4 reads stay on the burst form (the few-client kernel 71.6-74.8 against 76.2 %, s6/few34_k4.jsonl).
constexpr int kFewMaxReads = 3;
// 1 read since session 20 (profiles/r05/s20/f32_k1.jsonl, 3 interleaved rounds, outputs bit-equal): tile PAIRS, two
// blocks per CU, 4 register- + 2 LDS-held units of 2 x 16 KiB, LDS units two at a time -- 76.8 % against 74.5 % for
// (2, 8, 4, 2) on single tiles; pairs lost at 2 and 3 reads (76.6-77.2 against 80.0 %, 78.4-79.7 against 80.2 %).
constexpr FewForm kFewDefault[kFewMaxReads + 1] = {{0, 0, 0, 0}, {2, 4, 2, 2, 2}, {1, 4, 10, 1}, {1, 4, 10, 1}};
// A/B builds: launch variant bits 9-11 pick one of these per read count (1-6; 0 = the default)
// (5-6: tile pairs, p = 2 -- 32 KiB per client per unit, session 18's 16-bit finding carried over)
constexpr FewForm kFewAB[2][6] = {
    {{2, 8, 4, 2}, {1, 12, 10, 2}, {1, 8, 10, 1}, {2, 10, 4, 2}, {2, 4, 2, 1, 2}, {2, 3, 2, 2, 2}},
    {{1, 4, 10, 1}, {1, 6, 10, 1}, {1, 5, 10, 1}, {1, 4, 9, 1}, {1, 2, 5, 1, 2}, {2, 2, 2, 1, 2}}};
// A/B builds: the few-client kernel at 3-4 reads in other forms (variant bits 9-11 = 1-5; 6 and 7 select the burst
// form's client loop for 3-6 clients instead, fedavg_tiles.h launch_burst)
constexpr FewForm kFewAB34[2][6] = {
    {{1, 2, 10, 1}, {1, 3, 10, 1}, {1, 4, 10, 1}, {1, 2, 5, 1, 2}, {1, 1, 5, 1, 2}, {2, 3, 4, 1}},
    {{1, 2, 10, 1}, {1, 3, 10, 1}, {1, 1, 10, 1}, {2, 2, 4, 1}, {1, 2, 8, 1}, {1, 2, 10, 2}}};

// the few-client form of a launch with `reads` (1-3; A/B builds 4) client reads
inline FewForm few_form(int reads, int variant) {
    if (kABFew) {
        const int ix = (variant >> kVariantLoopShift) & 7;
        if (reads <= 2 && ix >= 1 && ix <= 6) return kFewAB[reads - 1][ix - 1];
        if (reads >= 3 && ix >= 1 && ix <= 5) return kFewAB34[reads - 3][ix - 1];
    }
    return kFewDefault[reads];
}
// The 16-bit few-client form (fedavg_narrow.hip fedavg_tiles_narrow_few, 1-3 reads): {blocks/CU, register units, LDS
// units, LDS units per load group, tiles per unit} -- a unit one 8 KiB tile, or (p = 2) a pair of consecutive tiles,
// K x 16 KiB of contiguous slab: the fp32 forms' geometry in bytes.  Session 17 found a 1-client COPY through single
// tiles no faster than the arithmetic (64-66 % of 8 TB/s); on pairs it runs 76.6 % and the torch-mode line 74.5 %
// (profiles/r05/s18/, same process, outputs bit-equal).  Defaults, bf16 x 1e9, % of 8 TB/s: 1 read -- pairs, G 4:
// 74.5 against 66.0 single (38.0 on the burst form); 2 reads -- single tiles: 72.2 against 66.8-69.2 on pairs (the
// 2-client arithmetic weighs on the longer units); 3 reads -- pairs, G 2: 75.0 against 73.9 single.
constexpr int kNarrowFewMaxReads = 3;
constexpr FewForm kNarrowFewDefault[kNarrowFewMaxReads + 1] = {
    {0, 0, 0, 0}, {2, 8, 4, 4, 2}, {2, 8, 8, 4}, {1, 4, 10, 2, 2}};
// A/B builds (-DFEDAVG_AB_FEW): launch variant bits 9-11 = 1-4 pick one of these per read count
constexpr FewForm kNarrowFewAB[3][4] = {
    {{2, 8, 8, 4}, {2, 8, 4, 2, 2}, {2, 4, 2, 2, 4}, {2, 4, 2, 1, 4}},
    {{1, 4, 10, 1, 2}, {1, 4, 10, 2, 2}, {1, 8, 20, 2}, {1, 6, 20, 4}},
    {{1, 8, 20, 4}, {1, 4, 10, 1, 2}, {1, 8, 20, 2}, {1, 6, 20, 2}}};

inline FewForm narrow_few_form(int reads, int form) {
    if (kABFew && form >= 1 && form <= 4) return kNarrowFewAB[reads - 1][form - 1];
    return kNarrowFewDefault[reads];
}

// The fp64 few-client form (fedavg_kernels.hip fedavg_tiles_f64x2_few, 1-3 reads): the same geometry fields, 32 KiB
// tiles (at two blocks per CU at most 2 LDS tiles per block, at one at most 5: 160 KiB per CU) -- the fp32 forms'
// bytes in flight with half the tiles.  Defaults from the same-process sweep of profiles/r05/s14/ (5e8 params, numpy
// mode): 1 / 2 / 3 reads 76.8 / 76.3 / 78.0 % of 8 TB/s against 74.0 / 73.7 / 75.0 % on the burst form.
constexpr int kF64FewMaxReads = 3;
constexpr FewForm kF64FewDefault[kF64FewMaxReads + 1] = {{0, 0, 0, 0}, {2, 4, 2, 2}, {1, 2, 5, 5}, {1, 3, 4, 1}};
// A/B builds (-DFEDAVG_AB_FEW): launch variant bits 9-11 = 1-4 pick one of these per read count
constexpr FewForm kF64FewAB[3][4] = {
    {{2, 4, 2, 1}, {1, 4, 4, 2}, {2, 3, 2, 2}, {1, 6, 4, 2}},
    {{1, 2, 5, 1}, {1, 3, 4, 1}, {1, 2, 4, 2}, {2, 2, 2, 1}},
    {{1, 2, 5, 1}, {1, 2, 4, 2}, {2, 2, 2, 1}, {1, 2, 5, 5}}};

inline FewForm f64_few_form(int reads, int form) {
    if (kABFew && form >= 1 && form <= 4) return kF64FewAB[reads - 1][form - 1];
    return kF64FewDefault[reads];
}

// Every few-client geometry must fit the CU: its blocks' LDS-held tiles within gfx950's 160 KiB of LDS per CU, whole
// load groups (a form that does not fit still runs, with fewer blocks resident than its grid assumes)
constexpr int kLdsBytesPerCu = 160 * 1024;
template <int N>
constexpr bool few_forms_fit(const FewForm (&forms)[N], int tile_bytes) {
    for (int i = 0; i < N; ++i) {
        const FewForm& f = forms[i];
        if (f.bpc == 0) continue;  // the unused read-count-0 slot
        if (f.bpc < 1 || f.r < 1 || f.l < 0 || f.g < 1 || (f.l > 0 && f.l % f.g != 0)) return false;
        if ((int64_t)f.bpc * f.l * tile_bytes * (f.p > 1 ? f.p : 1) > kLdsBytesPerCu) return false;
    }
    return true;
}
static_assert(few_forms_fit(kFewDefault, kDefaultTile * 4) && few_forms_fit(kFewAB[0], kDefaultTile * 4) &&
                  few_forms_fit(kFewAB[1], kDefaultTile * 4) && few_forms_fit(kFewAB34[0], kDefaultTile * 4) &&
                  few_forms_fit(kFewAB34[1], kDefaultTile * 4),
              "fp32 few-client forms");
static_assert(few_forms_fit(kNarrowFewDefault, 8192) && few_forms_fit(kNarrowFewAB[0], 8192) &&
                  few_forms_fit(kNarrowFewAB[1], 8192) && few_forms_fit(kNarrowFewAB[2], 8192),
              "16-bit few-client forms");
static_assert(few_forms_fit(kF64FewDefault, 32768) && few_forms_fit(kF64FewAB[0], 32768) &&
                  few_forms_fit(kF64FewAB[1], 32768) && few_forms_fit(kF64FewAB[2], 32768),
              "fp64 few-client forms");

// whether launch_tiles_f32x4 takes the burst kernel for this geometry (it then wants one block per CU at
// K >= kBurstOneBlockMinK clients, two below)
bool tiles_use_burst(int64_t tile4, int unroll, int variant);
// Blocks per CU of the fp32 burst kernels by client count (profiles/r02/ab/epi_bpc/, interleaved in one
// process, 1e9 params): plain kernel 1 vs 2 blocks at 8 / 16 / 32 / 64 clients 77.6/82.1, 85.0/87.2,
// 87.7/87.3, 89.5/88.7 %; fused Adam 77.8/80.3, 81.6/83.1, 84.8/85.5, 87.2/87.2 %.
constexpr int kBurstOneBlockMinK = 32;
constexpr int kEpiOneBlockMinK = 64;
// The 16-bit burst kernel: one block per CU from 48 clients on in torch / unweighted mode (bf16 / fp16 at 64
// clients 89.6-89.9 % against 85.6 % with two; 128 clients 87.7-88.1 vs 84.3 %), two below and always in numpy
// mode, whose two roundings per step leave one wave per SIMD short of VALU issue (K = 32: 83.3-84.1 vs 84.2-84.3 %;
// numpy fp16 at 64: 74.3 vs 85.4 %) -- profiles/r02/ab/narrow_bpc/.
constexpr int kNarrowOneBlockMinK = 48;
hipError_t launch_dequant_f32(const DequantLaunch& L, hipStream_t s);
hipError_t launch_tiles_epi_f32x4(const TileLaunch& L, const EpiParams& E, hipStream_t s,
                                  uint64_t* launch_count = nullptr);
hipError_t launch_torch16_tails(const RowTableNarrow& tab, int K, int64_t tile, int64_t tstride, const int64_t* idx,
                                int64_t m, const void* acc_in, void* vals, int fmt, int op, int fin, float fin_val,
                                hipStream_t s);
hipError_t launch_scatter16(const int64_t* idx, const void* vals, int64_t m, void* out, hipStream_t s);
hipError_t launch_rows_intsum(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n, int dtype,
                              int grid, hipStream_t s);
hipError_t launch_rows_generic(const RowTableGeneric& tab, int K, const void* acc_in, void* out, int64_t n,
                               int in_dtype, int acc_dtype, int op, int fin, double fin_val, int grid,
                               hipStream_t s);
hipError_t launch_rows_narrow(const RowTableNarrow& tab, int K, const void* acc_in, void* out, int64_t n, int fmt,
                              int op, int fin, float fin_val, int grid, hipStream_t s);
// burst: 2 = the burst form with LDS-held tiles (the default), 1 = the burst form with register-held tiles only
// (results held per block, stored at the end of each short launch), 0 = one launch of the per-tile-store kernel.
// launch_count is incremented per launch.
hipError_t launch_tiles_narrow(const RowTableNarrow& tab, int K, int64_t tstride_elems, const void* acc_in, void* out,
                               int64_t begin, int64_t end, int fmt, int op, int fin, float fin_val, int grid,
                               int burst, hipStream_t s, uint64_t* launch_count);
constexpr int kBurstLdsTiles16 = 8;  // 16-bit burst kernel: 8 x 8 KiB of LDS per block (2 blocks fit a CU)
constexpr int kTile16Elems = 4096;  // the only tile width of the 16-bit tiled kernel
constexpr int kTile64Elems = 4096;  // the only tile width of the fp64 tiled kernel
hipError_t launch_tiles_f64(const RowTableGeneric& tab, int K, int64_t tstride_elems, const void* acc_in, void* out,
                            int64_t begin, int64_t end, int op, int fin, double fin_val, int grid, int burst,
                            hipStream_t s, uint64_t* launch_count);
hipError_t launch_fill_synthetic_f32(float* dst, int64_t n, int64_t tile, int64_t tstride, uint64_t seed, uint64_t row,
                                     uint64_t col0, int grid, hipStream_t s);
hipError_t launch_gather_f32(const float* src, const uint64_t* idx, float* dst, int64_t m, hipStream_t s);
hipError_t launch_sqrt_f32(const float* x, float* out, int64_t n, int torch_sqrt, const uint32_t* rsqrtps, int grid,
                           hipStream_t s);

}  // namespace fedavg
