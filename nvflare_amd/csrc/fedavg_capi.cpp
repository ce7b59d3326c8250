// fedavg_capi.cpp -- C-ABI of libnvflare_amd_fedavg.so (see include/nvflare_amd_fedavg.h).
//
// House conventions of the reference's only C-ABI (integration/xgboost/encryption_plugins/shared/
// plugins/plugin_main.cc:24-111): opaque handle, int rc, thread-local last-error string, every entry
// point wrapped so that no C++ exception crosses the boundary.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <exception>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "fedavg_internal.h"

namespace {

thread_local std::string g_last_error;

struct Error : std::exception {
    std::string msg;
    explicit Error(std::string m) : msg(std::move(m)) {}
    const char* what() const noexcept override { return msg.c_str(); }
};

#define HIP_CHECK(expr)                                                                                     \
    do {                                                                                                    \
        hipError_t _e = (expr);                                                                             \
        if (_e != hipSuccess) {                                                                             \
            throw Error(std::string(#expr) + " failed: " + hipGetErrorName(_e) + " (" + hipGetErrorString(_e) + \
                        ")");                                                                               \
        }                                                                                                   \
    } while (0)

template <typename F>
int guarded(F&& f) {
    try {
        f();
        g_last_error.clear();
        return 0;
    } catch (const Error& e) {
        g_last_error = e.msg;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
    } catch (const std::exception& e) {
        g_last_error = std::string("exception: ") + e.what();
    } catch (...) {
        g_last_error = "unknown exception";
    }
    return 1;
}

constexpr size_t kRsqrtpsEntries = 8192;  // 2 exponent parities x 4096 top-12-bit mantissas
constexpr int kRingSlots = 4;
constexpr size_t kRingBytes = 64ull << 20;  // 64 MiB per pinned staging slot
constexpr size_t kParallelCopyMin = 8ull << 20;
constexpr int kCopyThreads = 8;

void check_dtype(int dt) {
    if (dt < FEDAVG_F32 || dt > FEDAVG_U64) throw Error("unknown dtype " + std::to_string(dt));
}

size_t dtype_size(int dt) {
    switch (dt) {
        case FEDAVG_F64:
        case FEDAVG_I64:
        case FEDAVG_U64:
            return 8;
        case FEDAVG_F32:
        case FEDAVG_I32:
        case FEDAVG_U32:
            return 4;
        case FEDAVG_F16:
        case FEDAVG_BF16:
        case FEDAVG_I16:
        case FEDAVG_U16:
            return 2;
        default:
            return 1;
    }
}

// The value of the float16 nearest to d (round to nearest even, subnormals, overflow to inf), rounded
// directly from fp64 -- numpy's npy_double_to_half, which NEP 50 applies to a python float meeting a
// float16 array.
float half_value(double d) {
    if (std::isnan(d)) return NAN;
    const double a = std::fabs(d);
    if (a >= 65520.0) return std::copysign(INFINITY, (float)d);  // halfway to 2^16 rounds to even = inf
    double q = 0x1p-24;                                            // subnormal quantum
    if (a >= 0x1p-14) {
        int e;
        std::frexp(a, &e);  // a in [2^(e-1), 2^e)
        q = std::ldexp(1.0, e - 11);
    }
    return (float)std::copysign(std::nearbyint(a / q) * q, d);
}

// The value of the bfloat16 nearest to f (c10::BFloat16 round_to_nearest_even).
float bf16_value(float f) {
    if (std::isnan(f)) return NAN;
    uint32_t u;
    memcpy(&u, &f, 4);
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    float r;
    memcpy(&r, &u, 4);
    return r;
}

// fp32 value a python float takes when torch casts it to the tensor's 16-bit dtype (Scalar::to<T>():
// fp64 -> fp32 -> 16-bit)
float torch16_value(int fmt, double w) {
    const float f = (float)w;
    return fmt == FEDAVG_BF16 ? bf16_value(f) : half_value((double)f);
}

void parallel_memcpy(void* dst, const void* src, size_t n) {
    if (n < kParallelCopyMin) {
        memcpy(dst, src, n);
        return;
    }
    const size_t chunk = ((n + kCopyThreads - 1) / kCopyThreads + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    th.reserve(kCopyThreads);
    for (int t = 0; t < kCopyThreads; ++t) {
        const size_t off = (size_t)t * chunk;
        if (off >= n) break;
        const size_t len = std::min(chunk, n - off);
        th.emplace_back([=] { memcpy(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off, len); });
    }
    for (auto& x : th) x.join();
}

// Copy a list of (dst, src, len) segments with the host copy threads, split by bytes (not by segment), so
// a ring slot filled from hundreds of small keys copies as fast as one large one.
struct Seg {
    char* dst;
    const char* src;
    size_t len;
};

void parallel_gather(const std::vector<Seg>& segs) {
    size_t total = 0;
    for (const Seg& s : segs) total += s.len;
    if (total < kParallelCopyMin) {
        for (const Seg& s : segs) memcpy(s.dst, s.src, s.len);
        return;
    }
    const size_t share = (total + kCopyThreads - 1) / kCopyThreads;
    std::vector<std::thread> th;
    th.reserve(kCopyThreads);
    size_t seg = 0, seg_off = 0;
    for (int t = 0; t < kCopyThreads && seg < segs.size(); ++t) {
        // this thread's work: `share` bytes starting at (seg, seg_off)
        std::vector<Seg> mine;
        size_t need = share;
        while (need && seg < segs.size()) {
            const size_t take = std::min(need, segs[seg].len - seg_off);
            mine.push_back({segs[seg].dst + seg_off, segs[seg].src + seg_off, take});
            need -= take;
            seg_off += take;
            if (seg_off == segs[seg].len) {
                ++seg;
                seg_off = 0;
            }
        }
        th.emplace_back([mine] {
            for (const Seg& s : mine) memcpy(s.dst, s.src, s.len);
        });
    }
    for (auto& x : th) x.join();
}

}  // namespace

struct fedavg_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t ext_stream = nullptr;  // caller-provided compute stream (not owned)
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr, ev_copy_done = nullptr;
    hipEvent_t ev_region_start = nullptr, ev_region_stop = nullptr;
    bool region_open = false;
    bool timing = false;
    bool timed_valid = false;
    void* ring[kRingSlots] = {};
    hipEvent_t ring_ev[kRingSlots] = {};
    bool ring_used[kRingSlots] = {};
    int ring_next = 0;
    int blocks_per_cu = 0;  // 0: each kernel's own default (bpc())
    uint64_t launches = 0;  // kernel launches issued on the compute stream (fedavg_launch_count)
    int unroll = fedavg::kDefaultUnroll;
    int variant = 0;
    int tile = fedavg::kDefaultTile;  // tile width of the contiguous-rows entry point
    // readiness marks for fedavg_d2h_marked: (event on the compute stream, bytes of the source final by then)
    std::vector<std::pair<hipEvent_t, size_t>> marks;
    std::vector<hipEvent_t> mark_pool;
    // torch scalar-remainder elements of a 16-bit launch: their indices and recomputed values (device)
    void* tails_buf = nullptr;
    size_t tails_bytes = 0;
    // this host's RSQRTPS estimates for FEDAVG_SQRT_TORCH_AMD (fedavg_set_rsqrtps_table): 8192 x 12 bits, two per
    // word, in device memory; staged into LDS by every kernel that computes that sqrt
    uint32_t* rsqrtps = nullptr;

    hipStream_t compute() const { return ext_stream ? ext_stream : own_stream; }
    int bpc(int dflt = fedavg::kDefaultBlocksPerCu) const { return blocks_per_cu ? blocks_per_cu : dflt; }
    void activate() const { HIP_CHECK(hipSetDevice(device)); }
};

namespace {

bool is_pinned_host(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

int stream_grid(const fedavg_ctx* ctx, int64_t work_items) {
    const int64_t cap = (int64_t)ctx->num_cus * 8;
    const int64_t need = (work_items + fedavg::kBlock - 1) / fedavg::kBlock;
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, need));
}

bool valid_tile(size_t t) { return t == 1024 || t == 2048 || t == 4096 || t == 8192; }

// Copy `len` bytes from `src` into the tiled storage of one client: logical byte b of the client's flat
// row lands at dst + (b / tile_b) * tstride_b + b % tile_b.  Issued as (partial head, one 2-D copy of
// whole tiles, partial tail) on `s`.
void copy_into_tiles(char* dst, size_t tile_b, size_t tstride_b, size_t logical_off, const char* src, size_t len,
                     hipMemcpyKind kind, hipStream_t s) {
    if (tstride_b == tile_b) {
        HIP_CHECK(hipMemcpyAsync(dst + logical_off, src, len, kind, s));
        return;
    }
    size_t b = logical_off;
    const size_t end = logical_off + len;
    auto place = [&](size_t lb) { return dst + (lb / tile_b) * tstride_b + lb % tile_b; };
    if (b % tile_b) {
        const size_t head = std::min(end, (b / tile_b + 1) * tile_b) - b;
        HIP_CHECK(hipMemcpyAsync(place(b), src, head, kind, s));
        src += head;
        b += head;
    }
    const size_t full = (end - b) / tile_b;
    if (full) {
        HIP_CHECK(hipMemcpy2DAsync(place(b), tstride_b, src, tile_b, tile_b, full, kind, s));
        src += full * tile_b;
        b += full * tile_b;
    }
    if (b < end) HIP_CHECK(hipMemcpyAsync(place(b), src, end - b, kind, s));
}

// H2D into (tiled) client storage.  Pageable sources go through the pinned ring: the host threads copy a
// 64 MiB slot while the DMA engine drains the previous ones.  The compute stream waits on the copies; the
// caller may reuse `src` as soon as this returns.
void h2d_impl(fedavg_ctx* ctx, char* dst, size_t tile_b, size_t tstride_b, size_t logical_off, const char* src,
              size_t len) {
    if (len == 0) return;
    ctx->activate();
    if (is_pinned_host(src)) {
        copy_into_tiles(dst, tile_b, tstride_b, logical_off, src, len, hipMemcpyHostToDevice, ctx->copy_stream);
        HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));  // a pinned source may be reused on return
        return;
    }
    size_t done = 0;
    while (done < len) {
        const int slot = ctx->ring_next;
        ctx->ring_next = (ctx->ring_next + 1) % kRingSlots;
        if (ctx->ring_used[slot]) HIP_CHECK(hipEventSynchronize(ctx->ring_ev[slot]));
        const size_t n = std::min(kRingBytes, len - done);
        parallel_memcpy(ctx->ring[slot], src + done, n);
        copy_into_tiles(dst, tile_b, tstride_b, logical_off + done, static_cast<const char*>(ctx->ring[slot]), n,
                        hipMemcpyHostToDevice, ctx->copy_stream);
        HIP_CHECK(hipEventRecord(ctx->ring_ev[slot], ctx->copy_stream));
        ctx->ring_used[slot] = true;
        done += n;
    }
    HIP_CHECK(hipEventRecord(ctx->ev_copy_done, ctx->copy_stream));
    HIP_CHECK(hipStreamWaitEvent(ctx->compute(), ctx->ev_copy_done, 0));
}

// Several host pieces of one client (its keys, in increasing logical order, non-overlapping) packed into
// the pinned ring by LOGICAL position, so each 64 MiB slot leaves in one tiled DMA however many keys it
// holds.  Gaps between pieces (key alignment padding) are copied as don't-care bytes.
// A piece that does not fit the rest of a slot is split: its remainder opens the next slot and the
// following pieces pack in behind it, so every slot but the last leaves full.
void h2d_multi_impl(fedavg_ctx* ctx, char* dst, size_t tile_b, size_t tstride_b, int n, const size_t* offs,
                    const void* const* srcs, const size_t* lens) {
    ctx->activate();
    int i = 0;
    size_t carried = 0;   // bytes of piece i already sent (split across slots)
    size_t prev_end = 0;  // logical end of the previous piece (pieces sorted, non-overlapping)
    while (i < n && lens[i] == 0) ++i;
    while (i < n) {
        const size_t win0 = offs[i] + carried;
        const int slot = ctx->ring_next;
        ctx->ring_next = (ctx->ring_next + 1) % kRingSlots;
        if (ctx->ring_used[slot]) HIP_CHECK(hipEventSynchronize(ctx->ring_ev[slot]));
        char* ring = static_cast<char*>(ctx->ring[slot]);
        size_t win_end = win0;
        std::vector<Seg> segs;
        // fill the slot with whole or partial pieces while they fit
        while (i < n) {
            if (lens[i] == 0) {
                ++i;
                continue;
            }
            if (carried == 0 && offs[i] < prev_end) throw Error("h2d pieces must be sorted and non-overlapping");
            const size_t start = offs[i] + carried;
            const size_t rel = start - win0;
            if (rel >= kRingBytes) break;  // starts beyond this slot's window: opens the next slot
            if (carried == 0) prev_end = offs[i] + lens[i];
            const size_t take = std::min(lens[i] - carried, kRingBytes - rel);
            segs.push_back({ring + rel, static_cast<const char*>(srcs[i]) + carried, take});
            win_end = start + take;
            carried += take;
            if (carried < lens[i]) break;  // slot full: the rest of this piece opens the next slot
            ++i;
            carried = 0;
        }
        parallel_gather(segs);
        if (win_end > win0) {
            copy_into_tiles(dst, tile_b, tstride_b, win0, ring, win_end - win0, hipMemcpyHostToDevice,
                            ctx->copy_stream);
            HIP_CHECK(hipEventRecord(ctx->ring_ev[slot], ctx->copy_stream));
            ctx->ring_used[slot] = true;
        }
    }
    HIP_CHECK(hipEventRecord(ctx->ev_copy_done, ctx->copy_stream));
    HIP_CHECK(hipStreamWaitEvent(ctx->compute(), ctx->ev_copy_done, 0));
}

void check_op_fin(int op, int fin) {
    if (op < FEDAVG_OP_NUMPY || op > FEDAVG_OP_TORCH_DEVICE) throw Error("bad op " + std::to_string(op));
    if (fin < FEDAVG_FIN_NONE || fin > FEDAVG_FIN_RECIP) throw Error("bad fin " + std::to_string(fin));
}

// The fp32 / fp64 kernels know three steps and two finalisations; torch-ROCm's device-tensor arithmetic
// (FEDAVG_OP_TORCH_DEVICE, FEDAVG_FIN_RECIP) maps onto them: the steps are FEDAVG_OP_TORCH's at these widths,
// and torch's reciprocal -- the fp64 quotient 1.0 / count cast to the opmath type (measured against torch on the
// GPU: tools/debug_device_f32.py) -- is exactly the library's FEDAVG_FIN_SCALE value acc_t(1.0 / count).
void normalize_wide(int& op, int& fin, double& count, bool acc_f32) {
    (void)count;
    (void)acc_f32;
    if (op == FEDAVG_OP_TORCH_DEVICE) op = FEDAVG_OP_TORCH;
    if (fin == FEDAVG_FIN_RECIP) fin = FEDAVG_FIN_SCALE;
}

// finalisation scalar, computed on the host exactly as the reference computes it:
//   numpy  T * (1.0 / count): python fp64 reciprocal, then cast to the array dtype
//   torch  T.div_(count):     the scalar operand cast to the tensor dtype
double fin_scalar(int fin, double count) { return fin == FEDAVG_FIN_SCALE ? 1.0 / count : count; }

// Fewest row reads per launch (clients, plus the chained partial sum) that take the burst kernels; fewer go to the
// per-tile-store kernels (same tile_sum and epilogue arithmetic, so the same bits).  With one or two row reads per
// result the burst kernel's read phase is too short to pay for holding the results.  Round 4, with the client count
// built into the burst kernel (no repeated loads) and the division-free FIN_DIV, same box, % of HBM peak, per-tile vs
// burst (profiles/r04/s4/divc_k*.jsonl; s2/ab_k*.jsonl on another box): 1 client 63.7 vs 53.9 (74.4 vs 54.7), 2
// clients 71.1 vs 69.2 (75.4 vs 71.6), 3 clients 70.2 vs 74.8 (71.7 vs 74.5), 4 clients 71.3 vs 72.2.  Round 3 (the
// burst kernel re-loading clients to fill its groups of four) had the switch at 4.  The fused epilogue keeps 4: its
// per-tile form wins further up, because its optimizer-state reads and writes fall in the same launch (Adam, 5e8
// params, per-tile vs burst: 1 client 73 vs 62 %, 2: 77.2 vs 63.6 %, 4: 76.2 vs 72.9 %; from 5 clients on the burst
// form wins by 1.5-14 points, profiles/r03/s25/, s26/).  The stand-alone server step (no clients, the aggregate as
// acc_in: one read) takes the per-tile form.
constexpr int kBurstMinClients = 3;
constexpr int kVariantFewBurst = 256;  // A/B variant bit 8 (A/B and -DFEDAVG_AB_FEW builds): launches under
                                       // kBurstMinClients reads (16-bit: 1-3 reads) keep the burst form
constexpr int kEpiBurstMinClients = 4;

// Tile-kernel launches over [b, e) (elements, multiples of 4) for any number of clients: chunks of at
// most kMaxRowsPerLaunch clients, later chunks continuing in place through `out`.
void run_tiles(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows, int64_t tile,
               int64_t tstride, int64_t b, int64_t e, const float* acc_in, float* out, int op, int fin, double count,
               hipStream_t s) {
    fedavg::TileLaunch L;
    L.op = op;
    L.unroll = ctx->unroll;
    L.tile4 = tile / 4;
    L.tstride4 = tstride / 4;
    L.b4 = b / 4;
    L.e4 = e / 4;
    const int64_t n_tiles = (L.e4 - 1) / L.tile4 - L.b4 / L.tile4 + 1;
    const float fv = (float)fin_scalar(fin, count);
    int k0 = 0;
    const float* cur_in = acc_in;
    do {
        const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
        // the kernel form per launch: a chained chunk (acc_in + kc clients) reads kc + 1 rows
        const int reads = kc + (cur_in ? 1 : 0);
        // 1-2 client reads without a chained sum: the few-client burst kernel (round 5) at the default geometry,
        // unless the public variant asks for the per-tile form (bit 3) or the general burst form (bit 8; A/B builds)
        // 1-3 client reads (kFewMaxReads) without a chained sum; A/B builds with -DFEDAVG_AB_FEW: 4 reads with variant
        // bits 9-11 = 1-5 too, and 3 reads with bits 9-11 = 6 or 7 on the burst form (its client-loop A/Bs)
        const int few_ab_ix = fedavg::kABFew ? (ctx->variant >> fedavg::kVariantLoopShift) & 7 : 0;
        const bool few_reads = (reads <= fedavg::kFewMaxReads && !(reads == 3 && few_ab_ix >= 6)) ||
                               (kc == 4 && few_ab_ix >= 1 && few_ab_ix <= 5);
        const bool few = few_reads && !cur_in && kc >= 1 && L.tile4 == fedavg::kDefaultTile / 4 &&
                         L.unroll == fedavg::kDefaultUnroll &&
                         !(ctx->variant & (fedavg::kVariantTileStores | fedavg::kVariantTemporalLoads |
                                           fedavg::kVariantTemporalStores | kVariantFewBurst));
        const int variant =
            ctx->variant | (reads < kBurstMinClients && !few && !(ctx->variant & kVariantFewBurst) ? fedavg::kVariantTileStores
                                                                                                  : 0);
        const bool burst = fedavg::tiles_use_burst(L.tile4, L.unroll, variant);
        int bpc = burst ? ctx->bpc(k_rows >= fedavg::kBurstOneBlockMinK ? 1 : 2) : ctx->bpc();
        if (few) bpc = ctx->bpc(fedavg::few_form(kc, ctx->variant).bpc);
        // one block per CU: the burst kernel holds 10 tiles in LDS (all 160 KiB); public bit 6 keeps the 4-tile
        // form, public bit 5 (register-held tiles only) keeps no LDS tiles at all
        const bool wide = !few && burst && bpc == 1 && !(variant & (fedavg::kVariantWideLds | fedavg::kVariantRegisterTiles));
        L.variant = (variant & ~fedavg::kVariantWideLds) | (wide ? fedavg::kVariantWideLds : 0) | (few ? fedavg::kVariantFew : 0);
        L.grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * bpc, n_tiles));
        memset(&L.tab, 0, sizeof(L.tab));
        for (int j = 0; j < kc; ++j) {
            L.tab.rows[j] = static_cast<const fedavg::f32x4*>(bases[k0 + j]);
            L.tab.w[j] = (float)weights[k0 + j];  // fp64 host weight -> fp32, round to nearest
        }
        L.k = kc;
        L.fin = (k0 + kc >= k_rows) ? fin : FEDAVG_FIN_NONE;
        L.fin_val = fv;
        L.acc_in = cur_in;
        L.out = out;
        HIP_CHECK(fedavg::launch_tiles_f32x4(L, s, &ctx->launches));
        cur_in = out;
        k0 += kc;
    } while (k0 < k_rows);
}

// Epilogue scalars as torch computes them: python-float (fp64) hyperparameters and bias corrections,
// cast to fp32 where they meet a tensor (oracle/fedavg_oracle.c oracle_epilogue_apply mirrors this).
fedavg::EpiParams make_epi(const fedavg_ctx* ctx, const fedavg_epilogue& e) {
    fedavg::EpiParams E;
    memset(&E, 0, sizeof(E));
    if (e.torch_sqrt == FEDAVG_SQRT_TORCH_AMD) {
        if (!ctx->rsqrtps)
            throw Error("FEDAVG_SQRT_TORCH_AMD needs this host's RSQRTPS table first (fedavg_set_rsqrtps_table)");
        E.rsqrtps = ctx->rsqrtps;
    }
    E.kind = e.kind;
    E.first_step = e.first_step;
    E.nesterov = e.nesterov;
    E.maximize = e.maximize;
    E.decoupled_weight_decay = e.decoupled_weight_decay;
    E.has_weight_decay = e.weight_decay != 0.0;
    E.has_momentum = e.momentum != 0.0;
    E.weight_decay = (float)e.weight_decay;
    E.momentum = (float)e.momentum;
    E.one_minus_dampening = (float)(1.0 - e.dampening);
    E.neg_lr = (float)(-e.lr);
    E.decoupled_scale = (float)(1.0 - e.lr * e.weight_decay);
    E.one_minus_beta1 = (float)(1.0 - e.beta1);
    E.one_minus_beta1_m1 = E.one_minus_beta1 - 1.0f;  // lerp_vec: weight - vec_t(1), in fp32
    E.one_minus_beta2 = (float)(1.0 - e.beta2);
    E.beta2 = (float)e.beta2;
    const double bc1 = 1.0 - std::pow(e.beta1, e.step);
    const double bc2 = 1.0 - std::pow(e.beta2, e.step);
    E.step_size_neg = (float)(-(e.lr / bc1));
    if (e.kind == FEDAVG_EPI_ADAGRAD)  // adagrad.py: clr = lr / (1 + (step - 1) * lr_decay), value = -clr
        E.step_size_neg = (float)(-(e.lr / (1.0 + (e.step - 1.0) * e.lr_decay)));
    E.bias_correction2_sqrt = (float)std::pow(bc2, 0.5);
    E.eps = (float)e.eps;
    E.param = e.param;
    E.state1 = e.state1;
    E.state2 = e.state2;
    E.base = e.base;
    E.amsgrad = e.kind == FEDAVG_EPI_ADAM && e.amsgrad;
    E.state3 = e.state3;
    if (e.torch_sqrt != FEDAVG_SQRT_IEEE && e.torch_sqrt != FEDAVG_SQRT_TORCH_AVX512 && e.torch_sqrt != FEDAVG_SQRT_TORCH_AMD)
        throw Error("epilogue torch_sqrt must be FEDAVG_SQRT_IEEE, _TORCH_AVX512 or _TORCH_AMD");
    E.torch_sqrt = e.torch_sqrt;
    if (e.kind == FEDAVG_EPI_RMSPROP) {  // rmsprop.py: square_avg.mul_(alpha).addcmul_(g, g, 1 - alpha), lerp(1 - alpha)
        E.beta2 = (float)e.alpha;
        E.one_minus_beta2 = (float)(1.0 - e.alpha);
        E.one_minus_beta1 = E.one_minus_beta2;
        E.one_minus_beta1_m1 = E.one_minus_beta1 - 1.0f;
        E.centered = e.centered != 0;
    }
    if (e.kind == FEDAVG_EPI_NADAM) {  // nadam.py _single_tensor_nadam (python floats; mu_product is an fp32 tensor)
        const double mu = e.beta1 * (1.0 - 0.5 * std::pow(0.96, e.step * e.momentum_decay));
        const double mu_next = e.beta1 * (1.0 - 0.5 * std::pow(0.96, (e.step + 1.0) * e.momentum_decay));
        const float mp = (float)e.mu_product * (float)mu;  // mu_product *= mu
        E.bias_correction2 = (float)bc2;
        E.coef_grad = (float)((-e.lr * (1.0 - mu)) / (1.0 - (double)mp));
        E.coef_avg = (float)((-e.lr * mu_next) / (1.0 - (double)mp * mu_next));
    }
    if (e.kind == FEDAVG_EPI_RPROP) {  // rprop.py: python floats written into / compared with fp32 tensors
        E.etaminus = (float)e.etaminus;
        E.etaplus = (float)e.etaplus;
        E.ss_min = (float)e.step_size_min;
        E.ss_max = (float)e.step_size_max;
    }
    if (e.kind == FEDAVG_EPI_ASGD) {  // asgd.py: eta_value = _get_value(eta) (fp32 state), python-float math
        E.decay = (float)(1.0 - e.lambd * e.eta);
        E.neg_eta = (float)(-e.eta);
        E.mu = (float)e.mu;
    }
    if (e.kind == FEDAVG_EPI_RADAM) {  // radam.py _single_tensor_radam
        const double rho_inf = 2.0 / (1.0 - e.beta2) - 1.0;
        const double rho_t = rho_inf - 2.0 * e.step * std::pow(e.beta2, e.step) / bc2;
        E.bias_correction1 = (float)bc1;
        E.lr = (float)e.lr;
        E.rectified = rho_t > 5.0;
        if (E.rectified)
            E.rect = (float)std::pow((rho_t - 4.0) * (rho_t - 2.0) * rho_inf / ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t), 0.5);
    }
    return E;
}

void run_generic(fedavg_ctx* ctx, const void* const* rows, const double* weights, int k_rows, size_t elem_off,
                 const void* acc_in, void* out, int64_t n, int in_dtype, int acc_dtype, int op, int fin, double count,
                 hipStream_t s) {
    const size_t in_sz = dtype_size(in_dtype);
    const size_t acc_sz = dtype_size(acc_dtype);
    const double fd = fin_scalar(fin, count);
    int k0 = 0;
    const char* cur_in = acc_in ? static_cast<const char*>(acc_in) + elem_off * acc_sz : nullptr;
    char* o = static_cast<char*>(out) + elem_off * acc_sz;
    do {
        const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
        fedavg::RowTableGeneric gt;
        memset(&gt, 0, sizeof(gt));
        for (int j = 0; j < kc; ++j) {
            gt.rows[j] = static_cast<const char*>(rows[k0 + j]) + elem_off * in_sz;
            // weight rounded to the accumulator type on the host (the kernel's cast is then exact)
            gt.w[j] = acc_dtype == FEDAVG_F32 ? (double)(float)weights[k0 + j] : weights[k0 + j];
        }
        const bool last = k0 + kc >= k_rows;
        const double fv = acc_dtype == FEDAVG_F32 ? (double)(float)fd : fd;
        HIP_CHECK(fedavg::launch_rows_generic(gt, kc, cur_in, o, n, in_dtype, acc_dtype, op,
                                              last ? fin : FEDAVG_FIN_NONE, fv, stream_grid(ctx, n), s));
        ++ctx->launches;
        cur_in = o;
        k0 += kc;
    } while (k0 < k_rows);
}

// integer / bool sums (weigh_by_local_iter=False numpy arrays), chained through out past 128 rows
void run_intsum(fedavg_ctx* ctx, const void* const* rows, int k_rows, const void* acc_in, void* out, int64_t n,
                int dtype, hipStream_t s) {
    int k0 = 0;
    const void* cur_in = acc_in;
    do {
        const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
        fedavg::RowTableGeneric gt;
        memset(&gt, 0, sizeof(gt));
        for (int j = 0; j < kc; ++j) gt.rows[j] = rows[k0 + j];
        HIP_CHECK(fedavg::launch_rows_intsum(gt, kc, cur_in, out, n, dtype, stream_grid(ctx, n), s));
        ++ctx->launches;
        cur_in = out;
        k0 += kc;
    } while (k0 < k_rows);
}

// 16-bit accumulators: the weights and the finalisation scalar are rounded here exactly as the reference
// library rounds them (see fedavg_narrow.hip).
float narrow_fin_value(int fmt, int fin, double count) {
    if (fin == FEDAVG_FIN_SCALE)  // numpy: total * (1.0 / count), the python float cast to the array dtype
        return fmt == FEDAVG_F16 ? half_value(1.0 / count) : bf16_value((float)(1.0 / count));
    if (fin == FEDAVG_FIN_DIV)  // torch: div_ by a CPU scalar in fp32
        return (float)count;
    if (fin == FEDAVG_FIN_RECIP)  // torch-ROCm: multiply by (float)(1.0 / count) (the kernel's SCALE form)
        return (float)(1.0 / count);
    return 0.0f;
}

// the narrow kernels' own fin for a C-ABI fin (the device reciprocal is their SCALE form with an fp32 scale);
// FEDAVG_OP_TORCH_DEVICE reaches them as is (float16: one rounding per add_ step; bfloat16: FEDAVG_OP_TORCH)
int narrow_kernel_op(int op) { return op; }
int narrow_kernel_fin(int fin) { return fin == FEDAVG_FIN_RECIP ? FEDAVG_FIN_SCALE : fin; }

void fill_narrow_table(fedavg::RowTableNarrow& t, const void* const* rows, const double* weights, int k0, int kc,
                       int fmt, int op) {
    memset(&t, 0, sizeof(t));
    for (int j = 0; j < kc; ++j) {
        const double w = weights[k0 + j];
        t.rows[j] = rows[k0 + j];
        if (op == FEDAVG_OP_NUMPY) {
            t.w_first[j] = t.w_step[j] = fmt == FEDAVG_F16 ? half_value(w) : bf16_value((float)w);
        } else if (op == FEDAVG_OP_TORCH_DEVICE) {  // torch-ROCm: mul and add_ keep the scalar in fp32
            t.w_first[j] = t.w_step[j] = (float)w;
        } else {  // torch: mul keeps the scalar in fp32, add_ casts alpha to the tensor dtype
            t.w_first[j] = (float)w;
            t.w_step[j] = torch16_value(fmt, w);
        }
    }
}

// Contiguous 16-bit rows: chunks of at most kMaxRowsPerLaunch clients chained through `out`.
void run_narrow(fedavg_ctx* ctx, const void* const* rows, const double* weights, int k_rows, const void* acc_in,
                void* out, int64_t n, int fmt, int op, int fin, double count, hipStream_t s) {
    const float fv = narrow_fin_value(fmt, fin, count);
    int k0 = 0;
    const void* cur_in = acc_in;
    do {
        const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
        fedavg::RowTableNarrow t;
        fill_narrow_table(t, rows, weights, k0, kc, fmt, op);
        const bool last = k0 + kc >= k_rows;
        // one lane per 8 elements; 2 x blocks_per_cu resident blocks per CU stride over the K row streams
        // (4 by default: +2 % over 2, flat above -- profiles/r01/narrow_sweep.jsonl)
        const int64_t need = (n / 8 + fedavg::kBlock) / fedavg::kBlock;
        const int grid =
            (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * 2 * ctx->bpc(), need));
        HIP_CHECK(fedavg::launch_rows_narrow(t, kc, cur_in, out, n, fmt, narrow_kernel_op(op),
                                             last ? narrow_kernel_fin(fin) : FEDAVG_FIN_NONE, fv, grid, s));
        ++ctx->launches;
        cur_in = out;
        k0 += kc;
    } while (k0 < k_rows);
}

// Tiled 16-bit client storage over [begin, end) (multiples of 8): chunks of 128 clients chained through out.
// tails / n_tails: sorted flat indices inside [begin, end) that take torch's scalar-remainder step (op TORCH
// only; fedavg_narrow.hip fedavg_torch16_tails), already on the device.
void run_tiles_narrow(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows, int64_t tstride,
                      int64_t begin, int64_t end, const void* acc_in, void* out, int fmt, int op, int fin, double count,
                      hipStream_t s, const int64_t* tails = nullptr, int64_t n_tails = 0, void* tail_vals = nullptr) {
    const float fv = narrow_fin_value(fmt, fin, count);
    const int64_t T = fedavg::kTile16Elems;
    const int64_t n_tiles = (end - 1) / T - begin / T + 1;
    // blocks per CU of the 16-bit burst kernel: fedavg_internal.h kNarrowOneBlockMinK
    const bool burst = !(ctx->variant & fedavg::kVariantTileStores);
    int k0 = 0;
    const void* cur_in = acc_in;
    do {
        const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
        // 1-3 client reads without a chained sum: the 16-bit few-client form (round 5); A/B builds with
        // -DFEDAVG_AB_FEW pick its geometry with launch variant bits 9-11 = 1-4
        const int few_ix = fedavg::kABFew ? (ctx->variant >> fedavg::kVariantLoopShift) & 7 : 0;
        const bool few = burst && !cur_in && kc <= fedavg::kNarrowFewMaxReads && !(ctx->variant & kVariantFewBurst);
        const int dflt = few ? fedavg::narrow_few_form(kc, few_ix).bpc
                             : (burst && op != FEDAVG_OP_NUMPY && kc >= fedavg::kNarrowOneBlockMinK ? 1 : 2);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * ctx->bpc(dflt), n_tiles));
        fedavg::RowTableNarrow t;
        fill_narrow_table(t, bases, weights, k0, kc, fmt, op);
        const bool last = k0 + kc >= k_rows;
        if (n_tails) {  // before the tile kernel: cur_in may be out
            HIP_CHECK(fedavg::launch_torch16_tails(t, kc, T, tstride, tails, n_tails, cur_in, tail_vals, fmt, op,
                                                   last ? narrow_kernel_fin(fin) : FEDAVG_FIN_NONE, fv, s));
            ++ctx->launches;
        }
        HIP_CHECK(fedavg::launch_tiles_narrow(t, kc, tstride, cur_in, out, begin, end, fmt, narrow_kernel_op(op),
                                              last ? narrow_kernel_fin(fin) : FEDAVG_FIN_NONE, fv, grid,
                                              few ? 3 + (few_ix <= 4 ? few_ix : 0)
                                                  : burst ? ((ctx->variant & fedavg::kVariantRegisterTiles) ? 1 : 2) : 0,
                                              s, &ctx->launches));
        if (n_tails) {
            HIP_CHECK(fedavg::launch_scatter16(tails, tail_vals, n_tails, out, s));
            ++ctx->launches;
        }
        cur_in = out;
        k0 += kc;
    } while (k0 < k_rows);
}

struct TimingScope {
    fedavg_ctx* ctx;
    hipStream_t s;
    TimingScope(fedavg_ctx* c, hipStream_t st) : ctx(c), s(st) {
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->ev_start, s));
    }
    void done() {
        if (ctx->timing) {
            HIP_CHECK(hipEventRecord(ctx->ev_stop, s));
            ctx->timed_valid = true;
        }
    }
};

}  // namespace

extern "C" {

const char* fedavg_last_error(void) { return g_last_error.c_str(); }

int fedavg_abi_version(void) { return FEDAVG_ABI_VERSION; }

size_t fedavg_struct_size(int which) {
    switch (which) {
        case 0:
            return sizeof(fedavg_epilogue);
        case 1:
            return sizeof(fedavg_quant);
        default:
            return 0;
    }
}

int fedavg_device_count(int* n) {
    return guarded([&] {
        if (!n) throw Error("n is NULL");
        int c = 0;
        HIP_CHECK(hipGetDeviceCount(&c));
        *n = c;
    });
}

int fedavg_create(int device, fedavg_ctx** out) {
    return guarded([&] {
        if (!out) throw Error("out is NULL");
        *out = nullptr;
        int n = 0;
        HIP_CHECK(hipGetDeviceCount(&n));
        if (device < 0 || device >= n)
            throw Error("device " + std::to_string(device) + " out of range (" + std::to_string(n) + " devices)");
        auto* ctx = new fedavg_ctx();
        ctx->device = device;
        try {
            ctx->activate();
            hipDeviceProp_t prop;
            HIP_CHECK(hipGetDeviceProperties(&prop, device));
            ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
            HIP_CHECK(hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking));
            HIP_CHECK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreate(&ctx->ev_start));
            HIP_CHECK(hipEventCreate(&ctx->ev_stop));
            HIP_CHECK(hipEventCreate(&ctx->ev_region_start));
            HIP_CHECK(hipEventCreate(&ctx->ev_region_stop));
            HIP_CHECK(hipEventCreateWithFlags(&ctx->ev_copy_done, hipEventDisableTiming));
            for (int i = 0; i < kRingSlots; ++i) {
                HIP_CHECK(hipHostMalloc(&ctx->ring[i], kRingBytes, hipHostMallocDefault));
                HIP_CHECK(hipEventCreateWithFlags(&ctx->ring_ev[i], hipEventDisableTiming));
            }
        } catch (...) {
            fedavg_destroy(ctx);
            throw;
        }
        *out = ctx;
    });
}

int fedavg_destroy(fedavg_ctx* ctx) {
    if (!ctx) return 0;
    int rc = guarded([&] {
        (void)hipSetDevice(ctx->device);
        if (ctx->own_stream) (void)hipStreamSynchronize(ctx->own_stream);
        if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
        for (int i = 0; i < kRingSlots; ++i) {
            if (ctx->ring[i]) (void)hipHostFree(ctx->ring[i]);
            if (ctx->ring_ev[i]) (void)hipEventDestroy(ctx->ring_ev[i]);
        }
        for (hipEvent_t ev : {ctx->ev_start, ctx->ev_stop, ctx->ev_copy_done, ctx->ev_region_start, ctx->ev_region_stop})
            if (ev) (void)hipEventDestroy(ev);
        for (auto& m : ctx->marks) (void)hipEventDestroy(m.first);
        for (hipEvent_t ev : ctx->mark_pool) (void)hipEventDestroy(ev);
        if (ctx->tails_buf) (void)hipFree(ctx->tails_buf);
        if (ctx->rsqrtps) (void)hipFree(ctx->rsqrtps);
        if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
        if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    });
    delete ctx;
    return rc;
}

int fedavg_device_info(fedavg_ctx* ctx, int* num_cus, size_t* free_bytes, size_t* total_bytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        ctx->activate();
        size_t f = 0, t = 0;
        HIP_CHECK(hipMemGetInfo(&f, &t));
        if (num_cus) *num_cus = ctx->num_cus;
        if (free_bytes) *free_bytes = f;
        if (total_bytes) *total_bytes = t;
    });
}

int fedavg_set_stream(fedavg_ctx* ctx, void* stream) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        ctx->ext_stream = static_cast<hipStream_t>(stream);
    });
}

int fedavg_get_stream(fedavg_ctx* ctx, void** stream) {
    return guarded([&] {
        if (!ctx || !stream) throw Error("NULL argument");
        *stream = ctx->compute();
    });
}

int fedavg_malloc(fedavg_ctx* ctx, size_t nbytes, void** dptr) {
    return guarded([&] {
        if (!ctx || !dptr) throw Error("NULL argument");
        ctx->activate();
        *dptr = nullptr;
        if (nbytes == 0) return;
        HIP_CHECK(hipMalloc(dptr, nbytes));
    });
}

int fedavg_free(fedavg_ctx* ctx, void* dptr) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (!dptr) return;
        ctx->activate();
        HIP_CHECK(hipStreamSynchronize(ctx->compute()));
        HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));
        HIP_CHECK(hipFree(dptr));
    });
}

int fedavg_h2d(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        h2d_impl(ctx, static_cast<char*>(dst), nbytes, nbytes, 0, static_cast<const char*>(src), nbytes);
    });
}

int fedavg_h2d_tiled(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes, size_t logical_offset,
                     const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!base || !src) throw Error("NULL pointer");
        if (tile_bytes == 0 || tile_stride_bytes < tile_bytes) throw Error("bad tile geometry");
        h2d_impl(ctx, static_cast<char*>(base), tile_bytes, tile_stride_bytes, logical_offset,
                 static_cast<const char*>(src), nbytes);
    });
}

int fedavg_h2d_tiled_multi(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes, int n_pieces,
                           const size_t* logical_offsets, const void* const* srcs, const size_t* nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (n_pieces <= 0) return;
        if (!base || !logical_offsets || !srcs || !nbytes) throw Error("NULL pointer");
        if (tile_bytes == 0 || tile_stride_bytes < tile_bytes) throw Error("bad tile geometry");
        for (int i = 0; i < n_pieces; ++i)
            if (nbytes[i] && !srcs[i]) throw Error("NULL source piece");
        h2d_multi_impl(ctx, static_cast<char*>(base), tile_bytes, tile_stride_bytes, n_pieces, logical_offsets, srcs,
                       nbytes);
    });
}

int fedavg_d2d_tiled(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes, size_t logical_offset,
                     const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!base || !src) throw Error("NULL pointer");
        if (tile_bytes == 0 || tile_stride_bytes < tile_bytes) throw Error("bad tile geometry");
        ctx->activate();
        copy_into_tiles(static_cast<char*>(base), tile_bytes, tile_stride_bytes, logical_offset,
                        static_cast<const char*>(src), nbytes, hipMemcpyDeviceToDevice, ctx->compute());
    });
}

static void d2h_impl(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes);

int fedavg_d2h(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        ctx->activate();
        d2h_impl(ctx, dst, src, nbytes);
    });
}

int fedavg_d2h_multi(fedavg_ctx* ctx, void* host_base, const void* dev_base, int n, const size_t* host_offsets,
                     const size_t* dev_offsets, const size_t* nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (n < 0) throw Error("negative piece count");
        if (n == 0) return;
        if (!host_base || !dev_base || !host_offsets || !dev_offsets || !nbytes) throw Error("NULL pointer");
        ctx->activate();
        hipStream_t s = ctx->compute();
        char* h = static_cast<char*>(host_base);
        const char* d = static_cast<const char*>(dev_base);
        if (is_pinned_host(host_base)) {  // every piece straight into the page-locked destination, one sync
            for (int i = 0; i < n; ++i)
                if (nbytes[i]) HIP_CHECK(hipMemcpyAsync(h + host_offsets[i], d + dev_offsets[i], nbytes[i], hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            return;
        }
        for (int i = 0; i < n; ++i)
            if (nbytes[i]) d2h_impl(ctx, h + host_offsets[i], d + dev_offsets[i], nbytes[i]);
    });
}

// D2H on the compute stream (after the work queued on it), returning when dst holds the bytes
static void d2h_impl(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    {
        hipStream_t s = ctx->compute();
        if (nbytes < kParallelCopyMin || is_pinned_host(dst)) {
            HIP_CHECK(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            return;
        }
        // pageable destination: DMA into the pinned ring, drained by the host threads one slot behind
        for (int i = 0; i < kRingSlots; ++i)
            if (ctx->ring_used[i]) HIP_CHECK(hipEventSynchronize(ctx->ring_ev[i]));
        const size_t nchunks = (nbytes + kRingBytes - 1) / kRingBytes;
        auto issue = [&](size_t c) {
            const int slot = (int)(c % kRingSlots);
            const size_t off = c * kRingBytes, len = std::min(kRingBytes, nbytes - off);
            HIP_CHECK(hipMemcpyAsync(ctx->ring[slot], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipEventRecord(ctx->ring_ev[slot], s));
            ctx->ring_used[slot] = true;
        };
        for (size_t c = 0; c < nchunks && c < (size_t)kRingSlots; ++c) issue(c);
        for (size_t c = 0; c < nchunks; ++c) {
            const int slot = (int)(c % kRingSlots);
            const size_t off = c * kRingBytes, len = std::min(kRingBytes, nbytes - off);
            HIP_CHECK(hipEventSynchronize(ctx->ring_ev[slot]));
            parallel_memcpy(static_cast<char*>(dst) + off, ctx->ring[slot], len);
            if (c + kRingSlots < nchunks) issue(c + kRingSlots);
        }
    }
}

int fedavg_host_register(fedavg_ctx* ctx, void* p, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (!p || nbytes == 0) throw Error("nothing to register");
        ctx->activate();
        HIP_CHECK(hipHostRegister(p, nbytes, hipHostRegisterPortable));
    });
}

int fedavg_host_unregister(fedavg_ctx* ctx, void* p) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (!p) throw Error("NULL pointer");
        ctx->activate();
        HIP_CHECK(hipHostUnregister(p));
    });
}

int fedavg_mark(fedavg_ctx* ctx, size_t ready_bytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (!ctx->marks.empty() && ready_bytes < ctx->marks.back().second)
            throw Error("marks must be recorded in non-decreasing ready_bytes order");
        ctx->activate();
        hipEvent_t ev;
        if (!ctx->mark_pool.empty()) {
            ev = ctx->mark_pool.back();
            ctx->mark_pool.pop_back();
        } else {
            HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        }
        HIP_CHECK(hipEventRecord(ev, ctx->compute()));
        ctx->marks.emplace_back(ev, ready_bytes);
    });
}

int fedavg_marks_reset(fedavg_ctx* ctx) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        for (auto& m : ctx->marks) ctx->mark_pool.push_back(m.first);
        ctx->marks.clear();
    });
}

// D2H that starts while the compute stream is still producing `src`: chunk [off, off+len) leaves on the
// copy stream as soon as the first mark covering off+len has fired (an event recorded right after the
// launch that finalised those bytes), through the pinned ring drained by the host copy threads.  Bytes
// past the last mark wait for everything enqueued on the compute stream so far.  Returns when `dst` holds
// all bytes; the marks are consumed.
int fedavg_d2h_marked(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        struct Recycle {  // marks go back to the pool on every exit path
            fedavg_ctx* c;
            ~Recycle() {
                for (auto& m : c->marks) c->mark_pool.push_back(m.first);
                c->marks.clear();
            }
        } recycle{ctx};
        if (nbytes == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        ctx->activate();
        HIP_CHECK(hipEventRecord(ctx->ev_copy_done, ctx->compute()));  // "everything so far"
        size_t mi = 0;
        auto wait_ready = [&](size_t end) {
            while (mi < ctx->marks.size() && ctx->marks[mi].second < end) ++mi;
            hipEvent_t ev = mi < ctx->marks.size() ? ctx->marks[mi].first : ctx->ev_copy_done;
            HIP_CHECK(hipStreamWaitEvent(ctx->copy_stream, ev, 0));
        };
        const bool direct = nbytes < kParallelCopyMin || is_pinned_host(dst);
        const size_t chunk = direct ? std::max<size_t>(kRingBytes, 1) : kRingBytes;
        const size_t nchunks = (nbytes + chunk - 1) / chunk;
        if (direct) {
            for (size_t c = 0; c < nchunks; ++c) {
                const size_t off = c * chunk, len = std::min(chunk, nbytes - off);
                wait_ready(off + len);
                HIP_CHECK(hipMemcpyAsync(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off, len,
                                         hipMemcpyDeviceToHost, ctx->copy_stream));
            }
            HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));
            return;
        }
        for (int i = 0; i < kRingSlots; ++i)
            if (ctx->ring_used[i]) HIP_CHECK(hipEventSynchronize(ctx->ring_ev[i]));
        auto issue = [&](size_t c) {
            const int slot = (int)(c % kRingSlots);
            const size_t off = c * chunk, len = std::min(chunk, nbytes - off);
            wait_ready(off + len);
            HIP_CHECK(hipMemcpyAsync(ctx->ring[slot], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost,
                                     ctx->copy_stream));
            HIP_CHECK(hipEventRecord(ctx->ring_ev[slot], ctx->copy_stream));
            ctx->ring_used[slot] = true;
        };
        for (size_t c = 0; c < nchunks && c < (size_t)kRingSlots; ++c) issue(c);
        for (size_t c = 0; c < nchunks; ++c) {
            const int slot = (int)(c % kRingSlots);
            const size_t off = c * chunk, len = std::min(chunk, nbytes - off);
            HIP_CHECK(hipEventSynchronize(ctx->ring_ev[slot]));
            parallel_memcpy(static_cast<char*>(dst) + off, ctx->ring[slot], len);
            if (c + kRingSlots < nchunks) issue(c + kRingSlots);
        }
        // later compute (e.g. the next round reusing src) is ordered after these reads
        HIP_CHECK(hipEventRecord(ctx->ev_copy_done, ctx->copy_stream));
        HIP_CHECK(hipStreamWaitEvent(ctx->compute(), ctx->ev_copy_done, 0));
    });
}

int fedavg_d2d(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        ctx->activate();
        HIP_CHECK(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToDevice, ctx->compute()));
    });
}

int fedavg_memset(fedavg_ctx* ctx, void* dst, int value, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!dst) throw Error("NULL pointer");
        ctx->activate();
        HIP_CHECK(hipMemsetAsync(dst, value, nbytes, ctx->compute()));
    });
}

int fedavg_sync(fedavg_ctx* ctx) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        ctx->activate();
        HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));
        HIP_CHECK(hipStreamSynchronize(ctx->compute()));
    });
}

int fedavg_accumulate(fedavg_ctx* ctx, const void* const* rows, const double* weights, int k_rows,
                      const void* acc_in, void* out, size_t n, int in_dtype, int acc_dtype, int op, int fin,
                      double count) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (k_rows < 0) throw Error("k_rows < 0");
        if (k_rows == 0 && !acc_in) throw Error("k_rows == 0 requires acc_in");
        check_op_fin(op, fin);
        check_dtype(in_dtype);
        check_dtype(acc_dtype);
        const bool narrow = acc_dtype == FEDAVG_F16 || acc_dtype == FEDAVG_BF16;
        const bool int_acc = acc_dtype != FEDAVG_F32 && acc_dtype != FEDAVG_F64 && !narrow;
        if (narrow) {
            if (in_dtype != acc_dtype) throw Error("a 16-bit accumulator needs inputs of the same dtype");
        } else if (int_acc) {
            if (in_dtype != acc_dtype || op != FEDAVG_OP_UNWEIGHTED || fin != FEDAVG_FIN_NONE)
                throw Error("an integer / bool accumulator needs inputs of its dtype, FEDAVG_OP_UNWEIGHTED and "
                            "FEDAVG_FIN_NONE");
        } else if (in_dtype == FEDAVG_BF16 ||
                   (acc_dtype == FEDAVG_F32 && (in_dtype == FEDAVG_F64 || in_dtype == FEDAVG_U16 ||
                                                in_dtype == FEDAVG_U32 || in_dtype == FEDAVG_U64))) {
            throw Error("unsupported (in_dtype, acc_dtype) pair");
        }
        if (!narrow && !int_acc) normalize_wide(op, fin, count, acc_dtype == FEDAVG_F32);
        if (n == 0) {
            ctx->timed_valid = false;
            return;
        }
        if (!out) throw Error("out is NULL");
        if (k_rows > 0 && (!rows || !weights)) throw Error("rows/weights NULL");
        for (int k = 0; k < k_rows; ++k)
            if (!rows[k]) throw Error("row " + std::to_string(k) + " is NULL");
        ctx->activate();
        hipStream_t s = ctx->compute();
        TimingScope ts(ctx, s);
        if (narrow) {
            run_narrow(ctx, rows, weights, k_rows, acc_in, out, (int64_t)n, acc_dtype, op, fin, count, s);
            ts.done();
            return;
        }
        if (int_acc) {
            run_intsum(ctx, rows, k_rows, acc_in, out, (int64_t)n, acc_dtype, s);
            ts.done();
            return;
        }
        bool vec = in_dtype == FEDAVG_F32 && acc_dtype == FEDAVG_F32 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(acc_in) % 16 == 0;
        for (int k = 0; vec && k < k_rows; ++k) vec = reinterpret_cast<uintptr_t>(rows[k]) % 16 == 0;
        // contiguous rows are tiled storage with tile_stride == tile: whole tiles take the streaming kernel,
        // the ragged remainder (< one tile) the scalar kernel
        const int64_t tile = ctx->tile;
        const int64_t n_full = vec ? ((int64_t)n / tile) * tile : 0;
        if (n_full > 0) {
            run_tiles(ctx, rows, weights, k_rows, tile, tile, 0, n_full, static_cast<const float*>(acc_in),
                      static_cast<float*>(out), op, fin, count, s);
        }
        if ((int64_t)n > n_full) {
            run_generic(ctx, rows, weights, k_rows, (size_t)n_full, acc_in, out, (int64_t)n - n_full, in_dtype,
                        acc_dtype, op, fin, count, s);
        }
        ts.done();
    });
}

int fedavg_accumulate_tiled(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                            size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                            void* out, int op, int fin, double count) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (k_rows < 0 || (k_rows == 0 && !acc_in)) throw Error("k_rows == 0 requires acc_in");
        check_op_fin(op, fin);
        normalize_wide(op, fin, count, true);
        if (!valid_tile(tile_elems)) throw Error("tile_elems must be 1024, 2048, 4096 or 8192");
        if (!fedavg::kAB && tile_elems != (size_t)fedavg::kDefaultTile)
            throw Error("tile_elems " + std::to_string(tile_elems) + " is an A/B form (this product library carries 4096)");
        if (tile_stride < tile_elems || tile_stride % 4) throw Error("tile_stride must be >= tile_elems, multiple of 4");
        if (begin % 4 || end % 4 || end < begin) throw Error("begin/end must be multiples of 4 with begin <= end");
        if (end == begin) {
            ctx->timed_valid = false;
            return;
        }
        if (!out) throw Error("out is NULL");
        if (reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(acc_in) % 16)
            throw Error("out/acc_in must be 16-byte aligned");
        if (k_rows > 0 && (!bases || !weights)) throw Error("bases/weights NULL");
        for (int k = 0; k < k_rows; ++k)
            if (!bases[k] || reinterpret_cast<uintptr_t>(bases[k]) % 16)
                throw Error("base " + std::to_string(k) + " NULL or not 16-byte aligned");
        ctx->activate();
        hipStream_t s = ctx->compute();
        TimingScope ts(ctx, s);
        run_tiles(ctx, bases, weights, k_rows, (int64_t)tile_elems, (int64_t)tile_stride, (int64_t)begin, (int64_t)end,
                  static_cast<const float*>(acc_in), static_cast<float*>(out), op, fin, count, s);
        ts.done();
    });
}

int fedavg_accumulate_tiled16(fedavg_ctx* ctx, int fmt, const void* const* bases, const double* weights, int k_rows,
                              size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                              void* out, int op, int fin, double count) {
    return fedavg_accumulate_tiled16_tails(ctx, fmt, bases, weights, k_rows, tile_elems, tile_stride, begin, end, acc_in,
                                           out, op, fin, count, nullptr, 0);
}

int fedavg_accumulate_tiled16_tails(fedavg_ctx* ctx, int fmt, const void* const* bases, const double* weights,
                                    int k_rows, size_t tile_elems, size_t tile_stride, size_t begin, size_t end,
                                    const void* acc_in, void* out, int op, int fin, double count,
                                    const int64_t* tails, size_t n_tails) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (fmt != FEDAVG_F16 && fmt != FEDAVG_BF16) throw Error("fmt must be FEDAVG_F16 or FEDAVG_BF16");
        if (k_rows < 0 || (k_rows == 0 && !acc_in)) throw Error("k_rows == 0 requires acc_in");
        check_op_fin(op, fin);
        if (tile_elems != (size_t)fedavg::kTile16Elems) throw Error("tile_elems must be 4096");
        if (tile_stride < tile_elems || tile_stride % 8) throw Error("tile_stride must be >= tile_elems, multiple of 8");
        if (begin % 8 || end % 8 || end < begin) throw Error("begin/end must be multiples of 8 with begin <= end");
        if (end == begin) {
            ctx->timed_valid = false;
            return;
        }
        if (!out) throw Error("out is NULL");
        if (reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(acc_in) % 16)
            throw Error("out/acc_in must be 16-byte aligned");
        if (k_rows > 0 && (!bases || !weights)) throw Error("bases/weights NULL");
        for (int k = 0; k < k_rows; ++k)
            if (!bases[k] || reinterpret_cast<uintptr_t>(bases[k]) % 16)
                throw Error("base " + std::to_string(k) + " is NULL or not 16-byte aligned");
        if (n_tails && !tails) throw Error("tails is NULL");
        for (size_t j = 1; j < n_tails; ++j)
            if (tails[j] <= tails[j - 1]) throw Error("tails must be strictly increasing");
        ctx->activate();
        hipStream_t s = ctx->compute();
        // the second path exists only in torch's add_ with alpha: the CPU scalar remainder (FEDAVG_OP_TORCH) and
        // torch-ROCm's unrolled float16 path (FEDAVG_OP_TORCH_DEVICE)
        const int64_t* lo = tails;
        const int64_t* hi = tails;
        if ((op == FEDAVG_OP_TORCH || (op == FEDAVG_OP_TORCH_DEVICE && fmt == FEDAVG_F16)) && n_tails) {
            lo = std::lower_bound(tails, tails + n_tails, (int64_t)begin);
            hi = std::lower_bound(lo, tails + n_tails, (int64_t)end);
        }
        const int64_t m = hi - lo;
        int64_t* d_idx = nullptr;
        void* d_vals = nullptr;
        if (m) {
            const size_t need = (size_t)m * (sizeof(int64_t) + sizeof(uint16_t));
            HIP_CHECK(hipStreamSynchronize(s));  // earlier launches may still read the side buffer
            if (ctx->tails_bytes < need) {
                if (ctx->tails_buf) HIP_CHECK(hipFree(ctx->tails_buf));
                ctx->tails_buf = nullptr;
                ctx->tails_bytes = 0;
                HIP_CHECK(hipMalloc(&ctx->tails_buf, need));
                ctx->tails_bytes = need;
            }
            d_idx = static_cast<int64_t*>(ctx->tails_buf);
            d_vals = d_idx + m;
            HIP_CHECK(hipMemcpy(d_idx, lo, (size_t)m * sizeof(int64_t), hipMemcpyHostToDevice));
        }
        TimingScope ts(ctx, s);
        run_tiles_narrow(ctx, bases, weights, k_rows, (int64_t)tile_stride, (int64_t)begin, (int64_t)end, acc_in, out,
                         fmt, op, fin, count, s, d_idx, m, d_vals);
        ts.done();
    });
}

int fedavg_accumulate_tiled64(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                              size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                              void* out, int op, int fin, double count) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (k_rows < 0 || (k_rows == 0 && !acc_in)) throw Error("k_rows == 0 requires acc_in");
        check_op_fin(op, fin);
        normalize_wide(op, fin, count, false);
        if (tile_elems != (size_t)fedavg::kTile64Elems) throw Error("tile_elems must be 4096");
        if (tile_stride < tile_elems || tile_stride % 2) throw Error("tile_stride must be >= tile_elems, multiple of 2");
        if (begin % 2 || end % 2 || end < begin) throw Error("begin/end must be multiples of 2 with begin <= end");
        if (end == begin) {
            ctx->timed_valid = false;
            return;
        }
        if (!out) throw Error("out is NULL");
        if (reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(acc_in) % 16)
            throw Error("out/acc_in must be 16-byte aligned");
        if (k_rows > 0 && (!bases || !weights)) throw Error("bases/weights NULL");
        for (int k = 0; k < k_rows; ++k)
            if (!bases[k] || reinterpret_cast<uintptr_t>(bases[k]) % 16)
                throw Error("base " + std::to_string(k) + " is NULL or not 16-byte aligned");
        ctx->activate();
        hipStream_t s = ctx->compute();
        TimingScope ts(ctx, s);
        const int64_t T = fedavg::kTile64Elems;
        const int64_t n_tiles = ((int64_t)end - 1) / T - (int64_t)begin / T + 1;
        const bool burst = !(ctx->variant & fedavg::kVariantTileStores);
        // two blocks per CU at every K (198 VGPRs: both resident): 1 block at 16 / 32 / 64 clients runs 1.4 /
        // 0.8 / 0.1 points slower (profiles/r02/ab/bpc_check/f64_k*.jsonl)
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * ctx->bpc(), n_tiles));
        const double fv = fin_scalar(fin, count);
        int k0 = 0;
        const void* cur_in = acc_in;
        do {  // more clients than one kernel-argument table holds chain a partial sum through out
            const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
            fedavg::RowTableGeneric t;
            memset(&t, 0, sizeof(t));
            for (int j = 0; j < kc; ++j) {
                t.rows[j] = bases[k0 + j];
                t.w[j] = weights[k0 + j];
            }
            const bool last = k0 + kc >= k_rows;
            // 1-3 client reads without a chained sum: the fp64 few-client form (round 5); A/B builds with
            // -DFEDAVG_AB_FEW pick its geometry with launch variant bits 9-11 = 1-4
            const int few_ix = fedavg::kABFew ? (ctx->variant >> fedavg::kVariantLoopShift) & 7 : 0;
            const bool few = burst && !cur_in && kc <= fedavg::kF64FewMaxReads && !(ctx->variant & kVariantFewBurst);
            const int fgrid = few ? (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus *
                                                                                    ctx->bpc(fedavg::f64_few_form(kc, few_ix).bpc),
                                                                                n_tiles))
                                  : grid;
            HIP_CHECK(fedavg::launch_tiles_f64(t, kc, (int64_t)tile_stride, cur_in, out, (int64_t)begin, (int64_t)end,
                                               op, last ? fin : FEDAVG_FIN_NONE, fv, fgrid,
                                               few    ? 3 + (few_ix <= 4 ? few_ix : 0)
                                               : burst ? ((ctx->variant & fedavg::kVariantRegisterTiles) ? 1 : 2)
                                                       : 0,
                                               s, &ctx->launches));
            cur_in = out;
            k0 += kc;
        } while (k0 < k_rows);
        ts.done();
    });
}

int fedavg_accumulate_tiled_epi(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                                size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                                void* out, int op, int fin, double count, const fedavg_epilogue* epi) {
    return guarded([&] {
        if (!ctx || !epi) throw Error("NULL argument");
        if (epi->kind == FEDAVG_EPI_NONE) {
            if (fedavg_accumulate_tiled(ctx, bases, weights, k_rows, tile_elems, tile_stride, begin, end, acc_in, out,
                                        op, fin, count))
                throw Error(g_last_error);
            return;
        }
        if (epi->kind < FEDAVG_EPI_ADD_BASE || epi->kind > FEDAVG_EPI_ASGD) throw Error("bad epilogue kind");
        if (k_rows < 0 || (k_rows == 0 && !acc_in)) throw Error("k_rows == 0 requires acc_in");
        check_op_fin(op, fin);
        normalize_wide(op, fin, count, true);
        if (tile_elems != (size_t)fedavg::kDefaultTile)
            throw Error("the epilogue kernel runs the default tile (" + std::to_string(fedavg::kDefaultTile) + ")");
        if (tile_stride < tile_elems || tile_stride % 4) throw Error("tile_stride must be >= tile_elems, multiple of 4");
        if (begin % 4 || end % 4 || end < begin) throw Error("begin/end must be multiples of 4 with begin <= end");
        if (end == begin) return;
        auto misaligned = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 != 0; };
        if (epi->kind == FEDAVG_EPI_ADD_BASE && (!epi->base || !out)) throw Error("ADD_BASE needs base and out");
        if (epi->kind == FEDAVG_EPI_SGD && (!epi->param || (epi->momentum != 0.0 && !epi->state1)))
            throw Error("SGD needs param (and state1 with momentum)");
        if (epi->kind == FEDAVG_EPI_ADAM && (!epi->param || !epi->state1 || !epi->state2))
            throw Error("ADAM needs param, state1 (exp_avg), state2 (exp_avg_sq)");
        if (epi->kind == FEDAVG_EPI_ADAM && epi->amsgrad && !epi->state3)
            throw Error("ADAM with amsgrad needs state3 (max_exp_avg_sq)");
        if (epi->kind == FEDAVG_EPI_ADAM && epi->step < 1.0) throw Error("ADAM step must be >= 1");
        if (epi->kind == FEDAVG_EPI_ADAGRAD && (!epi->param || !epi->state1))
            throw Error("ADAGRAD needs param and state1 (sum)");
        if (epi->kind == FEDAVG_EPI_ADAGRAD && epi->step < 1.0) throw Error("ADAGRAD step must be >= 1");
        if (epi->kind == FEDAVG_EPI_RMSPROP &&
            (!epi->param || !epi->state1 || (epi->momentum != 0.0 && !epi->state2) || (epi->centered && !epi->state3)))
            throw Error("RMSPROP needs param, state1 (square_avg), state2 with momentum, state3 when centered");
        if (epi->kind == FEDAVG_EPI_ADAMAX && (!epi->param || !epi->state1 || !epi->state2))
            throw Error("ADAMAX needs param, state1 (exp_avg), state2 (exp_inf)");
        if (epi->kind == FEDAVG_EPI_ADAMAX && epi->step < 1.0) throw Error("ADAMAX step must be >= 1");
        if ((epi->kind == FEDAVG_EPI_NADAM || epi->kind == FEDAVG_EPI_RADAM) &&
            (!epi->param || !epi->state1 || !epi->state2 || epi->step < 1.0))
            throw Error("NADAM/RADAM need param, state1 (exp_avg), state2 (exp_avg_sq) and step >= 1");
        if (epi->kind == FEDAVG_EPI_RPROP && (!epi->param || !epi->state1 || !epi->state2))
            throw Error("RPROP needs param, state1 (prev), state2 (step_size)");
        if (epi->kind == FEDAVG_EPI_ASGD && (!epi->param || !epi->state1))
            throw Error("ASGD needs param and state1 (ax)");
        for (const void* p : {(const void*)epi->param, (const void*)epi->state1, (const void*)epi->state2,
                              (const void*)epi->state3, (const void*)epi->base, (const void*)out, acc_in})
            if (misaligned(p)) throw Error("epilogue/out/acc_in pointers must be 16-byte aligned");
        for (int k = 0; k < k_rows; ++k)
            if (!bases[k] || misaligned(bases[k])) throw Error("base " + std::to_string(k) + " NULL or misaligned");
        ctx->activate();
        hipStream_t s = ctx->compute();
        TimingScope ts(ctx, s);
        // Leading chunks (beyond 128 clients) accumulate a partial sum; the last chunk runs the epilogue.
        // The partial sum goes to out unless out is absent or aliases an epilogue operand (in-place
        // WEIGHT_DIFF apply: out == base) -- then to a stream-ordered scratch covering [begin, end).
        int head = k_rows > fedavg::kMaxRowsPerLaunch ? (k_rows - 1) / fedavg::kMaxRowsPerLaunch * fedavg::kMaxRowsPerLaunch : 0;
        const float* cur_in = static_cast<const float*>(acc_in);
        void* scratch = nullptr;
        if (!fedavg::epi_direct(op, fin, k_rows, acc_in != nullptr)) {
            // A fused form the product library does not carry (fedavg_internal.h epi_direct: a chained partial sum,
            // more than 128 clients, a finalisation with no clients, numpy mode with FIN_DIV, FIN_NONE with clients):
            // the plain kernels finalise d = fin(acc) into a scratch, then the server step reads it as its chained sum
            // (no clients, FIN_NONE).  The per-element sequence is the fused one, so the bits are the same.
            // the intermediate is `out` itself when it aliases no epilogue operand (the server step then reads d there and
            // writes its result over it element by element, each thread reading before writing); else a scratch
            // (no 4-byte-per-parameter scratch where the caller's output can hold d)
            const void* operands[] = {epi->base, epi->param, epi->state1, epi->state2, epi->state3};
            bool alias = !out;
            for (const void* q : operands) alias = alias || (q && q == out);
            float* d = static_cast<float*>(out);
            if (alias) {
                HIP_CHECK(hipMallocAsync(&scratch, (end - begin) * sizeof(float), s));
                d = static_cast<float*>(scratch) - begin;  // indexed by global element, touched on [begin, end)
            }
            run_tiles(ctx, bases, weights, k_rows, (int64_t)tile_elems, (int64_t)tile_stride, (int64_t)begin,
                      (int64_t)end, cur_in, d, op, fin, count, s);
            cur_in = d;
            head = k_rows;
            op = FEDAVG_OP_TORCH;
            fin = FEDAVG_FIN_NONE;
        } else if (head > 0) {
            float* partial = static_cast<float*>(out);
            const void* operands[] = {epi->base, epi->param, epi->state1, epi->state2, epi->state3};
            bool alias = !out;
            for (const void* q : operands) alias = alias || (q && q == out);
            if (alias) {
                HIP_CHECK(hipMallocAsync(&scratch, (end - begin) * sizeof(float), s));
                partial = static_cast<float*>(scratch) - begin;  // indexed by global element, touched on [begin, end)
            }
            run_tiles(ctx, bases, weights, head, (int64_t)tile_elems, (int64_t)tile_stride, (int64_t)begin,
                      (int64_t)end, cur_in, partial, op, FEDAVG_FIN_NONE, count, s);
            cur_in = partial;
        }
        fedavg::TileLaunch L;
        memset(&L.tab, 0, sizeof(L.tab));
        for (int j = head; j < k_rows; ++j) {
            L.tab.rows[j - head] = static_cast<const fedavg::f32x4*>(bases[j]);
            L.tab.w[j - head] = (float)weights[j];
        }
        L.k = k_rows - head;
        L.op = op;
        L.fin = fin;
        L.unroll = fedavg::kDefaultUnroll;
        L.variant = ctx->variant & (fedavg::kVariantEpiPrefetch | fedavg::kVariantTileStores | fedavg::kVariantAnyOrder |
                                    fedavg::kVariantRegisterTiles | fedavg::kVariantEpiNoSplit |
                                    (7 << fedavg::kVariantLoopShift));
        L.tile4 = (int64_t)tile_elems / 4;
        L.tstride4 = (int64_t)tile_stride / 4;
        L.b4 = (int64_t)begin / 4;
        L.e4 = (int64_t)end / 4;
        const int64_t n_tiles = (L.e4 - 1) / L.tile4 - L.b4 / L.tile4 + 1;
        // under kEpiBurstMinClients row reads the per-tile form; from 2 reads on its cross-tile pipelined variant
        // (Adam at 2 / 3 clients +1.8 / +1.4 and +0.9 / +1.0 points on two boxes, 1 client -1.5 / +0.1:
        // profiles/r04/s9/epi_bpc_k*.jsonl, s10/epi_pipe_k*.jsonl), unless the public variant asks for tile stores
        // (product builds: the pipelined per-tile form at every read count under kEpiBurstMinClients -- at one read it
        // carries client 0, or nothing for the server step -- and for a chained sum; the unpipelined one is A/B only)
        const int reads = L.k + (cur_in ? 1 : 0);
        // (round 5's register-held few-client fused form, A/B only, ran 53 % and was removed in round 6; the A/B builds'
        // variant bits 9-11 now pick the LDS-DMA form's geometry, fedavg_epi.h launch_epi_dma_form)
        const fedavg::EpiParams E = make_epi(ctx, *epi);
        // 1-3 client reads without a chained sum or a separate aggregate output: the LDS-DMA few-client form (round 6;
        // fedavg_epi.h fedavg_tiles_epi_dma_f32x4), one block per CU, unless the public variant asks for the per-tile
        // form (bit 2, kVariantEpiPrefetch) or tile stores (bit 3)
        const bool dma = !cur_in && L.k >= 1 && L.k <= 3 && fedavg::epi_dma_nin(E, L.k) > 0 &&
                         (!out || epi->kind == FEDAVG_EPI_ADD_BASE) &&
                         !(ctx->variant & (fedavg::kVariantEpiPrefetch | fedavg::kVariantTileStores));
        if (dma) L.variant |= fedavg::kVariantEpiDma;
        if (!dma && (reads < kEpiBurstMinClients || (!fedavg::kAB && cur_in)))
            L.variant |= (reads >= 2 || !fedavg::kAB) && !(ctx->variant & fedavg::kVariantTileStores)
                             ? fedavg::kVariantEpiPrefetch
                             : fedavg::kVariantTileStores;
        const bool burst = !dma && !(L.variant & (fedavg::kVariantEpiPrefetch | fedavg::kVariantTileStores));
        const int bpc = dma ? 1 : burst ? ctx->bpc(L.k >= fedavg::kEpiOneBlockMinK ? 1 : 2) : ctx->bpc();
        // one block per CU: the LDS-held tiles fill the CU (9 instead of 4), unless the public variant has bit 6
        if (burst && bpc == 1 && !(ctx->variant & (fedavg::kVariantWideLds | fedavg::kVariantRegisterTiles)))
            L.variant |= fedavg::kVariantWideLds;
        L.grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * bpc, n_tiles));
        L.fin_val = (float)fin_scalar(fin, count);
        L.acc_in = cur_in;
        L.out = static_cast<float*>(out);
        const hipError_t rc = fedavg::launch_tiles_epi_f32x4(L, E, s, &ctx->launches);
        if (scratch) HIP_CHECK(hipFreeAsync(scratch, s));
        HIP_CHECK(rc);
        ts.done();
    });
}

int fedavg_set_timing(fedavg_ctx* ctx, int enable) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        ctx->timing = enable != 0;
        ctx->timed_valid = false;
    });
}

int fedavg_last_kernel_ms(fedavg_ctx* ctx, float* ms) {
    return guarded([&] {
        if (!ctx || !ms) throw Error("NULL argument");
        if (!ctx->timed_valid) throw Error("no timed accumulate call (enable with fedavg_set_timing)");
        ctx->activate();
        HIP_CHECK(hipEventSynchronize(ctx->ev_stop));
        HIP_CHECK(hipEventElapsedTime(ms, ctx->ev_start, ctx->ev_stop));
    });
}

int fedavg_timing_begin(fedavg_ctx* ctx) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        ctx->activate();
        HIP_CHECK(hipEventRecord(ctx->ev_region_start, ctx->compute()));
        ctx->region_open = true;
    });
}

int fedavg_timing_end(fedavg_ctx* ctx, float* ms) {
    return guarded([&] {
        if (!ctx || !ms) throw Error("NULL argument");
        if (!ctx->region_open) throw Error("fedavg_timing_end without fedavg_timing_begin");
        ctx->activate();
        HIP_CHECK(hipEventRecord(ctx->ev_region_stop, ctx->compute()));
        HIP_CHECK(hipEventSynchronize(ctx->ev_region_stop));
        HIP_CHECK(hipEventElapsedTime(ms, ctx->ev_region_start, ctx->ev_region_stop));
        ctx->region_open = false;
    });
}

int fedavg_launch_count(fedavg_ctx* ctx, uint64_t* n) {
    return guarded([&] {
        if (!ctx || !n) throw Error("NULL argument");
        *n = ctx->launches;
    });
}

int fedavg_set_launch(fedavg_ctx* ctx, int blocks_per_cu, int unroll) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (blocks_per_cu < 0 || blocks_per_cu > 32) throw Error("blocks_per_cu out of range");
        if (unroll != 0 && unroll != 4 && unroll != 8) throw Error("unroll must be 0, 4 or 8");
        if (!fedavg::kAB && unroll == 8)
            throw Error("unroll 8 is an A/B form (this product library carries unroll 4; tools/build_rev_lib.py builds A/B libraries)");
        ctx->blocks_per_cu = blocks_per_cu;
        ctx->unroll = unroll ? unroll : fedavg::kDefaultUnroll;
    });
}

int fedavg_set_variant(fedavg_ctx* ctx, int variant) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        // bits 0-11 and 15 are public; 12-14 are set inside the library by its routing (kVariantFew, kVariantEpiDma)
        if (variant < 0 || (variant & ~(4095 | fedavg::kVariantEpiNoSplit)))
            throw Error("variant must be 0..4095, optionally with bit 15 (32768)");
        const int accepted = fedavg::kVariantProductMask | (fedavg::kABFew ? 7 << fedavg::kVariantLoopShift | kVariantFewBurst : 0);
        if (!fedavg::kAB && (variant & ~accepted))
            throw Error("variant bits " + std::to_string(variant & ~accepted) +
                        " are A/B forms this product library does not carry (it accepts bits 2, 4, 6 and 15; "
                        "tools/build_rev_lib.py builds A/B libraries)");
        ctx->variant = variant;
    });
}

int fedavg_set_tile(fedavg_ctx* ctx, int tile_elems) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (tile_elems == 0) tile_elems = fedavg::kDefaultTile;
        if (!valid_tile((size_t)tile_elems)) throw Error("tile_elems must be 1024, 2048, 4096 or 8192");
        if (!fedavg::kAB && tile_elems != fedavg::kDefaultTile)
            throw Error("tile_elems " + std::to_string(tile_elems) +
                        " is an A/B form (this product library carries 4096; tools/build_rev_lib.py builds A/B libraries)");
        ctx->tile = tile_elems;
    });
}

int fedavg_dequantize(fedavg_ctx* ctx, const fedavg_quant* qs, const void* q, size_t n, float* out_base,
                      size_t tile_elems, size_t tile_stride, size_t logical_offset) {
    return guarded([&] {
        if (!ctx || !qs) throw Error("NULL argument");
        if (n == 0) return;
        if (!q || !out_base) throw Error("q / out_base is NULL");
        if (qs->qtype < FEDAVG_Q_F16 || qs->qtype > FEDAVG_Q_ADA_U16) throw Error("bad qtype");
        const bool blocked = qs->qtype == FEDAVG_Q_BLOCKWISE8 || qs->qtype == FEDAVG_Q_FP4 || qs->qtype == FEDAVG_Q_NF4;
        if (blocked && (!qs->absmax || qs->blocksize == 0 || qs->blocksize % 4))
            throw Error("blocked formats need absmax and a blocksize that is a positive multiple of 4");
        if (qs->qtype == FEDAVG_Q_BLOCKWISE8 && !qs->code) throw Error("blockwise8 needs code");
        if (qs->qtype >= FEDAVG_Q_ADA_U8 && qs->has_norm && !(qs->level > 0.0)) throw Error("adaquant needs level > 0");
        if (tile_elems == 0) tile_elems = tile_stride = (logical_offset + n + 3) / 4 * 4;
        if (tile_stride < tile_elems || tile_elems % 4 || tile_stride % 4 || logical_offset % 4)
            throw Error("tile_elems, tile_stride and logical_offset must be multiples of 4, stride >= tile");
        if (reinterpret_cast<uintptr_t>(out_base) % 16) throw Error("out_base must be 16-byte aligned");
        ctx->activate();
        fedavg::DequantLaunch L;
        L.qtype = qs->qtype;
        L.q = q;
        L.n = (int64_t)n;
        L.absmax = qs->absmax;
        L.code = qs->code;
        L.blocksize = blocked ? (int64_t)qs->blocksize : 1;
        L.norm = qs->norm;
        L.level = qs->level;
        L.offset = qs->offset;
        L.has_norm = qs->has_norm;
        L.out = out_base;
        L.tile = (int64_t)tile_elems;
        L.tstride = (int64_t)tile_stride;
        L.elem0 = (int64_t)logical_offset;
        L.grid = stream_grid(ctx, ((int64_t)n + 3) / 4);
        HIP_CHECK(fedavg::launch_dequant_f32(L, ctx->compute()));
        ++ctx->launches;
    });
}

int fedavg_fill_synthetic_f32(fedavg_ctx* ctx, float* dst, size_t n, size_t tile_elems, size_t tile_stride,
                              uint64_t seed, uint64_t row, uint64_t col0) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (n == 0) return;
        if (!dst) throw Error("dst is NULL");
        if (tile_elems == 0) tile_elems = tile_stride = n;
        if (tile_stride < tile_elems) throw Error("tile_stride < tile_elems");
        ctx->activate();
        HIP_CHECK(fedavg::launch_fill_synthetic_f32(dst, (int64_t)n, (int64_t)tile_elems, (int64_t)tile_stride, seed,
                                                    row, col0, stream_grid(ctx, (int64_t)n), ctx->compute()));
    });
}

int fedavg_sqrt_f32(fedavg_ctx* ctx, const float* x, float* out, size_t n, int torch_sqrt) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (n == 0) return;
        if (!x || !out) throw Error("NULL pointer");
        ctx->activate();
        const int grid = (int)std::min<size_t>((size_t)ctx->num_cus * 8, (n + fedavg::kBlock - 1) / fedavg::kBlock);
        if (torch_sqrt != FEDAVG_SQRT_IEEE && torch_sqrt != FEDAVG_SQRT_TORCH_AVX512 && torch_sqrt != FEDAVG_SQRT_TORCH_AMD)
            throw Error("torch_sqrt must be FEDAVG_SQRT_IEEE, _TORCH_AVX512 or _TORCH_AMD");
        if (torch_sqrt == FEDAVG_SQRT_TORCH_AMD && !ctx->rsqrtps)
            throw Error("FEDAVG_SQRT_TORCH_AMD needs this host's RSQRTPS table first (fedavg_set_rsqrtps_table)");
        HIP_CHECK(fedavg::launch_sqrt_f32(x, out, (int64_t)n, torch_sqrt, ctx->rsqrtps, grid, ctx->compute()));
    });
}

int fedavg_host_rsqrtps_table(uint16_t* table, size_t n) {
    return guarded([&] {
        if (!table) throw Error("table is NULL");
        if (n != kRsqrtpsEntries) throw Error("the RSQRTPS table has 8192 entries");
        // every fp32 of [1, 4), four per RSQRTPS: the estimate must have exponent 126, 11 clear low bits and one
        // value per 2^11-input block (a function of the exponent parity and the top 12 mantissa bits), which is the
        // shape the device sqrt (fedavg_arith.h sqrt_mkl_rsqrtps) indexes
        for (uint32_t b = 0x3F800000u; b < 0x40800000u; b += 4) {
            alignas(16) uint32_t in[4] = {b, b + 1, b + 2, b + 3}, est[4];
            __m128 v;
            memcpy(&v, in, 16);
            const __m128 r = _mm_rsqrt_ps(v);
            memcpy(est, &r, 16);
            for (int j = 0; j < 4; ++j) {
                const uint32_t off = in[j] - 0x3F800000u;
                if ((est[j] >> 23) != 126u || (est[j] & 0x7FFu) != 0u)
                    throw Error("this CPU's RSQRTPS estimate of " + std::to_string(in[j]) +
                                " is not a 12-bit estimate in [0.5, 1)");
                const uint16_t e12 = (uint16_t)((est[j] >> 11) & 0xFFFu);
                if ((off & 0x7FFu) == 0u) {
                    table[off >> 11] = e12;
                } else if (table[off >> 11] != e12) {
                    throw Error("this CPU's RSQRTPS depends on more than the top 12 mantissa bits");
                }
            }
        }
    });
}

int fedavg_set_rsqrtps_table(fedavg_ctx* ctx, const uint16_t* table, size_t n) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (!table) throw Error("table is NULL");
        if (n != kRsqrtpsEntries) throw Error("the RSQRTPS table has 8192 entries");
        std::vector<uint32_t> words(kRsqrtpsEntries / 2);
        for (size_t i = 0; i < words.size(); ++i) {
            if (table[2 * i] > 0xFFFu || table[2 * i + 1] > 0xFFFu) throw Error("RSQRTPS table entries are 12-bit");
            words[i] = (uint32_t)table[2 * i] | ((uint32_t)table[2 * i + 1] << 16);  // low half first
        }
        ctx->activate();
        if (!ctx->rsqrtps) HIP_CHECK(hipMalloc(&ctx->rsqrtps, words.size() * sizeof(uint32_t)));
        // ordered behind every earlier launch on the compute stream (one may be reading the old table)
        HIP_CHECK(hipStreamSynchronize(ctx->compute()));
        HIP_CHECK(hipMemcpy(ctx->rsqrtps, words.data(), words.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    });
}

int fedavg_gather_f32(fedavg_ctx* ctx, const float* src, const uint64_t* idx, size_t m, float* host_out) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (m == 0) return;
        if (!src || !idx || !host_out) throw Error("NULL pointer");
        ctx->activate();
        hipStream_t s = ctx->compute();
        uint64_t* d_idx = nullptr;
        float* d_out = nullptr;
        HIP_CHECK(hipMalloc(&d_idx, m * sizeof(uint64_t)));
        hipError_t e = hipMalloc(&d_out, m * sizeof(float));
        if (e != hipSuccess) {
            (void)hipFree(d_idx);
            HIP_CHECK(e);
        }
        try {
            HIP_CHECK(hipMemcpyAsync(d_idx, idx, m * sizeof(uint64_t), hipMemcpyHostToDevice, s));
            HIP_CHECK(fedavg::launch_gather_f32(src, d_idx, d_out, (int64_t)m, s));
            HIP_CHECK(hipMemcpyAsync(host_out, d_out, m * sizeof(float), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        } catch (...) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(d_idx);
            (void)hipFree(d_out);
            throw;
        }
        HIP_CHECK(hipFree(d_idx));
        HIP_CHECK(hipFree(d_out));
    });
}

}  // extern "C"
