// fedavg_capi.cpp -- C-ABI of libnvflare_amd_fedavg.so (see include/nvflare_amd_fedavg.h).
//
// House conventions of the reference's only C-ABI (integration/xgboost/encryption_plugins/shared/
// plugins/plugin_main.cc:24-111): opaque handle, int rc, thread-local last-error string, every entry
// point wrapped so that no C++ exception crosses the boundary.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
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

#define HIP_CHECK(expr)                                                                                 \
    do {                                                                                                \
        hipError_t _e = (expr);                                                                         \
        if (_e != hipSuccess) {                                                                         \
            throw Error(std::string(#expr) + " failed: " + hipGetErrorName(_e) + " (" + hipGetErrorString(_e) + \
                        ")");                                                                           \
        }                                                                                               \
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

constexpr int kRingSlots = 4;
constexpr size_t kRingBytes = 64ull << 20;  // 64 MiB per pinned slot
constexpr size_t kParallelCopyMin = 8ull << 20;
constexpr int kCopyThreads = 8;

size_t dtype_size(int dt) {
    switch (dt) {
        case FEDAVG_F32:
        case FEDAVG_I32:
            return 4;
        case FEDAVG_F64:
        case FEDAVG_I64:
            return 8;
        default:
            throw Error("unknown dtype " + std::to_string(dt));
    }
}

void parallel_memcpy(void* dst, const void* src, size_t n) {
    if (n < kParallelCopyMin) {
        memcpy(dst, src, n);
        return;
    }
    const int nt = kCopyThreads;
    const size_t chunk = ((n + nt - 1) / nt + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t) {
        const size_t off = (size_t)t * chunk;
        if (off >= n) break;
        const size_t len = std::min(chunk, n - off);
        th.emplace_back([=] { memcpy(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off, len); });
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
    int blocks_per_cu = 0;  // 0 = default
    int unroll = 0;         // 0 = default
    int variant = 0;        // streaming-kernel variant (bit 0: 2 columns per lane, bit 1: temporal loads)

    hipStream_t compute() const { return ext_stream ? ext_stream : own_stream; }
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
    const int bpc = ctx->blocks_per_cu > 0 ? ctx->blocks_per_cu : 8;
    const int64_t cap = (int64_t)ctx->num_cus * bpc;
    const int64_t need = (work_items + fedavg::kBlock - 1) / fedavg::kBlock;
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, need));
}

// streaming kernel grid: tiles of (VEC * kBlock) float4
int stream_grid_tiles(const fedavg_ctx* ctx, int64_t n4) {
    const int vec = (ctx->variant & 1) ? 2 : 1;
    return stream_grid(ctx, (n4 + vec - 1) / vec);
}

// H2D of `height` rows; pageable sources go through the pinned ring (memcpy on the host threads,
// DMA on the copy stream, overlapped slot by slot).  The compute stream waits on the copies.
void h2d_impl(fedavg_ctx* ctx, char* dst, size_t dpitch, const char* src, size_t spitch, size_t width,
              size_t height) {
    if (width == 0 || height == 0) return;
    ctx->activate();
    const bool contiguous = (dpitch == width && spitch == width);
    if (is_pinned_host(src)) {
        if (contiguous) {
            HIP_CHECK(hipMemcpyAsync(dst, src, width * height, hipMemcpyHostToDevice, ctx->copy_stream));
        } else {
            HIP_CHECK(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyHostToDevice,
                                       ctx->copy_stream));
        }
        // the caller may reuse a pinned source right after return: wait for this copy
        HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));
        return;
    }
    if (contiguous) {
        width = width * height;
        height = 1;
        dpitch = spitch = width;
    }
    for (size_t r = 0; r < height; ++r) {
        size_t off = 0;
        while (off < width) {
            const int slot = ctx->ring_next;
            ctx->ring_next = (ctx->ring_next + 1) % kRingSlots;
            if (ctx->ring_used[slot]) HIP_CHECK(hipEventSynchronize(ctx->ring_ev[slot]));
            const size_t len = std::min(kRingBytes, width - off);
            parallel_memcpy(ctx->ring[slot], src + r * spitch + off, len);
            HIP_CHECK(hipMemcpyAsync(dst + r * dpitch + off, ctx->ring[slot], len, hipMemcpyHostToDevice,
                                     ctx->copy_stream));
            HIP_CHECK(hipEventRecord(ctx->ring_ev[slot], ctx->copy_stream));
            ctx->ring_used[slot] = true;
            off += len;
        }
    }
    HIP_CHECK(hipEventRecord(ctx->ev_copy_done, ctx->copy_stream));
    HIP_CHECK(hipStreamWaitEvent(ctx->compute(), ctx->ev_copy_done, 0));
}

}  // namespace

extern "C" {

const char* fedavg_last_error(void) { return g_last_error.c_str(); }

int fedavg_abi_version(void) { return FEDAVG_ABI_VERSION; }

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
            HIP_CHECK(hipEventCreateWithFlags(&ctx->ev_copy_done, hipEventDisableTiming));
            HIP_CHECK(hipEventCreate(&ctx->ev_region_start));
            HIP_CHECK(hipEventCreate(&ctx->ev_region_stop));
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
        if (ctx->ev_start) (void)hipEventDestroy(ctx->ev_start);
        if (ctx->ev_stop) (void)hipEventDestroy(ctx->ev_stop);
        if (ctx->ev_copy_done) (void)hipEventDestroy(ctx->ev_copy_done);
        if (ctx->ev_region_start) (void)hipEventDestroy(ctx->ev_region_start);
        if (ctx->ev_region_stop) (void)hipEventDestroy(ctx->ev_region_stop);
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
        h2d_impl(ctx, static_cast<char*>(dst), nbytes, static_cast<const char*>(src), nbytes, nbytes, 1);
    });
}

int fedavg_h2d_2d(fedavg_ctx* ctx, void* dst, size_t dst_pitch, const void* src, size_t src_pitch, size_t width,
                  size_t height) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (width == 0 || height == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        if (dst_pitch < width || src_pitch < width) throw Error("pitch smaller than width");
        h2d_impl(ctx, static_cast<char*>(dst), dst_pitch, static_cast<const char*>(src), src_pitch, width, height);
    });
}

int fedavg_d2h(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (nbytes == 0) return;
        if (!dst || !src) throw Error("NULL pointer");
        ctx->activate();
        HIP_CHECK(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToHost, ctx->compute()));
        HIP_CHECK(hipStreamSynchronize(ctx->compute()));
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
        if (!ctx->timed_valid) throw Error("no timed fedavg_accumulate call (enable with fedavg_set_timing)");
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

int fedavg_set_variant(fedavg_ctx* ctx, int variant) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (variant < 0 || variant > 15) throw Error("variant must be 0..15");
        ctx->variant = variant;
    });
}

int fedavg_set_launch(fedavg_ctx* ctx, int blocks_per_cu, int unroll) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (blocks_per_cu < 0 || blocks_per_cu > 64) throw Error("blocks_per_cu out of range");
        if (unroll != 0 && unroll != 4 && unroll != 8 && unroll != 16) throw Error("unroll must be 0, 4, 8 or 16");
        ctx->blocks_per_cu = blocks_per_cu;
        ctx->unroll = unroll;
    });
}

int fedavg_accumulate(fedavg_ctx* ctx, const void* const* rows, const double* weights, int k_rows,
                      const void* acc_in, void* out, size_t n, int in_dtype, int acc_dtype, int op, int fin,
                      double count) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (k_rows < 0) throw Error("k_rows < 0");
        if (k_rows == 0 && !acc_in) throw Error("k_rows == 0 requires acc_in");
        if (op < FEDAVG_OP_NUMPY || op > FEDAVG_OP_UNWEIGHTED) throw Error("bad op");
        if (fin < FEDAVG_FIN_NONE || fin > FEDAVG_FIN_DIV) throw Error("bad fin");
        const size_t in_sz = dtype_size(in_dtype);
        const size_t acc_sz = dtype_size(acc_dtype);
        (void)in_sz;
        if (acc_dtype != FEDAVG_F32 && acc_dtype != FEDAVG_F64) throw Error("acc_dtype must be F32 or F64");
        const bool pair_ok = (acc_dtype == FEDAVG_F32 && in_dtype != FEDAVG_F64) || acc_dtype == FEDAVG_F64;
        if (!pair_ok) throw Error("unsupported (in_dtype, acc_dtype) pair");
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
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->ev_start, s));

        // finalisation scalar, computed on the host exactly as the reference computes it:
        //   numpy  T * (1.0 / count): python fp64 reciprocal, then cast to the array dtype
        //   torch  T.div_(count):     the scalar operand cast to the tensor dtype
        const double fin_d = (fin == FEDAVG_FIN_SCALE) ? (1.0 / count) : count;

        const bool vec_ok = in_dtype == FEDAVG_F32 && acc_dtype == FEDAVG_F32;
        bool aligned = vec_ok && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                       (!acc_in || reinterpret_cast<uintptr_t>(acc_in) % 16 == 0);
        for (int k = 0; aligned && k < k_rows; ++k) aligned = reinterpret_cast<uintptr_t>(rows[k]) % 16 == 0;

        // chunks of at most kMaxRowsPerLaunch rows; each later chunk continues in place through `out`
        int k0 = 0;
        const void* cur_in = acc_in;
        do {
            const int kc = std::min(k_rows - k0, fedavg::kMaxRowsPerLaunch);
            const bool last = (k0 + kc >= k_rows);
            const int fin_c = last ? fin : FEDAVG_FIN_NONE;
            if (aligned) {
                fedavg::RowTableF32 tab;
                memset(&tab, 0, sizeof(tab));
                for (int j = 0; j < kc; ++j) {
                    tab.rows[j] = static_cast<const fedavg::f32x4*>(rows[k0 + j]);
                    tab.w[j] = (float)weights[k0 + j];  // fp64 host weight -> fp32, round to nearest
                }
                const int64_t n4 = (int64_t)(n / 4);
                const int64_t tail = (int64_t)(n % 4);
                if (n4 > 0) {
                    HIP_CHECK(fedavg::launch_rows_f32x4(tab, kc, static_cast<const float*>(cur_in),
                                                        static_cast<float*>(out), n4, op, fin_c, (float)fin_d,
                                                        stream_grid_tiles(ctx, n4), ctx->unroll, ctx->variant, s));
                }
                if (tail > 0) {
                    fedavg::RowTableGeneric gt;
                    memset(&gt, 0, sizeof(gt));
                    for (int j = 0; j < kc; ++j) {
                        gt.rows[j] = static_cast<const float*>(rows[k0 + j]) + n4 * 4;
                        gt.w[j] = (double)(float)weights[k0 + j];
                    }
                    const void* tin = cur_in ? static_cast<const void*>(static_cast<const float*>(cur_in) + n4 * 4)
                                             : nullptr;
                    HIP_CHECK(fedavg::launch_rows_generic(gt, kc, tin, static_cast<float*>(out) + n4 * 4, tail,
                                                          FEDAVG_F32, FEDAVG_F32, op, fin_c, (double)(float)fin_d, 1,
                                                          s));
                }
            } else {
                fedavg::RowTableGeneric gt;
                memset(&gt, 0, sizeof(gt));
                for (int j = 0; j < kc; ++j) {
                    gt.rows[j] = rows[k0 + j];
                    // weight rounded to the accumulator type on the host (the kernel's cast is then exact)
                    gt.w[j] = acc_dtype == FEDAVG_F32 ? (double)(float)weights[k0 + j] : weights[k0 + j];
                }
                const double fv = acc_dtype == FEDAVG_F32 ? (double)(float)fin_d : fin_d;
                HIP_CHECK(fedavg::launch_rows_generic(gt, kc, cur_in, out, (int64_t)n, in_dtype, acc_dtype, op, fin_c,
                                                      fv, stream_grid(ctx, (int64_t)n), s));
            }
            (void)acc_sz;
            cur_in = out;
            k0 += kc;
        } while (k0 < k_rows);

        if (ctx->timing) {
            HIP_CHECK(hipEventRecord(ctx->ev_stop, s));
            ctx->timed_valid = true;
        }
    });
}

int fedavg_accumulate_tiled(fedavg_ctx* ctx, const void* slab, size_t tile_elems, size_t seg_stride, size_t tile_stride,
                            int k_max, const int* slots, const double* weights, int k_rows, const void* acc_in, void* out,
                            size_t n, int op, int fin, double count) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (k_rows < 0 || (k_rows == 0 && !acc_in)) throw Error("k_rows == 0 requires acc_in");
        if (k_rows > fedavg::kMaxRowsPerLaunch) throw Error("tiled path takes at most 128 rows per call");
        if (tile_elems != 1024 && tile_elems != 2048 && tile_elems != 4096 && tile_elems != 8192)
            throw Error("tile_elems must be 1024, 2048, 4096 or 8192");
        if (seg_stride < tile_elems || seg_stride % 4 || tile_stride % 4 || k_max <= 0 ||
            tile_stride < (size_t)k_max * seg_stride)
            throw Error("need seg_stride >= tile_elems, tile_stride >= k_max * seg_stride, both multiples of 4");
        if (n % 4 != 0) throw Error("tiled path needs n % 4 == 0");
        if (op < FEDAVG_OP_NUMPY || op > FEDAVG_OP_UNWEIGHTED || fin < FEDAVG_FIN_NONE || fin > FEDAVG_FIN_DIV)
            throw Error("bad op/fin");
        if (n == 0) return;
        if (!slab || !out) throw Error("NULL pointer");
        if (reinterpret_cast<uintptr_t>(slab) % 16 || reinterpret_cast<uintptr_t>(out) % 16 ||
            reinterpret_cast<uintptr_t>(acc_in) % 16)
            throw Error("tiled path needs 16-byte aligned slab/out/acc_in");
        fedavg::SlotTableF32 tab;
        memset(&tab, 0, sizeof(tab));
        for (int j = 0; j < k_rows; ++j) {
            if (slots[j] < 0 || slots[j] >= k_max) throw Error("slot out of range");
            tab.slot[j] = slots[j];
            tab.w[j] = (float)weights[j];
        }
        ctx->activate();
        hipStream_t s = ctx->compute();
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->ev_start, s));
        const double fin_d = (fin == FEDAVG_FIN_SCALE) ? (1.0 / count) : count;
        const int64_t n4 = (int64_t)(n / 4);
        const int64_t tile4 = (int64_t)(tile_elems / 4);
        const int64_t n_tiles = (n4 + tile4 - 1) / tile4;
        const int bpc = ctx->blocks_per_cu > 0 ? ctx->blocks_per_cu : 2;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cus * bpc, n_tiles));
        HIP_CHECK(fedavg::launch_tiled_f32x4(tab, k_rows, static_cast<const float*>(slab), (int64_t)seg_stride / 4,
                                             (int64_t)tile_stride / 4, tile4, static_cast<const float*>(acc_in),
                                             static_cast<float*>(out), n4, op, fin, (float)fin_d, grid, ctx->unroll,
                                             ctx->variant, s));
        if (ctx->timing) {
            HIP_CHECK(hipEventRecord(ctx->ev_stop, s));
            ctx->timed_valid = true;
        }
    });
}

int fedavg_fill_synthetic_tiled_f32(fedavg_ctx* ctx, float* slab, int k_max, size_t tile_elems, size_t seg_stride,
                                    size_t tile_stride, size_t n, uint64_t seed, uint64_t col0) {
    return guarded([&] {
        if (!ctx || !slab) throw Error("NULL argument");
        if (seg_stride < tile_elems || tile_stride < (size_t)k_max * seg_stride) throw Error("bad strides");
        const int64_t n_tiles = (int64_t)((n + tile_elems - 1) / tile_elems);
        const int64_t total = n_tiles * (int64_t)k_max * (int64_t)tile_elems;
        ctx->activate();
        HIP_CHECK(fedavg::launch_fill_synthetic_tiled_f32(slab, k_max, (int64_t)tile_elems, (int64_t)seg_stride,
                                                          (int64_t)tile_stride, (int64_t)n, seed, col0,
                                                          stream_grid(ctx, total), ctx->compute()));
    });
}

int fedavg_fill_synthetic_f32(fedavg_ctx* ctx, float* dst, size_t n, uint64_t seed, uint64_t row, uint64_t col0) {
    return guarded([&] {
        if (!ctx) throw Error("ctx is NULL");
        if (n == 0) return;
        if (!dst) throw Error("dst is NULL");
        ctx->activate();
        HIP_CHECK(fedavg::launch_fill_synthetic_f32(dst, (int64_t)n, seed, row, col0, stream_grid(ctx, (int64_t)n),
                                                    ctx->compute()));
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
