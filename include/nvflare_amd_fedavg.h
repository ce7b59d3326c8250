/*
 * nvflare_amd_fedavg.h -- C-ABI of the MI355X (gfx950) FedAvg weighted-aggregation library
 * (libnvflare_amd_fedavg.so).
 *
 * This is the drop-in boundary: NVFlare's Aggregator surface is Python
 * (nvflare/app_common/abstract/aggregator.py:22-58); the Python adapter in nvflare_amd/ binds the
 * entry points below with ctypes (INTEGRATION.md shows the binding).  The reference has no native
 * code on this path: every entry point replaces a Python/numpy/torch operation, cited per function.
 *
 * Conventions follow the reference's own C-ABI (integration/xgboost/encryption_plugins/shared/
 * plugins/plugin_main.cc:24-111): an opaque handle, int return code (0 = success), a thread-local
 * error string (fedavg_last_error), and no C++ exception ever crosses the ABI.  Plain pointers and
 * sizes only; no torch types.  One handle is used by one host thread at a time (the adapter holds a
 * lock, mirroring weighted_aggregation_helper.py:162,228).
 *
 * Device pointers passed to fedavg_accumulate may come from fedavg_malloc or from any other HIP
 * allocation on the handle's device (e.g. a torch tensor's data_ptr(): zero-copy hand-off).
 */
#ifndef NVFLARE_AMD_FEDAVG_H
#define NVFLARE_AMD_FEDAVG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever a struct layout or an entry point changes (v3: Rprop / ASGD fields appended to struct
 * fedavg_epilogue; v4: fedavg_launch_count; v5: fedavg_d2h_multi; v6: fedavg_accumulate_tiled16_tails and
 * integer accumulators in fedavg_accumulate; v7: fedavg_epilogue.torch_sqrt; v8: its FEDAVG_SQRT_* values; v9:
 * fedavg_host_rsqrtps_table / fedavg_set_rsqrtps_table -- FEDAVG_SQRT_TORCH_AMD uses the host CPU's RSQRTPS captured at
 * run time instead of a table compiled in).  fedavg_struct_size() lets a binding check each struct's size as well. */
#define FEDAVG_ABI_VERSION 9

/* element types of client rows (in_dtype) and of the running sum / result (acc_dtype) */
enum fedavg_dtype {
    FEDAVG_F32 = 0,
    FEDAVG_F64 = 1,
    FEDAVG_I32 = 2,
    FEDAVG_I64 = 3,
    FEDAVG_F16 = 4,  /* IEEE binary16 (numpy float16 / torch.float16) */
    FEDAVG_BF16 = 5, /* bfloat16 (torch.bfloat16) */
    FEDAVG_U8 = 6,
    FEDAVG_I8 = 7,
    FEDAVG_I16 = 8,
    FEDAVG_BOOL = 9, /* one byte, 0 or 1 */
    FEDAVG_U16 = 10,
    FEDAVG_U32 = 11,
    FEDAVG_U64 = 12,
};

/* per-step arithmetic, reference weighted_aggregation_helper.py:
 *   FEDAVG_OP_NUMPY      first T = v*w, then T = T + v*w  (two roundings per step)   :188-193, :210-214
 *   FEDAVG_OP_TORCH      first T = v*w, then T = fma(v, w, T) (torch add_ alpha)     :181-187, :203-209
 *   FEDAVG_OP_UNWEIGHTED first T = v,   then T = T + v (weigh_by_local_iter=False)   :186-199, :208-215 */
enum fedavg_op {
    FEDAVG_OP_NUMPY = 0,
    FEDAVG_OP_TORCH = 1,
    FEDAVG_OP_UNWEIGHTED = 2,
    /* torch-ROCm's GPU kernels, for device-resident tensors: the steps of FEDAVG_OP_TORCH, except that a
     * float16 / bfloat16 total keeps alpha in fp32 (the GPU add_ converts alpha to its fp32 opmath type, the
     * CPU kernel to the tensor dtype):  first r(v*float(w))  step r(fma(v, float(w), T)).  Elements listed to
     * fedavg_accumulate_tiled16_tails (float16 only) take torch-ROCm's unrolled path instead, where the fma is
     * rounded once, straight to fp16 (v_fma_mixlo_f16)  (v6) */
    FEDAVG_OP_TORCH_DEVICE = 3,
};

/* finalisation after the last row, reference get_result (:226-240):
 *   FEDAVG_FIN_NONE   keep the running sum (a later call continues it through acc_in)
 *   FEDAVG_FIN_SCALE  numpy: T * acc_t(1.0 / count)                                   :236
 *   FEDAVG_FIN_DIV    torch: T / acc_t(count), correctly rounded                         :233 */
enum fedavg_fin {
    FEDAVG_FIN_NONE = 0,
    FEDAVG_FIN_SCALE = 1,
    FEDAVG_FIN_DIV = 2,
    /* torch-ROCm's div_ by a CPU scalar on device-resident tensors: a multiplication by the reciprocal, the
     * fp64 quotient cast to the opmath type: T * (float)(1.0 / count) for fp32 / float16 / bfloat16 totals
     * (rounded to the total's format), T * (1.0 / count) for fp64 (v6) */
    FEDAVG_FIN_RECIP = 3,
};

/* server-optimizer epilogue fused behind the finalisation (fedavg_accumulate_tiled_epi) */
enum fedavg_epi {
    FEDAVG_EPI_NONE = 0,
    FEDAVG_EPI_ADD_BASE = 1, /* w = base + d        full_model_shareable_generator.py:58-67 */
    FEDAVG_EPI_SGD = 2,      /* torch SGD on g = -d   app_opt/pt/fedopt.py:157-182 */
    FEDAVG_EPI_ADAM = 3,     /* torch Adam/AdamW on g = -d  (torch/optim/adam.py:347-551) */
    FEDAVG_EPI_ADAGRAD = 4,  /* torch Adagrad on g = -d  (torch/optim/adagrad.py _single_tensor_adagrad) */
    FEDAVG_EPI_RMSPROP = 5,  /* torch RMSprop on g = -d  (torch/optim/rmsprop.py _single_tensor_rmsprop) */
    FEDAVG_EPI_ADAMAX = 6,   /* torch Adamax on g = -d  (torch/optim/adamax.py _single_tensor_adamax) */
    FEDAVG_EPI_NADAM = 7,    /* torch NAdam on g = -d  (torch/optim/nadam.py _single_tensor_nadam) */
    FEDAVG_EPI_RADAM = 8,    /* torch RAdam on g = -d  (torch/optim/radam.py _single_tensor_radam) */
    FEDAVG_EPI_RPROP = 9,    /* torch Rprop on g = -d  (torch/optim/rprop.py _single_tensor_rprop) */
    FEDAVG_EPI_ASGD = 10,    /* torch ASGD on g = -d  (torch/optim/asgd.py _single_tensor_asgd) */
};

/* fedavg_epilogue.torch_sqrt (v8): the sqrt of the reference's server step, torch CPU's Tensor.sqrt on the host it runs
 * on (nvflare_amd/torch_sqrt.py picks it by probing that host's torch) */
enum fedavg_sqrt {
    FEDAVG_SQRT_IEEE = 0,           /* correctly rounded */
    FEDAVG_SQRT_TORCH_AVX512 = 1,   /* MKL vsSqrt, AVX-512 path (Intel): VRSQRT14PS estimate + one Newton step */
    FEDAVG_SQRT_TORCH_AMD = 2,      /* MKL vsSqrt, SSE4.2 / AVX path (AMD EPYC): the host's RSQRTPS + a Newton step;
                                       needs fedavg_set_rsqrtps_table on the handle first (v9) */
};

typedef struct fedavg_epilogue {
    int kind;                   /* enum fedavg_epi */
    int first_step;             /* SGD: the momentum buffer starts as a clone of the gradient */
    int nesterov;               /* SGD */
    int maximize;               /* SGD/Adam: optimise the positive update */
    int decoupled_weight_decay; /* Adam: AdamW */
    double lr, momentum, dampening, weight_decay;
    double beta1, beta2, eps;
    double step;                /* Adam: step count after this update (1, 2, ...) */
    float* param;               /* SGD/Adam: flat fp32 params, updated in place */
    float* state1;              /* SGD momentum buffer / Adam exp_avg (in place) */
    float* state2;              /* Adam exp_avg_sq / Adamax exp_inf (in place) */
    const float* base;          /* ADD_BASE: flat fp32 base weights (out may alias it) */
    int amsgrad;                /* Adam: normalise by max_exp_avg_sq = max(max_exp_avg_sq, exp_avg_sq) */
    float* state3;              /* Adam amsgrad: max_exp_avg_sq (in place) */
    double lr_decay;            /* Adagrad: clr = lr / (1 + (step - 1) * lr_decay); state1 = sum, eps */
    double alpha;               /* RMSprop: smoothing constant; state1 = square_avg, state2 = momentum_buffer */
    int centered;               /* RMSprop: state3 = grad_avg */
    double momentum_decay;      /* NAdam: mu_t = beta1 * (1 - 0.5 * 0.96^(step * momentum_decay)) */
    double mu_product;          /* NAdam: the fp32 mu_product state BEFORE this step (1.0 at the first) */
    double etaminus, etaplus;   /* Rprop: etas; state1 = prev, state2 = step_size (lr-filled before step 1) */
    double step_size_min, step_size_max; /* Rprop: step_sizes */
    double eta, mu, lambd;      /* ASGD: fp32 eta / mu states before this step, lambd; state1 = ax */
    /* v8: which sqrt every sqrt of the step computes -- FEDAVG_SQRT_IEEE (correctly rounded), FEDAVG_SQRT_TORCH_AVX512
     * (torch CPU's on Intel AVX-512 hosts: MKL vsSqrt, one Newton step from the VRSQRT14PS estimate) or
     * FEDAVG_SQRT_TORCH_AMD (torch CPU's on AMD EPYC hosts: MKL's SSE4.2 / AVX kernel, a Newton step from that CPU's
     * RSQRTPS estimate); both restated exactly, see nvflare_amd/torch_sqrt.py.  Other values: error. */
    int torch_sqrt;
} fedavg_epilogue;

/* Quantized payload formats (nvflare/app_opt/pt/quantization/dequantizer.py:47-185, row f4). */
enum fedavg_qtype {
    FEDAVG_Q_F16 = 1,        /* "float16": fp16 values                                   */
    FEDAVG_Q_BF16 = 2,       /* bf16 values                                              */
    FEDAVG_Q_BLOCKWISE8 = 3, /* "blockwise8": uint8 codes, fp32 code[256], fp32 absmax   */
    FEDAVG_Q_FP4 = 4,        /* "float4": packed nibbles (high first), fp32 absmax       */
    FEDAVG_Q_NF4 = 5,        /* "normfloat4": packed nibbles (high first), fp32 absmax   */
    FEDAVG_Q_ADA_U8 = 6,     /* "adaquant": uint8 levels, fp64 norm / level / offset     */
    FEDAVG_Q_ADA_U16 = 7,    /* "adaquant": uint16 levels                                */
};

typedef struct fedavg_quant {
    int qtype;          /* enum fedavg_qtype */
    int has_norm;       /* adaquant: 0 = all-constant tensor (value -offset) */
    size_t blocksize;   /* blockwise8 / fp4 / nf4: elements per absmax entry (multiple of 4) */
    const float* absmax; /* device pointer */
    const float* code;   /* device pointer, blockwise8 only (256 entries) */
    double norm, level, offset; /* adaquant */
} fedavg_quant;

typedef struct fedavg_ctx fedavg_ctx;

/* Last error message of the calling thread ("" if none). */
const char* fedavg_last_error(void);
int fedavg_abi_version(void);
/* sizeof the ABI's structs as this library was compiled: which = 0 struct fedavg_epilogue,
 * 1 struct fedavg_quant; 0 for any other value. */
size_t fedavg_struct_size(int which);
int fedavg_device_count(int* n);

/* Handle bound to one HIP device: owns a compute stream, a copy stream, timing events and a pinned
 * staging ring for pageable host buffers. */
int fedavg_create(int device, fedavg_ctx** out);
int fedavg_destroy(fedavg_ctx* ctx);
int fedavg_device_info(fedavg_ctx* ctx, int* num_cus, size_t* free_bytes, size_t* total_bytes);

/* Run compute work on an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the handle's own stream. */
int fedavg_set_stream(fedavg_ctx* ctx, void* stream);
int fedavg_get_stream(fedavg_ctx* ctx, void** stream);

/* Device memory owned by the caller through this handle. */
int fedavg_malloc(fedavg_ctx* ctx, size_t nbytes, void** dptr);
int fedavg_free(fedavg_ctx* ctx, void* dptr);

/* Stage client bytes into device memory (replaces the host-side arrays that
 * weighted_aggregation_helper.py:170-216 reads).  Pageable sources are copied through the pinned
 * ring with the DMA overlapped; on return the caller may reuse `src` (the aggregator must not alias
 * caller arrays, weighted_aggregation_helper.py:181-199).  Later compute on the handle is ordered
 * after the copy. */
int fedavg_h2d(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes);
/* The same into TILED client storage: logical byte b (b >= logical_offset) of one client's flat row is
 * written to base + (b / tile_bytes) * tile_stride_bytes + b % tile_bytes (see fedavg_accumulate_tiled). */
int fedavg_h2d_tiled(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes,
                     size_t logical_offset, const void* src, size_t nbytes);
/* Several host pieces of one client at once (its keys: sorted, non-overlapping logical byte offsets),
 * packed into the pinned ring by logical position so each 64 MiB leaves in one tiled DMA. */
int fedavg_h2d_tiled_multi(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes,
                           int n_pieces, const size_t* logical_offsets, const void* const* srcs,
                           const size_t* nbytes);
/* Device-resident source (e.g. a torch tensor on the GPU) into tiled client storage, on the compute stream. */
int fedavg_d2d_tiled(fedavg_ctx* ctx, void* base, size_t tile_bytes, size_t tile_stride_bytes,
                     size_t logical_offset, const void* src, size_t nbytes);
/* Device -> host; returns when the bytes are in `dst` (waits for prior compute on the handle).  Large
 * pageable destinations are drained through the pinned ring by the host copy threads. */
int fedavg_d2h(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes);
/* n device -> host copies in one call: piece i is nbytes[i] bytes from dev_base + dev_offsets[i] to
 * host_base + host_offsets[i], after the work queued on the context so far; returns when the host holds them.
 * A page-locked host_base (fedavg_host_register) takes one DMA per piece and one synchronisation.  Serves
 * the sharded server optimizer's egress (every parameter's bucket on this device into the host weights). */
int fedavg_d2h_multi(fedavg_ctx* ctx, void* host_base, const void* dev_base, int n, const size_t* host_offsets,
                     const size_t* dev_offsets, const size_t* nbytes);
/* Page-lock caller-owned host memory for direct DMA (hipHostRegister, portable across devices): copies to
 * and from it skip the pinned ring.  The caller unregisters it before the memory is freed. */
int fedavg_host_register(fedavg_ctx* ctx, void* p, size_t nbytes);
int fedavg_host_unregister(fedavg_ctx* ctx, void* p);
/* Pipelined egress: fedavg_mark records, on the compute stream, that bytes [0, ready_bytes) of the next
 * fedavg_d2h_marked source are final once the work enqueued so far has run (marks in non-decreasing order);
 * fedavg_d2h_marked then copies each 64 MiB chunk as soon as its covering mark has fired, so the D2H of the
 * aggregated model overlaps the launches still producing the rest (get_result, weighted_aggregation_helper.py:
 * 226-240, on a large model).  Returns when dst holds every byte; consumes the marks. */
int fedavg_mark(fedavg_ctx* ctx, size_t ready_bytes);
/* Drop marks recorded for a copy that will not happen (a producer starts a new marked sequence with it). */
int fedavg_marks_reset(fedavg_ctx* ctx);
int fedavg_d2h_marked(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes);
int fedavg_d2d(fedavg_ctx* ctx, void* dst, const void* src, size_t nbytes);
int fedavg_memset(fedavg_ctx* ctx, void* dst, int value, size_t nbytes);
int fedavg_sync(fedavg_ctx* ctx);

/* THE HOT PATH, contiguous client rows.  For every element i < n, in arrival order k = 0..k_rows-1:
 *   acc = acc_in ? acc_in[i] : first(rows[0][i])      (first row consumed when acc_in == NULL)
 *   acc = step(acc, rows[k][i], acc_t(weights[k]))
 *   out[i] = fin(acc)
 * rows: host array of k_rows DEVICE pointers, each to n elements of in_dtype.
 * weights: host array of k_rows fp64 weights; rounded to acc_dtype as the reference does.
 * count: fp64 arrival-order sum of weights (weighted_aggregation_helper.py:201,216), used by fin.
 * acc_in may equal out (in-place continuation).  Any k_rows >= 0 (k_rows == 0 needs acc_in).
 * Supported (in_dtype, acc_dtype): (F32,F32) streaming fast path (16-byte aligned pointers; whole tiles
 * of fedavg_set_tile elements, the ragged tail and unaligned rows take a scalar kernel); (F64,F64);
 * (F32|F16,F64); (F16,F32); (I32|I64, F32|F64); (U8|I8|I16|BOOL, F32|F64); (U16|U32|U64, F64).
 * 16-bit accumulators, (F16,F16) and (BF16,BF16), run the reference's reduced-precision sequence in fp32
 * registers with a rounding to the 16-bit format after every reference operation:
 *   NUMPY (float16 arrays, NEP 50: w -> half(w) from fp64):  first h(v*w)   step h(T + h(v*w))   SCALE h(T*half(1/count))
 *   TORCH (CPU vectorised path: mul/div in fp32 with the scalar as float, add_ alpha rounded to the format):
 *                                   first r(v*float(w))   step r(fma(v, r(w), T))   DIV r(T/float(count))
 *   UNWEIGHTED                      first v               step r(T + v)
 * (weighted_aggregation_helper.py:181-236 with float16 / bfloat16 values).
 * Integer / bool accumulators, (X,X) for X in I8, I16, I32, I64, U8, U16, U32, U64, BOOL, with
 * FEDAVG_OP_UNWEIGHTED and FEDAVG_FIN_NONE only: numpy's integer sum of weigh_by_local_iter=False arrays
 * (:195-199, :214-215) -- two's-complement wraparound in the array's dtype, logical OR for BOOL; weights and
 * count unused.  The caller finalises it as numpy does (:236) with a (X, F64) call: one row (the sum), weight
 * 1.0 / count, FEDAVG_OP_NUMPY, FEDAVG_FIN_NONE, which computes float64(T) * (1.0 / count). */
int fedavg_accumulate(fedavg_ctx* ctx, const void* const* rows, const double* weights, int k_rows,
                      const void* acc_in, void* out, size_t n, int in_dtype, int acc_dtype, int op,
                      int fin, double count);

/* THE HOT PATH, tiled client storage (fp32; the engine's slab layout).  Element i of client k lives at
 *   bases[k] + (i / tile_elems) * tile_stride + i % tile_elems          (in elements)
 * so a slab of S clients with tile_stride = S * tile_elems keeps one tile's S client segments contiguous
 * in HBM.  Computes out[i] for begin <= i < end with the same per-element sequence as fedavg_accumulate;
 * out and acc_in are flat arrays indexed by i.  Every client's storage must cover the whole tiles that
 * [begin, end) touches.  tile_elems 4096 (A/B builds: 1024, 2048, 4096, 8192); tile_stride, begin, end multiples of 4;
 * pointers 16-byte aligned; any k_rows (more than 128 are chained through out). */
int fedavg_accumulate_tiled(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                            size_t tile_elems, size_t tile_stride, size_t begin, size_t end,
                            const void* acc_in, void* out, int op, int fin, double count);

/* fedavg_accumulate_tiled for float16 / bfloat16 client storage and totals (fmt = FEDAVG_F16 | FEDAVG_BF16), with
 * the reduced-precision operation sequence documented at fedavg_accumulate.  tile_elems must be 4096 (8 KiB
 * segments); tile_stride, begin, end multiples of 8 elements; pointers 16-byte aligned; out / acc_in flat
 * 16-bit arrays indexed by i; any k_rows (more than 128 are chained through out). */
int fedavg_accumulate_tiled16(fedavg_ctx* ctx, int fmt, const void* const* bases, const double* weights, int k_rows,
                              size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                              void* out, int op, int fin, double count);

/* fedavg_accumulate_tiled16 with torch's scalar remainder.  torch CPU runs T.add_(v, alpha=w) on float16 /
 * bfloat16 tensors (weighted_aggregation_helper.py:207) over the element ranges at::parallel_for gives its
 * threads, each through a vectorised loop (the TORCH step above, one fp32 fma) and, for the last
 * (range length mod 32) elements of the range, a scalar loop whose c10::Half / c10::BFloat16 operators round
 * twice: step p = r(v * r(w)), T = r(T + p).  tails: n_tails strictly increasing flat element indices (host
 * memory) that take that step; those outside [begin, end) are ignored, as are all of them for an op other
 * than FEDAVG_OP_TORCH -- except FEDAVG_OP_TORCH_DEVICE on float16, where the listed elements take torch-ROCm's
 * unrolled step instead, T = fp16(exact fma(v, float(w), T)).  The listed elements are recomputed into a side buffer before the tile kernel (acc_in
 * may alias out) and written over its results after it: two small extra launches when any lies in the range. */
int fedavg_accumulate_tiled16_tails(fedavg_ctx* ctx, int fmt, const void* const* bases, const double* weights,
                                    int k_rows, size_t tile_elems, size_t tile_stride, size_t begin, size_t end,
                                    const void* acc_in, void* out, int op, int fin, double count,
                                    const int64_t* tails, size_t n_tails);

/* fedavg_accumulate_tiled for fp64 client storage and totals (numpy's default dtype; the engine's fp64 arena):
 * tile_elems = 4096, begin/end multiples of 2, every pointer 16-byte aligned.  fp64 arithmetic in arrival
 * order with fp64 weights -- numpy: T = T + v*w then T * (1.0/count); torch (float64 tensors): fma, T / count
 * (weighted_aggregation_helper.py:181-236). */
int fedavg_accumulate_tiled64(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                              size_t tile_elems, size_t tile_stride, size_t begin, size_t end, const void* acc_in,
                              void* out, int op, int fin, double count);

/* fedavg_accumulate_tiled with a server-optimizer epilogue applied per element to d = fin(acc) in the
 * same launch (rows a9/a10): ADD_BASE writes base + d to out; SGD/ADAM update epi->param/state in place
 * and also store d to out when out != NULL.  Product libraries fuse the (op, fin) pairs the drop-in produces
 * (numpy * SCALE, torch * DIV | SCALE, unweighted * SCALE | DIV) for 1-128 clients, and the server step alone (k_rows
 * == 0, acc_in = the aggregate, FEDAVG_FIN_NONE); any other call -- more than 128 clients, a chained acc_in with
 * clients, numpy * DIV, FIN_NONE with clients -- runs the plain aggregation into a stream-ordered scratch and then that
 * server step on it, the same per-element sequence.  (A/B libraries fuse every case: more than 128 clients chained
 * through a partial sum kept in out, or in a scratch when out is NULL or aliases an epilogue operand.) */
int fedavg_accumulate_tiled_epi(fedavg_ctx* ctx, const void* const* bases, const double* weights, int k_rows,
                                size_t tile_elems, size_t tile_stride, size_t begin, size_t end,
                                const void* acc_in, void* out, int op, int fin, double count,
                                const fedavg_epilogue* epi);

/* Dequantize n elements of a device-resident payload q into fp32, written at logical element offset
 * logical_offset of a tiled buffer (tile_elems, tile_stride; 0, 0 = flat).  The aggregation slab layout,
 * so a quantized contribution is dequantized straight into its client slot.  Replaces the per-format
 * branches of ModelDequantizer.dequantization (dequantizer.py:98-160) + the fp32 cast (:168-173).
 * logical_offset and tile_elems multiples of 4; the 16-byte-aligned out must cover the written range. */
int fedavg_dequantize(fedavg_ctx* ctx, const fedavg_quant* qs, const void* q, size_t n, float* out_base,
                      size_t tile_elems, size_t tile_stride, size_t logical_offset);

/* Timing of the kernels launched by the last fedavg_accumulate call, measured with HIP events on
 * the stream they ran on (enable first; costs two event records per call). */
int fedavg_set_timing(fedavg_ctx* ctx, int enable);
int fedavg_last_kernel_ms(fedavg_ctx* ctx, float* ms);

/* Event bracket over a region of compute-stream work (e.g. K back-to-back fedavg_accumulate calls):
 * begin records a start event, end records a stop event, waits for it and returns the elapsed ms. */
int fedavg_timing_begin(fedavg_ctx* ctx);
int fedavg_timing_end(fedavg_ctx* ctx, float* ms);

/* Aggregation / epilogue / dequantization kernel launches issued on the context's compute stream so far.
 * One fedavg_accumulate* call may issue several (the fp32 burst kernels: one per grid x tiles-per-block tiles --
 * 18 tiles per block on the one-block-per-CU grids of the plain kernel at 32+ clients (17 for the fused kernel at
 * 64+), 12 on two-block grids; the fused LDS-DMA form at 1-3 reads 4-10 tiles per block, one block per CU); relates a
 * profiler's per-launch durations to per-call times. */
int fedavg_launch_count(fedavg_ctx* ctx, uint64_t* n);
/* Launch tuning (0 = default): blocks per CU (default: each kernel's own -- 1 for the burst aggregation
 * kernel at >= 32 clients, the fused one at >= 64, the 16-bit one at >= 48 in torch mode, 2 otherwise),
 * clients whose loads are issued together (4; 8 in A/B builds only -- see below). */
int fedavg_set_launch(fedavg_ctx* ctx, int blocks_per_cu, int unroll);
/* Kernel variants (default 0).  By default a plain launch with 3 or more row reads (fused: 4 or more -- its clients,
 * plus the chained partial sum of a launch after the first 128 clients) runs the BURST form: each block holds its
 * tiles' results (the fused kernel: its differences) in registers and LDS and stores them (runs the epilogue) as
 * chip-wide bursts at the end of a short launch -- per launch 8 register-held tiles per block plus 4 LDS-held ones on
 * two-block-per-CU grids, or 10 (fused: 9) on the one-block-per-CU grids of the plain kernel at 32+ clients (fused:
 * 64+).  A plain launch with 1-3 client reads and no chained sum (most NVFlare jobs run 2 clients) runs the FEW-CLIENT
 * burst form (round 5): every register-held tile's loads go out before any arithmetic, the results are stored as a
 * burst; a chained sum with fewer than 3 reads runs the PER-TILE-STORE form, which stores each tile's results as it
 * finishes.  The fused kernel with 1-3 client reads, no chained sum and no separate aggregate output (out only for
 * ADD_BASE) runs its LDS-DMA few-client form (round 6) for every kind (Adam with amsgrad at 3 reads only, RMSprop
 * centered only with momentum): every input goes HBM -> LDS by LDS-DMA while the wave computes the units already
 * landed, the results are held on chip and stored as a burst; the rest and chained sums under 4 reads run its per-tile
 * form pipelined across tiles.  Every load
 * and store is
 * nontemporal.  The 16-bit and fp64 tile kernels (fedavg_accumulate_tiled16 / _tiled64) likewise run 1-3 client
 * reads without a chained sum on their few-client burst forms, the rest on their burst forms.  The plain burst kernel has the launch's client count
 * built in for 5 clients and the count's
 * remainder mod 4 otherwise (no repeated loads); each full four-client group's loads go out as two pairs (plain burst
 * kernel from 4 clients on, fused from 8).  Results are bit-identical in every variant.
 * The PRODUCT library (nvflare_amd/_build.py) carries only the routed kernel forms and accepts:
 * bit 2 = the fused per-tile form (pipelined across tiles: the next tile's first client loads overlap the epilogue) at
 *         every read count (the round-5 route at 1-3 reads, instead of the LDS-DMA form);
 * bit 4 = burst launches after the first of a call go out without the AQL barrier bit (hipExtAnyOrderLaunch), so
 *         one launch's blocks start as the previous launch drains;
 * bit 6 = one-block-per-CU grids keep the 4-LDS-tile form (12 tiles per block per launch).
 * A/B libraries (tools/build_rev_lib.py, -DFEDAVG_AB) also carry, and accept:
 * bit 0 / bit 1 = the per-tile-store plain kernel with temporal client loads / temporal result stores (imply bit 3);
 * bit 3 = every launch on the per-tile-store form (fused: unpipelined);
 * bit 5 = the burst kernels without their LDS-held tiles (register-held tiles only: 8 per block per launch);
 * bit 7 = the plain burst kernel's round-3 runtime client loop (its last group of 4 re-loads the last client in the
 *         missing slots when the count is not a multiple of 4);
 * bit 8 = plain launches with fewer than 3 row reads (16-bit, fp64: 1-3) on the general burst form (also accepted by
 *         product-sized -DFEDAVG_AB_FEW builds);
 * bits 9-11 = the fused burst kernel's client loop in shape 1-6 (fedavg_epi.h launch_epi_loop_ab; built for torch-mode
 *         FIN_DIV Adam with the AMD-host sqrt and no chained partial sum), the plain burst kernel's (fedavg_tiles.h
 *         launch_burst; 6 / 7 = 3-6 clients on a built-in count / the remainder forms), the few-client form's
 *         geometry at 1-2 reads (1-6) and 3-4 reads (1-5) (fedavg_internal.h kFewAB, kFewAB34), the 16-bit
 *         and fp64 few-client forms' at 1-3 reads (1-4, kNarrowFewAB, kF64FewAB), and the fused LDS-DMA
 *         form's geometry at 1-3 reads (1-7: waves per block, units per wave, the RSQRTPS table's staging; fedavg_epi.h
 *         launch_epi_dma_form; torch-mode FIN_DIV ADD_BASE / SGD / Adam with the AMD-host sqrt, -DFEDAVG_AB_FEW builds);
 * and unroll 8 (fedavg_set_launch) and tile widths 1024 / 2048 / 8192 (fedavg_set_tile, fedavg_accumulate_tiled).
 * A product library refuses those with an error ("... A/B form ..."), never running another form in their place. */
int fedavg_set_variant(fedavg_ctx* ctx, int variant);
/* Tile width used by fedavg_accumulate for contiguous rows (default 4096 elements; other widths in A/B builds). */
int fedavg_set_tile(fedavg_ctx* ctx, int tile_elems);

/* Synthetic inputs for benchmarks/tests: logical element j of a client row (tiled like
 * fedavg_accumulate_tiled; tile_elems == 0 means contiguous) = synth(seed, row, col0 + j), fp32,
 * bit-identical to the host twin oracle_synth_value() in oracle/fedavg_oracle.c. */
int fedavg_fill_synthetic_f32(fedavg_ctx* ctx, float* dst, size_t n, size_t tile_elems, size_t tile_stride,
                              uint64_t seed, uint64_t row, uint64_t col0);
/* Gather m fp32 elements src[idx[j]] (idx: host array) into host_out (spot checks at full size). */
int fedavg_gather_f32(fedavg_ctx* ctx, const float* src, const uint64_t* idx, size_t m, float* host_out);
/* Test entry (v8): out[i] = the epilogues' sqrt of x[i] on the compute stream (device pointers); torch_sqrt is a
 * FEDAVG_SQRT_* value as in struct fedavg_epilogue. */
int fedavg_sqrt_f32(fedavg_ctx* ctx, const float* x, float* out, size_t n, int torch_sqrt);

/* v9 -- torch CPU's sqrt on hosts where MKL runs vsSqrt's SSE4.2 / AVX kernel (FEDAVG_SQRT_TORCH_AMD) starts from the
 * CPU's RSQRTPS estimate, which is vendor-specific.  fedavg_host_rsqrtps_table (host only, no device needed) captures
 * THIS CPU's estimates: table[parity * 4096 + (m >> 11)] = mantissa bits 22..11 of RSQRTPS(x) for x = 2^parity * 1.m
 * (n must be 8192); it fails if the CPU's estimate is not a function of the exponent parity and the top 12 mantissa
 * bits (every fp32 of [1, 4) is checked).  fedavg_set_rsqrtps_table uploads such a table for the handle's kernels;
 * until it is called, FEDAVG_SQRT_TORCH_AMD steps and sqrt calls fail.  (Replaces a table compiled in from one
 * host; nvflare_amd/torch_sqrt.py verifies the restatement against the host's torch.sqrt before selecting it.) */
int fedavg_host_rsqrtps_table(uint16_t* table, size_t n);
int fedavg_set_rsqrtps_table(fedavg_ctx* ctx, const uint16_t* table, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* NVFLARE_AMD_FEDAVG_H */
