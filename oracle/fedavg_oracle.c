/*
 * fedavg_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product path).
 *
 * CPU restatement of the arithmetic of NVFlare's WeightedAggregationHelper, element by element,
 * in arrival order.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (nvflare_amd/) never links or calls it.
 *
 * Reference (relative to the NVFlare tree):
 *   nvflare/app_common/aggregators/weighted_aggregation_helper.py
 *     numpy branch, first contribution   :188-193   T = v * w           (fp32 mul, w -> fl32)
 *     numpy branch, later contributions  :210-214   T = T + v * w       (fp32 mul, then fp32 add)
 *     numpy get_result                   :236       T * (1.0 / count)   (fp64 reciprocal -> fl32, mul)
 *     torch branch, first contribution   :181-187   T = v.mul(w)        (fp32 mul)
 *     torch branch, later contributions  :203-209   T.add_(v, alpha=w)  (one fused multiply-add)
 *     torch get_result                   :233       T.div_(count)       (correctly rounded fp32 division)
 *     weigh_by_local_iter=False          :186-199,208-215  T = copy(v); T = T + v
 *
 * The fp32 weight is the fp64 host weight rounded to nearest (NEP-50 weak scalar for numpy; the
 * scalar operand cast of torch's TensorIterator).  This file must be compiled with
 * -ffp-contract=off so that the numpy mode's multiply and add round separately; the torch mode
 * uses C99 fmaf()/fma(), which round once.
 *
 * Parity pin: tests/test_oracle_golden.py checks this restatement bit-for-bit against the golden
 * vectors in tests/golden/, which were produced by running the reference helper itself
 * (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#ifdef _OPENMP
#include <omp.h>
#endif

enum { ORACLE_MODE_NUMPY = 0, ORACLE_MODE_TORCH = 1 };
enum { ORACLE_FIN_NONE = 0, ORACLE_FIN_NUMPY_SCALE = 1, ORACLE_FIN_TORCH_DIV = 2 };

int oracle_abi_version(void) { return 1; }

/* Core loop for one accumulator type.  rows[k] points at client k's (already converted) values
 * in arrival order.  acc_in == NULL means the first row starts the running sum. */
#define DEFINE_ORACLE(NAME, T, FMA)                                                              \
    void NAME(const T* const* rows, int K, const double* weights, int mode, int weighted,       \
              int fin, double count, const T* acc_in, T* out, size_t n, int nthreads) {         \
        T w[4096];                                                                               \
        int kk;                                                                                  \
        if (K > 4096) K = 4096;                                                                  \
        for (kk = 0; kk < K; ++kk) w[kk] = (T)weights[kk];                                       \
        const T scale = (T)(1.0 / count); /* numpy: python float 1.0/count, then cast */          \
        const T cnt = (T)count;           /* torch: scalar operand cast to fp32/fp64 */           \
        (void)nthreads;                                                                          \
        long long i;                                                                             \
        _Pragma("omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)")    \
        for (i = 0; i < (long long)n; ++i) {                                                     \
            T acc;                                                                               \
            int k0;                                                                              \
            if (acc_in) {                                                                        \
                acc = acc_in[i];                                                                 \
                k0 = 0;                                                                          \
            } else {                                                                             \
                acc = weighted ? rows[0][i] * w[0] : rows[0][i];                                 \
                k0 = 1;                                                                          \
            }                                                                                    \
            for (int k = k0; k < K; ++k) {                                                       \
                const T v = rows[k][i];                                                          \
                if (!weighted) {                                                                 \
                    acc = acc + v;                                                               \
                } else if (mode == ORACLE_MODE_TORCH) {                                          \
                    acc = FMA(v, w[k], acc);                                                     \
                } else {                                                                         \
                    const T p = v * w[k];                                                        \
                    acc = acc + p;                                                               \
                }                                                                                \
            }                                                                                    \
            if (fin == ORACLE_FIN_NUMPY_SCALE) acc = acc * scale;                                \
            else if (fin == ORACLE_FIN_TORCH_DIV) acc = acc / cnt;                               \
            out[i] = acc;                                                                        \
        }                                                                                        \
    }

DEFINE_ORACLE(oracle_fedavg_f32, float, fmaf)
DEFINE_ORACLE(oracle_fedavg_f64, double, fma)

/* Synthetic-input generator shared with the device generator in nvflare_amd/csrc/fedavg_kernels.hip
 * (kernel fedavg_fill_synthetic_f32).  Integer-only hashing plus one exact int->float conversion and
 * one IEEE multiply, so host and device produce identical bits.  Irwin-Hall(4) of 24-bit uniforms,
 * scaled to unit variance: approximately N(0,1). */
static inline uint32_t oracle_mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

float oracle_synth_value(uint64_t seed, uint64_t row, uint64_t col) {
    const uint64_t base = (seed * 0x9E3779B97F4A7C15ULL) ^ (row * 0xD1B54A32D192ED03ULL);
    int32_t s = 0;
    for (int j = 0; j < 4; ++j) {
        s += (int32_t)(oracle_mix32(base + col * 4ULL + (uint64_t)j) >> 8);
    }
    s -= (int32_t)(1 << 25); /* centre: sum of 4 values in [0, 2^24) */
    /* variance of one U[0,2^24) = 2^48/12, four of them: 2^48/3 -> sd = 2^24/sqrt(3) */
    return (float)s * 1.0323827e-07f; /* sqrt(3) / 2^24, rounded to fp32 */
}

void oracle_synth_fill_f32(uint64_t seed, uint64_t row, const uint64_t* cols, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_synth_value(seed, row, cols[i]);
}

/* ------------------------------------------------------------------------------------------------
 * Server-optimizer epilogues, applied to the aggregated update
 * d = fin(acc) of each element (computed exactly as above):
 *   ADD_BASE  w = base + d            full_model_shareable_generator.py:58-67 (WEIGHT_DIFF apply)
 *   SGD       torch/optim/sgd.py _single_tensor_sgd on grad g = -1.0 * d   (app_opt/pt/fedopt.py:175)
 *   ADAM      torch/optim/adam.py _single_tensor_adam (:347-551) on g = -1.0 * d
 * Rounding sequence pinned against torch 2.10 CPU (tests/test_fedopt_oracle.py):
 *   add(alpha)  fma(b, alpha, a);   lerp  |w| < .5 ? fma(w, e - s, s) : fma(w - 1, e - s, e)
 *   addcmul     fma(val * t1, t2, self);   addcdiv  self + (val * t1) / t2
 *   sqrt        IEEE (correctly rounded).  torch CPU's MKL sqrt is not: ~0.6 % of its results are 1 ulp
 *               off, so Adam params are compared within 1 ulp, m and v bit-exactly.
 * Scalars follow torch: python-float hyperparameters and bias corrections computed in fp64, cast to
 * fp32 where they meet a tensor.
 * ------------------------------------------------------------------------------------------------ */
enum { ORACLE_EPI_NONE = 0, ORACLE_EPI_ADD_BASE = 1, ORACLE_EPI_SGD = 2, ORACLE_EPI_ADAM = 3 };

typedef struct {
    int kind;
    int first_step;  /* SGD: momentum buffer starts as a clone of the gradient */
    int nesterov;
    int maximize;
    int decoupled_weight_decay; /* AdamW */
    double lr, momentum, dampening, weight_decay; /* SGD (+ lr, weight_decay for Adam) */
    double beta1, beta2, eps, step;               /* Adam: step after increment (1, 2, ...) */
} oracle_epilogue;

static inline float lerp_torch(float s, float e, float w) {
    const float d = e - s;
    return fabsf(w) < 0.5f ? fmaf(w, d, s) : fmaf(w - 1.0f, d, e);
}

void oracle_epilogue_apply(const float* delta, size_t n, const oracle_epilogue* epi, float* p, float* m, float* v,
                           const float* base, float* out) {
    for (size_t i = 0; i < n; ++i) {
        const float d = delta[i];
        if (epi->kind == ORACLE_EPI_NONE) {
            out[i] = d;
        } else if (epi->kind == ORACLE_EPI_ADD_BASE) {
            out[i] = base[i] + d;
        } else if (epi->kind == ORACLE_EPI_SGD) {
            float g = epi->maximize ? d : -d;
            if (epi->weight_decay != 0.0) g = fmaf(p[i], (float)epi->weight_decay, g);
            if (epi->momentum != 0.0) {
                float b;
                if (epi->first_step) b = g;
                else b = fmaf(g, (float)(1.0 - epi->dampening), m[i] * (float)epi->momentum);
                m[i] = b;
                g = epi->nesterov ? fmaf(b, (float)epi->momentum, g) : b;
            }
            p[i] = fmaf(g, (float)(-epi->lr), p[i]);
        } else { /* ADAM */
            float g = epi->maximize ? d : -d;
            float pv = p[i];
            if (epi->weight_decay != 0.0) {
                if (epi->decoupled_weight_decay) pv = pv * (float)(1.0 - epi->lr * epi->weight_decay);
                else g = fmaf(pv, (float)epi->weight_decay, g);
            }
            const float mm = lerp_torch(m[i], g, (float)(1.0 - epi->beta1));
            const float vv = fmaf((float)(1.0 - epi->beta2) * g, g, v[i] * (float)epi->beta2);
            const double bc1 = 1.0 - pow(epi->beta1, epi->step);
            const double bc2 = 1.0 - pow(epi->beta2, epi->step);
            const float step_size_neg = (float)(-(epi->lr / bc1));
            const float bc2s = (float)pow(bc2, 0.5); /* python: bias_correction2**0.5 */
            const float denom = sqrtf(vv) / bc2s + (float)epi->eps;
            pv = pv + (step_size_neg * mm) / denom;
            m[i] = mm;
            v[i] = vv;
            p[i] = pv;
        }
    }
}
