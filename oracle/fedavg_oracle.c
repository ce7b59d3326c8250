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
#include <immintrin.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

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
 *   ADAGRAD   torch/optim/adagrad.py _single_tensor_adagrad on g = -1.0 * d (m holds state_sum)
 *   RMSPROP   torch/optim/rmsprop.py _single_tensor_rmsprop (m square_avg, v momentum_buffer, vmax grad_avg)
 *   ADAMAX    torch/optim/adamax.py _single_tensor_adamax on g = -1.0 * d (m exp_avg, v exp_inf)
 *   NADAM     torch/optim/nadam.py _single_tensor_nadam (m exp_avg, v exp_avg_sq; mu_product passed in)
 *   RADAM     torch/optim/radam.py _single_tensor_radam (m exp_avg, v exp_avg_sq)
 *   RPROP     torch/optim/rprop.py _single_tensor_rprop (m prev, v step_size filled with lr before step 1)
 *   ASGD      torch/optim/asgd.py _single_tensor_asgd (m ax; eta and mu passed in)
 *   ADAM      torch/optim/adam.py _single_tensor_adam (:347-551) on g = -1.0 * d; amsgrad divides by
 *             sqrt(vmax), vmax = torch.maximum(vmax, v) kept as a third state
 * Rounding sequence pinned against torch 2.10 CPU (tests/test_fedopt_oracle.py):
 *   add(alpha)  fma(b, alpha, a);   lerp  |w| < .5 ? fma(w, e - s, s) : fma(w - 1, e - s, e)
 *   addcmul     fma(val * t1, t2, self);   addcdiv  self + (val * t1) / t2
 *   sqrt        IEEE (correctly rounded) when sqrt_table is NULL and sqrt_sse2 is 0; with the table, torch CPU's
 *               own sqrt: MKL VML vsSqrt on the AVX-512 path (ATen vml.h IMPLEMENT_VML_MKL(sqrt, Sqrt)), which
 *               is one Newton step from the VRSQRT14PS estimate, restated in oracle_sqrt_torch_cpu below
 *               (~0.5 % of its results are 1 ulp below the correctly rounded value; tools/sqrt_probe.c);
 *               with rsqrtps_table, MKL's SSE4.2 / AVX path (AMD hosts), oracle_sqrt_mkl_rsqrtps.
 * Scalars follow torch: python-float hyperparameters and bias corrections computed in fp64, cast to
 * fp32 where they meet a tensor.
 * ------------------------------------------------------------------------------------------------ */
enum { ORACLE_EPI_NONE = 0, ORACLE_EPI_ADD_BASE = 1, ORACLE_EPI_SGD = 2, ORACLE_EPI_ADAM = 3, ORACLE_EPI_ADAGRAD = 4,
       ORACLE_EPI_RMSPROP = 5, ORACLE_EPI_ADAMAX = 6, ORACLE_EPI_NADAM = 7, ORACLE_EPI_RADAM = 8,
       ORACLE_EPI_RPROP = 9, ORACLE_EPI_ASGD = 10 };

typedef struct {
    int kind;
    int first_step;  /* SGD: momentum buffer starts as a clone of the gradient */
    int nesterov;
    int maximize;
    int decoupled_weight_decay; /* AdamW */
    double lr, momentum, dampening, weight_decay; /* SGD (+ lr, weight_decay for Adam) */
    double beta1, beta2, eps, step;               /* Adam: step after increment (1, 2, ...) */
    int amsgrad;                                  /* Adam: normalise by the running max of v (vmax) */
    double lr_decay;                              /* Adagrad: clr = lr / (1 + (step - 1) * lr_decay) */
    double alpha;                                 /* RMSprop smoothing constant */
    int centered;                                 /* RMSprop: vmax holds grad_avg */
    double momentum_decay;                        /* NAdam */
    double mu_product;                            /* NAdam: fp32 mu_product state before this step */
    double etaminus, etaplus, step_size_min, step_size_max; /* Rprop */
    double eta, mu, lambd;                        /* ASGD: fp32 eta / mu states before this step */
    const uint16_t* sqrt_table;                   /* NULL: IEEE sqrt; else the VRSQRT14 mantissa table */
    const uint16_t* rsqrtps_table;                /* non-NULL: MKL's SSE4.2 / AVX vsSqrt (oracle_sqrt_mkl_rsqrtps) */
} oracle_epilogue;

/* torch CPU's fp32 Tensor.sqrt, restated (torch 2.10 + MKL 2024.2 on AVX-512; measured bit-exact against torch
 * over every fp32 mantissa of [1, 4), every subnormal and 1 in 61 of every other binade -- tools/sqrt_probe.py):
 *   y = rsqrt14(x); s = x * y; r = fma(-s, s, x); sqrt = fma(r, 0.5 * y, s)
 * rsqrt14 (VRSQRT14PS) depends on the exponent parity and the top 15 mantissa bits only: tab[parity << 15 | m >> 8]
 * holds mantissa bits 22..7 of its result for x in [1, 4) (exponent 126 throughout), a power of four giving its
 * exact reciprocal root.  Inputs below 2^-96 are computed at x * 2^64 and scaled back by 2^-32 (vsSqrt keeps the
 * Newton residual out of the subnormal range; every scale from 2^32 to 2^200 gives the same bits).  Zero, inf,
 * NaN and negative inputs take the IEEE results. */
float oracle_sqrt_torch_cpu(const uint16_t* tab, float x) {
    if (!(x > 0.0f) || isinf(x)) return sqrtf(x);
    const int tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p64f : x;
    uint32_t b;
    memcpy(&b, &xs, 4);
    const int e = (int)(b >> 23) - 127;
    const uint32_t m = b & 0x7FFFFFu;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint32_t yb = (p == 0 && m == 0) ? 0x3F800000u : (0x3F000000u | ((uint32_t)tab[(p << 15) | (m >> 8)] << 7));
    const uint32_t yk = (uint32_t)((int32_t)yb - k * 8388608);
    float y;
    memcpy(&y, &yk, 4);
    const float s = xs * y;
    const float r = fmaf(-s, s, xs);
    const float res = fmaf(r, 0.5f * y, s);
    return tiny ? res * 0x1p-32f : res;
}

void oracle_sqrt_torch_cpu_n(const uint16_t* tab, const float* x, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_sqrt_torch_cpu(tab, x[i]);
}

/* MKL vsSqrt's SSE2 kernel (mkl_vml_kernel_sSqrt_E2HAynn): not what torch runs on the hosts seen so far, but the
 * plain-fp32 refinement it shares with the SSE4.2 / AVX kernels below, pinned exhaustively on any x86-64 host because
 * its estimate uses only IEEE operations.  It refines the correctly rounded sqrtps result with a coupled Newton step
 * (SSE2: every operation rounds, no FMA), starting from a reciprocal truncated to 12 significant bits:
 *   s0 = sqrt(x);  y = trunc12(1 / s0);  s = x * y;  h = y * 0.5;  r = 0.5 - s * h;
 *   s1 = s * r + s;  h1 = h * r + h;  sqrt = (x - s1 * s1) * h1 + s1
 * for positive normal x up to 0x7f7ff000; everything else (zero, subnormals, the top 4095 finite values, inf, NaN,
 * negatives) takes the kernel's scalar callout, which returns the correctly rounded sqrt.  Checked equal to the MKL
 * kernel itself (called from libtorch_cpu) on all 2^32 inputs, NaN payloads aside -- tools/sqrt_mkl_sse2_check.py. */
float oracle_sqrt_mkl_sse2(float x) {
    uint32_t b;
    memcpy(&b, &x, 4);
    if (b < 0x00800000u || b > 0x7F7FF000u) return sqrtf(x);
    const float s0 = sqrtf(x);
    float y = 1.0f / s0;
    uint32_t yb;
    memcpy(&yb, &y, 4);
    yb &= 0xFFFFF800u;
    memcpy(&y, &yb, 4);
    const float s = x * y;
    const float h = y * 0.5f;
    const float t = s * h;
    const float r = 0.5f - t;
    const float sr = s * r, hr = h * r;
    const float s1 = sr + s;
    const float h1 = hr + h;
    const float q = s1 * s1;
    const float d = x - q;
    const float dh = d * h1;
    return dh + s1;
}

void oracle_sqrt_mkl_sse2_n(const float* x, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_sqrt_mkl_sse2(x[i]);
}

/* torch CPU's fp32 Tensor.sqrt on the GPU pool's AMD EPYC hosts: there MKL runs vsSqrt's SSE4.2 / AVX kernels
 * (mkl_vml_kernel_sSqrt_EXHAynn / _H8HAynn, identical results), which start the same coupled Newton step as the SSE2
 * kernel above from the RSQRTPS estimate instead:
 *   y = rsqrtps(x);  s = x * y;  h = y * 0.5;  r = 0.5 - s * h;  s1 = s * r + s;  h1 = h * r + h;
 *   sqrt = (x - s1 * s1) * h1 + s1
 * (positive normals up to 0x7f7ff000; everything else the correctly rounded callout).  RSQRTPS differs between CPU
 * vendors; it depends on the exponent parity and the top 12 mantissa bits only, so tab[parity << 12 | m >> 11] holds
 * mantissa bits 22..11 of its result for x in [1, 4) (exponent 126 throughout; tools/rsqrtps_dump.c captures it) and
 * y = that estimate * 2^-k for x = 4^k * x0.  With this CPU's table the sequence equals MKL's EX kernel on all 2^32
 * inputs (tools/sqrt_mkl_sse2_check.py); with the AMD host's table, that host's torch.sqrt (tools/sqrt_box_kernels.py). */
float oracle_sqrt_mkl_rsqrtps(const uint16_t* tab, float x) {
    uint32_t b;
    memcpy(&b, &x, 4);
    if (b < 0x00800000u || b > 0x7F7FF000u) return sqrtf(x);
    const int e = (int)(b >> 23) - 127;
    const int p = e & 1;
    const int k = (e - p) / 2;
    const uint32_t yb = (0x3F000000u | ((uint32_t)tab[(p << 12) | ((b & 0x7FFFFFu) >> 11)] << 11)) - (uint32_t)(k * 8388608);
    float y;
    memcpy(&y, &yb, 4);
    const float s = x * y;
    const float h = y * 0.5f;
    const float t = s * h;
    const float r = 0.5f - t;
    const float sr = s * r, hr = h * r;
    const float s1 = sr + s;
    const float h1 = hr + h;
    const float q = s1 * s1;
    const float d = x - q;
    const float dh = d * h1;
    return dh + s1;
}

void oracle_sqrt_mkl_rsqrtps_n(const uint16_t* tab, const float* x, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_sqrt_mkl_rsqrtps(tab, x[i]);
}

/* THIS CPU's RSQRTPS table in the layout above, from the packed instruction MKL's SSE kernel executes (RSQRTPS,
 * _mm_rsqrt_ps; ADVICE r04: the scalar RSQRTSS is another instruction) over EVERY fp32 of [1, 4), four per
 * instruction: entry i = the estimate of block i (2^11 consecutive inputs sharing the exponent parity and the top 12
 * mantissa bits).  Returns the number of blocks whose inputs do not all give one 12-bit estimate with exponent 126 (0
 * on the CPUs the restatement covers), independently of the product's own capture (fedavg_host_rsqrtps_table). */
int oracle_host_rsqrtps_table(uint16_t* tab) {
    int bad = 0;
    for (uint32_t i = 0; i < 8192; ++i) {
        uint32_t first = 0;
        int block_bad = 0;
        for (uint32_t j = 0; j < 2048; j += 4) {
            uint32_t in[4], out[4];
            for (int l = 0; l < 4; ++l) in[l] = 0x3F800000u + (i << 11) + j + (uint32_t)l;
            __m128 x;
            memcpy(&x, in, 16);
            const __m128 y = _mm_rsqrt_ps(x);
            memcpy(out, &y, 16);
            if (j == 0) first = out[0];
            for (int l = 0; l < 4; ++l) block_bad |= out[l] != first;
        }
        bad += block_bad || (first >> 23) != 126u || (first & 0x7FFu) != 0u;
        tab[i] = (uint16_t)((first >> 11) & 0xFFFu);
    }
    return bad;
}

static inline float sqrt_e(const oracle_epilogue* epi, float x) {
    if (epi->rsqrtps_table) return oracle_sqrt_mkl_rsqrtps(epi->rsqrtps_table, x);
    return epi->sqrt_table ? oracle_sqrt_torch_cpu(epi->sqrt_table, x) : sqrtf(x);
}

/* torch.maximum: a NaN operand is the result */
static inline float max_torch(float a, float b) {
    if (a != a) return a;
    if (b != b) return b;
    return a > b ? a : b;
}

static inline float lerp_torch(float s, float e, float w) {
    const float d = e - s;
    return fabsf(w) < 0.5f ? fmaf(w, d, s) : fmaf(w - 1.0f, d, e);
}

void oracle_epilogue_apply(const float* delta, size_t n, const oracle_epilogue* epi, float* p, float* m, float* v,
                           float* vmax, const float* base, float* out) {
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
        } else if (epi->kind == ORACLE_EPI_ADAGRAD) { /* torch/optim/adagrad.py _single_tensor_adagrad, m = sum */
            float g = epi->maximize ? d : -d;
            if (epi->weight_decay != 0.0) g = fmaf(p[i], (float)epi->weight_decay, g);
            const float neg_clr = (float)(-(epi->lr / (1.0 + (epi->step - 1.0) * epi->lr_decay)));
            m[i] = fmaf(g, g, m[i]);                                  /* state_sum.addcmul_(g, g, value=1) */
            const float std_ = sqrt_e(epi, m[i]) + (float)epi->eps;         /* state_sum.sqrt().add_(eps) */
            p[i] = p[i] + (neg_clr * g) / std_;                       /* param.addcdiv_(g, std, value=-clr) */
        } else if (epi->kind == ORACLE_EPI_RMSPROP) { /* torch/optim/rmsprop.py _single_tensor_rmsprop */
            /* m = square_avg, v = momentum_buffer, vmax = grad_avg */
            float g = epi->maximize ? d : -d;
            if (epi->weight_decay != 0.0) g = fmaf(p[i], (float)epi->weight_decay, g);
            const float oma = (float)(1.0 - epi->alpha);
            m[i] = fmaf(oma * g, g, m[i] * (float)epi->alpha);       /* mul_(alpha).addcmul_(g, g, 1 - alpha) */
            float avg;
            if (epi->centered) {
                vmax[i] = lerp_torch(vmax[i], g, oma);                /* grad_avg.lerp_(g, 1 - alpha) */
                avg = sqrt_e(epi, fmaf(-vmax[i], vmax[i], m[i]));          /* addcmul(ga, ga, value=-1).sqrt_() */
            } else {
                avg = sqrt_e(epi, m[i]);
            }
            avg = avg + (float)epi->eps;
            if (epi->momentum > 0.0) {
                v[i] = v[i] * (float)epi->momentum + g / avg;         /* buf.mul_(momentum).addcdiv_(g, avg) */
                p[i] = fmaf(v[i], (float)(-epi->lr), p[i]);           /* param.add_(buf, alpha=-lr) */
            } else {
                p[i] = p[i] + ((float)(-epi->lr) * g) / avg;          /* param.addcdiv_(g, avg, value=-lr) */
            }
        } else if (epi->kind == ORACLE_EPI_ADAMAX) { /* torch/optim/adamax.py _single_tensor_adamax */
            float g = epi->maximize ? d : -d;
            if (epi->weight_decay != 0.0) g = fmaf(p[i], (float)epi->weight_decay, g); /* grad.add(param, alpha=wd) */
            m[i] = lerp_torch(m[i], g, (float)(1.0 - epi->beta1));                    /* exp_avg.lerp_(g, 1 - beta1) */
            v[i] = max_torch(v[i] * (float)epi->beta2, fabsf(g) + (float)epi->eps);    /* maximum(exp_inf.mul_(b2), |g|+eps) */
            const float neg_clr = (float)(-(epi->lr / (1.0 - pow(epi->beta1, epi->step))));
            p[i] = p[i] + (neg_clr * m[i]) / v[i];                                    /* addcdiv_(exp_avg, exp_inf, -clr) */
        } else if (epi->kind == ORACLE_EPI_ASGD) { /* torch/optim/asgd.py _single_tensor_asgd, m = ax */
            float g = epi->maximize ? d : -d;
            if (epi->weight_decay != 0.0) g = fmaf(p[i], (float)epi->weight_decay, g);
            float pv = p[i] * (float)(1.0 - epi->lambd * epi->eta);       /* param.mul_(1 - lambd * eta) */
            pv = fmaf(g, (float)(-epi->eta), pv);                          /* param.add_(grad, alpha=-eta) */
            const float mu = (float)epi->mu;
            m[i] = mu != 1.0f ? m[i] + (pv - m[i]) * mu : pv;             /* ax.add_(p.sub(ax).mul_(mu)) / copy_ */
            p[i] = pv;
        } else if (epi->kind == ORACLE_EPI_RPROP) { /* torch/optim/rprop.py _single_tensor_rprop */
            float g = epi->maximize ? d : -d;
            const float s = g * m[i];
            float sv;                                                     /* sign -> etaplus / etaminus / 1 */
            if (s > 0.0f) sv = (float)epi->etaplus;
            else if (s < 0.0f) sv = (float)epi->etaminus;
            else if (s == 0.0f) sv = 1.0f;
            else sv = s;                                                  /* NaN stays NaN */
            float st = v[i] * sv;
            if (st == st) {                                               /* clamp_(min, max); NaN propagates */
                if (st < (float)epi->step_size_min) st = (float)epi->step_size_min;
                if (st > (float)epi->step_size_max) st = (float)epi->step_size_max;
            }
            if (sv == (float)epi->etaminus) g = 0.0f;                     /* grad[sign.eq(etaminus)] = 0 */
            float sg = g > 0.0f ? 1.0f : (g < 0.0f ? -1.0f : (g == 0.0f ? 0.0f : g));
            p[i] = fmaf(-1.0f * sg, st, p[i]);                            /* addcmul_(grad.sign(), step_size, -1) */
            m[i] = g;
            v[i] = st;
        } else if (epi->kind == ORACLE_EPI_NADAM || epi->kind == ORACLE_EPI_RADAM) {
            float g = epi->maximize ? d : -d;
            float pv = p[i];
            if (epi->weight_decay != 0.0) {
                if (epi->decoupled_weight_decay) pv = pv * (float)(1.0 - epi->lr * epi->weight_decay);
                else g = fmaf(pv, (float)epi->weight_decay, g);
            }
            m[i] = lerp_torch(m[i], g, (float)(1.0 - epi->beta1));
            v[i] = fmaf((float)(1.0 - epi->beta2) * g, g, v[i] * (float)epi->beta2);
            const double bc1 = 1.0 - pow(epi->beta1, epi->step);
            const double bc2 = 1.0 - pow(epi->beta2, epi->step);
            if (epi->kind == ORACLE_EPI_NADAM) { /* nadam.py: two addcdiv_ on denom = sqrt(v / bc2) + eps */
                const double mu = epi->beta1 * (1.0 - 0.5 * pow(0.96, epi->step * epi->momentum_decay));
                const double mu_next = epi->beta1 * (1.0 - 0.5 * pow(0.96, (epi->step + 1.0) * epi->momentum_decay));
                const float mp = (float)epi->mu_product * (float)mu;          /* mu_product *= mu (fp32 tensor) */
                const float c_grad = (float)((-epi->lr * (1.0 - mu)) / (1.0 - (double)mp));
                const float c_avg = (float)((-epi->lr * mu_next) / (1.0 - (double)mp * mu_next));
                const float denom = sqrt_e(epi, v[i] / (float)bc2) + (float)epi->eps;
                pv = pv + (c_grad * g) / denom;
                pv = pv + (c_avg * m[i]) / denom;
            } else { /* radam.py: rectified when rho_t > 5 */
                const double rho_inf = 2.0 / (1.0 - epi->beta2) - 1.0;
                const double rho_t = rho_inf - 2.0 * epi->step * pow(epi->beta2, epi->step) / bc2;
                float t = (m[i] / (float)bc1) * (float)epi->lr;                /* exp_avg / bc1 * lr */
                if (rho_t > 5.0) {
                    const float rect = (float)pow((rho_t - 4.0) * (rho_t - 2.0) * rho_inf /
                                                  ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t), 0.5);
                    const float a = (1.0f / (sqrt_e(epi, v[i]) + (float)epi->eps)) * (float)pow(bc2, 0.5); /* bc2**.5 / x */
                    t = (t * a) * rect;
                }
                pv = pv - t;                                                   /* param.add_(t, alpha=-1) */
            }
            p[i] = pv;
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
            float vden = vv;
            if (epi->amsgrad) { /* adam.py: torch.maximum(max_exp_avg_sq, exp_avg_sq, out=max_exp_avg_sq) */
                vmax[i] = max_torch(vmax[i], vv);
                vden = vmax[i];
            }
            const float denom = sqrt_e(epi, vden) / bc2s + (float)epi->eps;
            pv = pv + (step_size_neg * mm) / denom;
            m[i] = mm;
            v[i] = vv;
            p[i] = pv;
        }
    }
}

/* ------------------------------------------------------------------------------------------------
 * Dequantisation, nvflare/app_opt/pt/quantization/dequantizer.py:47-185.
 *   float16     fp16 -> fp32 (exact widening)                                     :98-100, :168-173
 *   blockwise8  code[q[i]] * absmax[i / blocksize]          bitsandbytes dequantize_blockwise (kernel
 *               kDequantizeBlockwise, General8bit: one fp32 multiply)
 *   float4      (fp4(nib) * absmax[i / blocksize]) * sign   bitsandbytes dDequantizeFP4Tree
 *   normfloat4  nf4(nib) * absmax[i / blocksize]            bitsandbytes dDequantizeNF4
 *               byte k: element 2k = high nibble, 2k+1 = low nibble
 *   adaquant    (float)(((double)q * norm) / level - offset)   ada_quant.py:76-87 (+ .float(), :168-173)
 * bitsandbytes is third-party (setup.cfg:74, unpinned) and absent here: its published arithmetic is
 * restated; "parity unpinned" for blockwise8 / float4 / normfloat4.
 * ------------------------------------------------------------------------------------------------ */
enum { ORACLE_Q_F16 = 1, ORACLE_Q_BF16 = 2, ORACLE_Q_BLOCKWISE8 = 3, ORACLE_Q_FP4 = 4, ORACLE_Q_NF4 = 5,
       ORACLE_Q_ADA_U8 = 6, ORACLE_Q_ADA_U16 = 7 };

static const float oracle_nf4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                     -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                     0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                     0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                     0.7229568362236023f, 1.0f};
static const float oracle_fp4[8] = {0.0f, 5.208333333e-03f, 0.66666667f, 1.0f, 0.33333333f, 0.5f, 0.16666667f, 0.25f};

static float oracle_half_to_float(uint16_t h) {
    const uint32_t sign = (uint32_t)(h >> 15) << 31;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = sign;
        } else { /* subnormal half: normalise */
            int sh = 0;
            while (!(m & 0x400)) { m <<= 1; ++sh; }
            m &= 0x3ff;
            bits = sign | ((uint32_t)(127 - 15 + 1 - sh) << 23) | (m << 13);
        }
    } else if (e == 31) {
        bits = sign | 0x7f800000u | (m << 13);
    } else {
        bits = sign | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

void oracle_dequantize(int qtype, const void* q, size_t n, const float* absmax, const float* code, size_t blocksize,
                       double norm, double level, double offset, int has_norm, float* out) {
    const uint8_t* q8 = (const uint8_t*)q;
    const uint16_t* q16 = (const uint16_t*)q;
    for (size_t i = 0; i < n; ++i) {
        float v;
        switch (qtype) {
            case ORACLE_Q_F16: v = oracle_half_to_float(q16[i]); break;
            case ORACLE_Q_BF16: {
                const uint32_t b = (uint32_t)q16[i] << 16;
                memcpy(&v, &b, 4);
                break;
            }
            case ORACLE_Q_BLOCKWISE8: v = code[q8[i]] * absmax[i / blocksize]; break;
            case ORACLE_Q_FP4:
            case ORACLE_Q_NF4: {
                const unsigned byte = q8[i >> 1];
                const unsigned nib = (i & 1) ? (byte & 15u) : (byte >> 4);
                const float am = absmax[i / blocksize];
                if (qtype == ORACLE_Q_NF4) {
                    v = oracle_nf4[nib] * am;
                } else {
                    const float sign = (nib & 8u) ? -1.0f : 1.0f;
                    v = (oracle_fp4[nib & 7u] * am) * sign;
                }
                break;
            }
            default: { /* adaquant */
                if (!has_norm) {
                    v = (float)(0.0 - offset);
                } else {
                    const double x = qtype == ORACLE_Q_ADA_U8 ? (double)q8[i] : (double)q16[i];
                    v = (float)((x * norm) / level - offset);
                }
            }
        }
        out[i] = v;
    }
}
