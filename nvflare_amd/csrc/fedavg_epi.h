// fedavg_epi.h -- the fp32 tiled aggregation kernel with a fused server-optimizer epilogue (SURVEY.md section 8
// rows a9 / a10) and its launch templates; included by fedavg_epi_{numpy,torch,unweighted}.hip.
#pragma once

#include <type_traits>

#include "fedavg_arith.h"

namespace fedavg {

// ---------------------------------------------------------------------------------------------
// The hot kernel with a server-optimizer EPILOGUE fused behind the finalisation (SURVEY.md section 8
// rows a9/a10): d = fin(acc) is not stored but consumed per element by
//   EPI_ADD_BASE  w = base + d                          full_model_shareable_generator.py:58-67
//   EPI_SGD       torch _single_tensor_sgd on g = -d     app_opt/pt/fedopt.py:157-182
//   EPI_ADAM      torch _single_tensor_adam on g = -d    torch/optim/adam.py:347-551
//   EPI_ADAGRAD / RMSPROP / ADAMAX / NADAM / RADAM / RPROP / ASGD   torch _single_tensor_{adagrad,...,asgd} on g = -d
// Per parameter: 4K bytes of client reads + 12 B (p, m, v) read + 12 B written for Adam, so the
// optimizer costs one pass instead of the reference's separate aggregate / H2D / step / D2H round trip.
// Rounding sequence pinned against torch CPU by tests/test_fedopt_oracle.py (fma for add(alpha), lerp
// and addcmul; torch CPU's sqrt or IEEE: sqrt_e).  Geometry fixed at the tuned default (T = 4096, unroll 4, nontemporal).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float lerp_torch(float s, float e, float w, float w_m1) {
    const float d = e - s;
    return fabsf(w) < 0.5f ? __builtin_fmaf(w, d, s) : __builtin_fmaf(w_m1, d, e);
}

// Epilogue operands of one f32x4 column group, loaded at the START of the tile so their HBM latency
// hides behind the client stream instead of stalling the wave after the last client.
struct EpiIn {
    f32x4 a, b, c, d;  // ADD_BASE: base | SGD: p, momentum buffer | ADAM: p, exp_avg, exp_avg_sq (, max_exp_avg_sq)
};

template <int SQ>  // EPI & kEpiSqrtMask
__device__ __forceinline__ float sqrt_e(const EpiParams& E, const float x) {
    if constexpr (SQ == kEpiTorchSqrt) return sqrt_torch_cpu(x);
    if constexpr (SQ == kEpiTorchSqrtAmd) return sqrt_mkl_rsqrtps(x);
    return __builtin_sqrtf(x);
}

// torch.maximum: a NaN operand is the result
__device__ __forceinline__ float max_torch(float a, float b) {
    if (a != a) return a;
    if (b != b) return b;
    return a > b ? a : b;
}

// the epilogues' launch-constant divisors, prepared once per thread (fedavg_arith.h div_const)
struct EpiConsts {
    FinConst bc2s;  // Adam: sqrt(bias_correction2)
    FinConst bc2;   // NAdam: bias_correction2
    FinConst bc1;   // RAdam: bias_correction1
};

template <int EPI>
__device__ __forceinline__ EpiConsts epi_consts(const EpiParams& E) {
    constexpr int KIND = EPI & 0xFF;
    EpiConsts C{};
    if constexpr (KIND == FEDAVG_EPI_ADAM) C.bc2s = div_const_init(E.bias_correction2_sqrt);
    if constexpr (KIND == FEDAVG_EPI_NADAM) C.bc2 = div_const_init(E.bias_correction2);
    if constexpr (KIND == FEDAVG_EPI_RADAM) C.bc1 = div_const_init(E.bias_correction1);
    return C;
}

template <int EPI>
__device__ __forceinline__ EpiIn epi_load(const EpiParams& E, const int64_t i) {
    constexpr int KIND = EPI & 0xFF;
    EpiIn in;
    if constexpr (KIND == FEDAVG_EPI_ADD_BASE) {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.base) + i);
    } else if constexpr (KIND == FEDAVG_EPI_SGD) {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.param) + i);
        if (E.has_momentum && !E.first_step) in.b = load4<true>(reinterpret_cast<const f32x4*>(E.state1) + i);
    } else if constexpr (KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_ASGD) {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.param) + i);
        in.b = load4<true>(reinterpret_cast<const f32x4*>(E.state1) + i);
    } else if constexpr (KIND == FEDAVG_EPI_RMSPROP) {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.param) + i);
        in.b = load4<true>(reinterpret_cast<const f32x4*>(E.state1) + i);
        if (E.has_momentum) in.c = load4<true>(reinterpret_cast<const f32x4*>(E.state2) + i);
        if (E.centered) in.d = load4<true>(reinterpret_cast<const f32x4*>(E.state3) + i);
    } else if constexpr (KIND == FEDAVG_EPI_ADAMAX || KIND == FEDAVG_EPI_RPROP) {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.param) + i);
        in.b = load4<true>(reinterpret_cast<const f32x4*>(E.state1) + i);
        in.c = load4<true>(reinterpret_cast<const f32x4*>(E.state2) + i);
    } else {
        in.a = load4<true>(reinterpret_cast<const f32x4*>(E.param) + i);
        in.b = load4<true>(reinterpret_cast<const f32x4*>(E.state1) + i);
        in.c = load4<true>(reinterpret_cast<const f32x4*>(E.state2) + i);
        if (E.amsgrad) in.d = load4<true>(reinterpret_cast<const f32x4*>(E.state3) + i);
    }
    return in;
}

// The epilogues' sqrt and constant-divisor quotient (round 5), in one of three forms EM, every one bit-identical:
// kEmFast -- straight-line, each rare input (sqrt_torch_cpu / sqrt_mkl_rsqrtps callouts, div_const outside its checked
// range) only noted in `slow`; epilogue4 recomputes the column group with kEmElem when any lane noted one, so the
// common case has one branch per column group instead of one per sqrt and quotient; kEmElem -- the per-element forms
// with their rare-case branches (round 4); kEmIeee -- the constant-divisor quotients as the IEEE division, branch-free
// (round 3), the sqrt per element.
constexpr int kEmFast = 0;
constexpr int kEmElem = 1;
constexpr int kEmIeee = 2;

template <int SQ, int EM>
__device__ __forceinline__ float sqrt_x(const EpiParams& E, const float x, uint32_t& slow) {
    if constexpr (EM == kEmFast && SQ == kEpiTorchSqrt) return sqrt_torch_cpu_fast(x, slow);
    if constexpr (EM == kEmFast && SQ == kEpiTorchSqrtAmd) return sqrt_mkl_rsqrtps_fast(x, slow);
    return sqrt_e<SQ>(E, x);
}

template <int EM>
__device__ __forceinline__ float div_x(const float a, const FinConst& f, uint32_t& slow) {
    if constexpr (EM == kEmFast) return div_const_fast_z(a, f, slow);
    if constexpr (EM == kEmIeee) return a / f.v;
    return div_const(a, f);
}

// whether the optimizer kind has a rare-input path at all (a restated sqrt, or a constant-divisor quotient)
template <int EPI>
constexpr bool epi_has_rare() {
    constexpr int KIND = EPI & 0xFF;
    constexpr bool sq = (EPI & kEpiSqrtMask) != 0 &&
                        (KIND == FEDAVG_EPI_ADAM || KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_RMSPROP ||
                         KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM);
    return sq || KIND == FEDAVG_EPI_ADAM || KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM;
}

// one column group's optimizer step: the new parameter (ADD_BASE: the result) in .a, the new states in .b / .c / .d
template <int EPI, int EM>
__device__ __forceinline__ EpiIn epi_compute(const EpiParams& E, const EpiConsts& C, const f32x4 d, const EpiIn& in,
                                             uint32_t& slow) {
    constexpr int KIND = EPI & 0xFF;
    constexpr int TSQ = EPI & kEpiSqrtMask;
    EpiIn o = in;
    if constexpr (KIND == FEDAVG_EPI_ADD_BASE) {
        o.a = in.a + d;
    } else if constexpr (KIND == FEDAVG_EPI_SGD) {
        f32x4 p = in.a;
        f32x4 buf = in.b;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            if (E.has_weight_decay) g = __builtin_fmaf(p[c], E.weight_decay, g);
            if (E.has_momentum) {
                const float b = E.first_step ? g : __builtin_fmaf(g, E.one_minus_dampening, buf[c] * E.momentum);
                buf[c] = b;
                g = E.nesterov ? __builtin_fmaf(b, E.momentum, g) : b;
            }
            p[c] = __builtin_fmaf(g, E.neg_lr, p[c]);
        }
        o.a = p;
        o.b = buf;
    } else if constexpr (KIND == FEDAVG_EPI_ADAGRAD) {
        f32x4 p = in.a;
        f32x4 sum = in.b;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            if (E.has_weight_decay) g = __builtin_fmaf(p[c], E.weight_decay, g);  // grad.add(param, alpha=wd)
            sum[c] = __builtin_fmaf(g, g, sum[c]);                                 // state_sum.addcmul_(g, g, value=1)
            const float std_ = sqrt_x<TSQ, EM>(E, sum[c], slow) + E.eps;        // state_sum.sqrt().add_(eps)
            p[c] = p[c] + (E.step_size_neg * g) / std_;                            // param.addcdiv_(g, std, value=-clr)
        }
        o.a = p;
        o.b = sum;
    } else if constexpr (KIND == FEDAVG_EPI_RMSPROP) {
        f32x4 p = in.a;
        f32x4 sq = in.b;
        f32x4 buf = in.c;
        f32x4 ga = in.d;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            if (E.has_weight_decay) g = __builtin_fmaf(p[c], E.weight_decay, g);       // grad.add(param, alpha=wd)
            sq[c] = __builtin_fmaf(E.one_minus_beta2 * g, g, sq[c] * E.beta2);       // mul_(alpha).addcmul_(g, g, 1-alpha)
            float avg;
            if (E.centered) {
                ga[c] = lerp_torch(ga[c], g, E.one_minus_beta1, E.one_minus_beta1_m1);  // grad_avg.lerp_(g, 1-alpha)
                avg = sqrt_x<TSQ, EM>(E, __builtin_fmaf(-ga[c], ga[c], sq[c]), slow);  // addcmul(ga, ga, -1).sqrt_()
            } else {
                avg = sqrt_x<TSQ, EM>(E, sq[c], slow);
            }
            avg = avg + E.eps;
            if (E.has_momentum) {
                buf[c] = buf[c] * E.momentum + g / avg;                               // buf.mul_(m).addcdiv_(g, avg)
                p[c] = __builtin_fmaf(buf[c], E.neg_lr, p[c]);                        // param.add_(buf, alpha=-lr)
            } else {
                p[c] = p[c] + (E.neg_lr * g) / avg;                                   // param.addcdiv_(g, avg, -lr)
            }
        }
        o.a = p;
        o.b = sq;
        o.c = buf;
        o.d = ga;
    } else if constexpr (KIND == FEDAVG_EPI_ADAMAX) {
        f32x4 p = in.a;
        f32x4 m = in.b;
        f32x4 u = in.c;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            if (E.has_weight_decay) g = __builtin_fmaf(p[c], E.weight_decay, g);     // grad.add(param, alpha=wd)
            m[c] = lerp_torch(m[c], g, E.one_minus_beta1, E.one_minus_beta1_m1);      // exp_avg.lerp_(g, 1-beta1)
            u[c] = max_torch(u[c] * E.beta2, fabsf(g) + E.eps);                      // maximum(exp_inf*b2, |g|+eps)
            p[c] = p[c] + (E.step_size_neg * m[c]) / u[c];                            // addcdiv_(exp_avg, exp_inf, -clr)
        }
        o.a = p;
        o.b = m;
        o.c = u;
    } else if constexpr (KIND == FEDAVG_EPI_ASGD) {
        f32x4 p = in.a;
        f32x4 ax = in.b;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            if (E.has_weight_decay) g = __builtin_fmaf(p[c], E.weight_decay, g);  // grad.add(param, alpha=wd)
            float pv = p[c] * E.decay;                                             // param.mul_(1 - lambd * eta)
            pv = __builtin_fmaf(g, E.neg_eta, pv);                                 // param.add_(grad, alpha=-eta)
            ax[c] = E.mu != 1.0f ? ax[c] + (pv - ax[c]) * E.mu : pv;               // ax.add_(p.sub(ax).mul_(mu)) | copy_
            p[c] = pv;
        }
        o.a = p;
        o.b = ax;
    } else if constexpr (KIND == FEDAVG_EPI_RPROP) {
        f32x4 p = in.a;
        f32x4 prev = in.b;
        f32x4 ss = in.c;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            const float s = g * prev[c];                                   // grad.mul(prev).sign() -> etas / 1
            const float sv = s > 0.0f ? E.etaplus : (s < 0.0f ? E.etaminus : (s == 0.0f ? 1.0f : s));
            float st = ss[c] * sv;                                         // step_size.mul_(sign).clamp_(min, max)
            st = st != st ? st : fminf(fmaxf(st, E.ss_min), E.ss_max);
            if (sv == E.etaminus) g = 0.0f;                                // grad[sign.eq(etaminus)] = 0
            const float sg = g > 0.0f ? 1.0f : (g < 0.0f ? -1.0f : (g == 0.0f ? 0.0f : g));
            p[c] = __builtin_fmaf(-1.0f * sg, st, p[c]);                  // param.addcmul_(grad.sign(), step_size, -1)
            prev[c] = g;                                                   // prev.copy_(grad)
            ss[c] = st;
        }
        o.a = p;
        o.b = prev;
        o.c = ss;
    } else if constexpr (KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM) {
        f32x4 p = in.a;
        f32x4 m = in.b;
        f32x4 v = in.c;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            float pv = p[c];
            if (E.has_weight_decay) {
                if (E.decoupled_weight_decay) pv = pv * E.decoupled_scale;  // param.mul_(1 - lr * wd)
                else g = __builtin_fmaf(pv, E.weight_decay, g);              // grad.add(param, alpha=wd)
            }
            m[c] = lerp_torch(m[c], g, E.one_minus_beta1, E.one_minus_beta1_m1);
            v[c] = __builtin_fmaf(E.one_minus_beta2 * g, g, v[c] * E.beta2);
            if constexpr (KIND == FEDAVG_EPI_NADAM) {
                // exp_avg_sq.div(bc2).sqrt().add_(eps)
                const float denom = sqrt_x<TSQ, EM>(E, div_x<EM>(v[c], C.bc2, slow), slow) + E.eps;
                pv = pv + (E.coef_grad * g) / denom;                                    // addcdiv_(grad, denom, value)
                pv = pv + (E.coef_avg * m[c]) / denom;                                  // addcdiv_(exp_avg, denom, value)
            } else {
                float t = div_x<EM>(m[c], C.bc1, slow) * E.lr;                        // exp_avg / bc1 * lr
                if (E.rectified) {
                    const float a = (1.0f / (sqrt_x<TSQ, EM>(E, v[c], slow) + E.eps)) * E.bias_correction2_sqrt;
                    t = (t * a) * E.rect;                                               // bc2**0.5 / (sqrt+eps)
                }
                pv = __builtin_fmaf(t, -1.0f, pv);                                      // param.add_(..., alpha=-1)
            }
            p[c] = pv;
        }
        o.a = p;
        o.b = m;
        o.c = v;
    } else {  // EPI_ADAM
        f32x4 p = in.a;
        f32x4 m = in.b;
        f32x4 v = in.c;
        f32x4 vmax = in.d;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float g = E.maximize ? d[c] : -d[c];
            float pv = p[c];
            if (E.has_weight_decay) {
                if (E.decoupled_weight_decay) pv = pv * E.decoupled_scale;
                else g = __builtin_fmaf(pv, E.weight_decay, g);
            }
            const float mm = lerp_torch(m[c], g, E.one_minus_beta1, E.one_minus_beta1_m1);
            const float vv = __builtin_fmaf(E.one_minus_beta2 * g, g, v[c] * E.beta2);
            float vden = vv;
            if (E.amsgrad) {  // adam.py: torch.maximum(max_exp_avg_sq, exp_avg_sq, out=max_exp_avg_sq)
                vmax[c] = max_torch(vmax[c], vv);
                vden = vmax[c];
            }
            const float denom = div_x<EM>(sqrt_x<TSQ, EM>(E, vden, slow), C.bc2s, slow) + E.eps;  // sqrt(v)/sqrt(bc2)+eps
            pv = pv + (E.step_size_neg * mm) / denom;
            m[c] = mm;
            v[c] = vv;
            p[c] = pv;
        }
        o.a = p;
        o.b = m;
        o.c = v;
        o.d = vmax;
    }
    return o;
}

// the epilogue's stores are nontemporal; A/B builds with -DFEDAVG_EPI_TEMPORAL (tools/build_rev_lib.py -D) make them
// temporal, for the device cache to absorb a launch's write burst and write it back on its own schedule: config 5 87.9
// against 88.0 %, the 2-client LDS-DMA form 70.5 against 74.7 % (profiles/r06/s10/, processes alternating) -- not kept
#if defined(FEDAVG_EPI_TEMPORAL)
constexpr bool kEpiNtStores = false;
#else
constexpr bool kEpiNtStores = true;
#endif

template <int EPI>
__device__ __forceinline__ void epi_store(const EpiParams& E, const int64_t i, const EpiIn& o, f32x4* out) {
    constexpr int KIND = EPI & 0xFF;
    constexpr bool NT = kEpiNtStores;
    if constexpr (KIND == FEDAVG_EPI_ADD_BASE) {
        store4<NT>(out + i, o.a);
        return;
    }
    store4<NT>(reinterpret_cast<f32x4*>(E.param) + i, o.a);
    f32x4* s1 = reinterpret_cast<f32x4*>(E.state1) + i;
    f32x4* s2 = reinterpret_cast<f32x4*>(E.state2) + i;
    f32x4* s3 = reinterpret_cast<f32x4*>(E.state3) + i;
    if constexpr (KIND == FEDAVG_EPI_SGD) {
        if (E.has_momentum) store4<NT>(s1, o.b);
    } else if constexpr (KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_ASGD) {
        store4<NT>(s1, o.b);
    } else if constexpr (KIND == FEDAVG_EPI_RMSPROP) {
        store4<NT>(s1, o.b);
        if (E.has_momentum) store4<NT>(s2, o.c);
        if (E.centered) store4<NT>(s3, o.d);
    } else if constexpr (KIND == FEDAVG_EPI_ADAMAX || KIND == FEDAVG_EPI_RPROP || KIND == FEDAVG_EPI_NADAM ||
                         KIND == FEDAVG_EPI_RADAM) {
        store4<NT>(s1, o.b);
        store4<NT>(s2, o.c);
    } else {  // ADAM
        store4<NT>(s1, o.b);
        store4<NT>(s2, o.c);
        if (E.amsgrad) store4<NT>(s3, o.d);
    }
}

template <int EPI, int EM>
__device__ __forceinline__ void epilogue4(const EpiParams& E, const EpiConsts& C, const int64_t i, const f32x4 d,
                                          const EpiIn& in, f32x4* out) {
    if constexpr (EM != kEmFast || !epi_has_rare<EPI>()) {
        uint32_t unused = 0;
        epi_store<EPI>(E, i, epi_compute<EPI, EM == kEmFast ? kEmElem : EM>(E, C, d, in, unused), out);
    } else {
        uint32_t slow = 0;
        if constexpr ((EPI & 0xFF) == FEDAVG_EPI_ADAM) slow = C.bc2s.fast ? 0u : 1u;
        if constexpr ((EPI & 0xFF) == FEDAVG_EPI_NADAM) slow = C.bc2.fast ? 0u : 1u;
        if constexpr ((EPI & 0xFF) == FEDAVG_EPI_RADAM) slow = C.bc1.fast ? 0u : 1u;
        EpiIn o = epi_compute<EPI, kEmFast>(E, C, d, in, slow);
        if (__builtin_expect(wave_any(slow), 0)) {  // every lane: see wave_any
            uint32_t unused = 0;
            o = epi_compute<EPI, kEmElem>(E, C, d, in, unused);
        }
        epi_store<EPI>(E, i, o, out);
    }
}

// the finalisation of one tile's CPL columns in the epilogue's form: one rare-case branch for the tile (kEmFast),
// per element (kEmElem), or the IEEE division (kEmIeee)
template <int FIN, int EM, int CPL>
__device__ __forceinline__ void fin_tile_em(f32x4 (&r)[CPL], const f32x4 (&a)[CPL], const FinConst& f) {
    if constexpr (EM == kEmFast) {
        fin_tile<FIN, CPL>(r, a, f);
    } else if constexpr (EM == kEmElem) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) r[c] = fin4c<FIN>(a[c], f);
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) r[c] = fin4<FIN>(a[c], f.v);
    }
}

// the forms the kernels use (A/B builds: -DFEDAVG_EM_TILE=n / -DFEDAVG_EM_BURST=n), from interleaved A/Bs, fused Adam
// with the AMD-host sqrt, % of 8 TB/s: the burst form kEmFast (64 clients x 2.5e8: 87.4 against 86.8 per element and
// 86.8 with IEEE divisions, profiles/r05/s3/adam_k64_*); the per-tile form kEmElem (2 / 3 clients x 5e8: 69.4 / 68.9
// against 68.5 / 68.7 with kEmFast, s5/adam_k*_tilee, _prod -- its epilogue is one tile at a time, and the fast
// form's longer live ranges cost more there than its fewer branches save)
#if defined(FEDAVG_EM_TILE)
constexpr int kEmTile = FEDAVG_EM_TILE;
#else
constexpr int kEmTile = kEmElem;
#endif
#if defined(FEDAVG_EM_BURST)
constexpr int kEmBurst = FEDAVG_EM_BURST;
#else
constexpr int kEmBurst = kEmFast;
#endif

// PIPE: software-pipelined across tiles -- after the client loop of tile t the lane issues the epilogue
// operand loads of t, then the first UNROLL client loads of its next tile, and only then waits for the
// operands and runs the epilogue (ALU, three store streams) while the next tile's loads are in flight.
// BURST form (the default; see fedavg_tiles.h fedavg_tiles_burst_f32x4): each launch gives every block TPB
// tiles; the aggregated differences d of all of them stay in registers while the client stream runs, and
// the epilogue (operand loads, optimizer arithmetic, the state / parameter stores) runs for all TPB tiles
// at the end of the launch -- the client-read phase carries no writes, and every block's epilogue phase
// falls at about the same time.  `out` (when given) also receives d, as in the per-tile kernel.  TPB_LDS > 0:
// that many more tiles per block, their d held in LDS (each lane reads back only what it wrote).
// LOOP: 0 -- the default, tile_sum_rrem (four-client groups as two pairs from 8 clients on, client_group4 shape 2;
// four together below); A/B only (launch variant bits 9-11): 1 -- tile_sum's GROUPED loop with round 3's repeats;
// 2-4 -- tile_sum_rrem with client_group4 shape LOOP; 5 -- shape 0 (four clients' loads together) everywhere;
// 6 -- the default loop, the epilogue phase without its operand prefetch.  Fused Adam, % of 8 TB/s, shapes 0 / 1 / 2 /
// 3 / 4 in one process (profiles/r04/s6/loop_k*.jsonl): 64 clients 83.2 / 85.6 / 85.4 / 83.8 / 80.4, 32: 80.1 / 82.3 /
// 81.3 / 80.5 / 78.3, 8: 73.5 / 76.6 / 76.4 / 75.9 / 74.0, 10: 75.7 / 75.5 / 75.0 / 75.6 / 76.8, 6: 74.2 / 70.4 /
// 73.6 / 73.7 / 75.7 -- fewer loads in flight per wave stream better once a tile holds two groups or more; the pairs
// are within about a point of the best everywhere and re-load nothing.
template <int OP, int FIN, bool ACC_IN, int EPI, int TPB, int TPB_LDS = 0, int LOOP = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
fedavg_tiles_epi_burst_f32x4(const RowTableF32 tab, const int K, const int64_t tstride4, const f32x4* acc_in,
                             f32x4* out, const int64_t b4, const int64_t e4, const float fin_val, const EpiParams E,
                             const int64_t t0, const int64_t t_end) {
    constexpr int UNROLL = kDefaultUnroll;
    constexpr int CPL = kDefaultTile / (4 * kBlock);
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    constexpr int NT = TPB + TPB_LDS;
    f32x4 dd[TPB][CPL];
    __shared__ f32x4 staged[TPB_LDS > 0 ? TPB_LDS * CPL * kBlock : 1];
    const FinConst fc = fin_const<FIN>(fin_val);
    const EpiConsts C = epi_consts<EPI>(E);
    if constexpr ((EPI & kEpiTorchSqrt) != 0) rsqrt14_stage();
    if constexpr ((EPI & kEpiTorchSqrtAmd) != 0) rsqrtps_stage(E.rsqrtps);
    auto sum = [&](f32x4 (&acc)[CPL], const int64_t t) __attribute__((always_inline)) {
        if constexpr (LOOP == 1)
            tile_sum<OP, ACC_IN, UNROLL, CPL, 2>(acc, tab, K, t * tstride4 + threadIdx.x, t * T4 + threadIdx.x, acc_in,
                                                 b4, e4);
        else
            tile_sum_rrem<OP, ACC_IN, CPL, LOOP == 0 || LOOP == 6 ? -1 : LOOP == 5 ? 0 : LOOP>(
                acc, tab, K, t * tstride4 + threadIdx.x, t * T4 + threadIdx.x, acc_in, b4, e4);
    };
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f32x4 acc[CPL];
            sum(acc, t);
            fin_tile_em<FIN, kEmBurst, CPL>(dd[m], acc, fc);
        }
    }
#pragma unroll 1
    for (int m = TPB; m < NT; ++m) {  // rolled: one more copy of the client loop, not TPB_LDS of them
        const int64_t t = t0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (t < t_end) {
            f32x4 acc[CPL], r[CPL];
            sum(acc, t);
            fin_tile_em<FIN, kEmBurst, CPL>(r, acc, fc);
#pragma unroll
            for (int c = 0; c < CPL; ++c) staged[((m - TPB) * CPL + c) * kBlock + threadIdx.x] = r[c];
        }
    }
    // Epilogue phase, double-buffered: tile m+1's operand loads are issued before tile m's arithmetic and
    // stores (program order keeps them ahead of those stores, which may alias nothing they read but the
    // compiler cannot know).  Loads are unconditional at a clamped in-range address so the waits count
    // exactly one tile's loads; only in-range columns of real tiles are computed and stored.
    const int64_t t_base = t0 + blockIdx.x;
    const int64_t t_cap = t_end - 1;
    auto operands = [&](EpiIn (&in)[CPL], const int m) __attribute__((always_inline)) {
        const int64_t t = t_base + (int64_t)m * gridDim.x;
        const int64_t tc = t < t_cap ? t : t_cap;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            int64_t i = tc * T4 + threadIdx.x + c * kBlock;
            i = i < b4 ? b4 : (i >= e4 ? e4 - 1 : i);
            in[c] = epi_load<EPI>(E, i);
        }
    };
    // cur / nxt with static indices only (a pre[m & 1] buffer in the rolled LDS-tile loop, or in an epilogue too
    // large for the compiler to unroll fully, went to scratch memory: 528 bytes per lane for Adam with the restated
    // torch sqrt)
    // PF (A/B builds: -DFEDAVG_EPI_PF=2): the operands PF tiles ahead (a third buffer, rotated by copies)
#if defined(FEDAVG_EPI_PF)
    constexpr int PF = FEDAVG_EPI_PF;
#else
    constexpr int PF = 1;
#endif
    EpiIn cur[CPL], nxt[CPL], nx2[PF > 1 ? CPL : 1];
    operands(cur, 0);
    if constexpr (PF > 1) {
        if (1 < NT) operands(nxt, 1);
    }
    auto tile_epilogue = [&](const int m, const int64_t t, auto&& d_of) __attribute__((always_inline)) {
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + threadIdx.x + c * kBlock;
                if (i >= b4 && i < e4) {
                    const f32x4 d = d_of(c);
                    if (out != nullptr && (EPI & 0xFF) != FEDAVG_EPI_ADD_BASE) store4<true>(out + i, d);
                    epilogue4<EPI, kEmBurst>(E, C, i, d, cur[c], out);
                }
            }
        }
    };
    constexpr bool PREFETCH = LOOP != 6;  // A/B 6: tile m+1's operands loaded after tile m's stores
    auto rotate = [&](const int m) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) cur[c] = nxt[c];
        if constexpr (PF > 1) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) nxt[c] = nx2[c];
        }
    };
#pragma unroll
    for (int m = 0; m < TPB; ++m) {
        if constexpr (PF > 1) {
            if (m + 2 < NT) operands(nx2, m + 2);
        } else if (PREFETCH && m + 1 < NT) {
            operands(nxt, m + 1);
        }
        tile_epilogue(m, t_base + (int64_t)m * gridDim.x, [&](int c) __attribute__((always_inline)) { return dd[m][c]; });
        if (PF == 1 && !PREFETCH && m + 1 < NT) operands(nxt, m + 1);
        rotate(m);
    }
#pragma unroll 1
    for (int m = TPB; m < NT; ++m) {
        if constexpr (PF > 1) {
            if (m + 2 < NT) operands(nx2, m + 2);
        } else if (PREFETCH && m + 1 < NT) {
            operands(nxt, m + 1);
        }
        tile_epilogue(m, t_base + (int64_t)m * gridDim.x,
                      [&](int c) __attribute__((always_inline)) {
                          return staged[((m - TPB) * CPL + c) * kBlock + threadIdx.x];
                      });
        if (PF == 1 && !PREFETCH && m + 1 < NT) operands(nxt, m + 1);
        rotate(m);
    }
}

// SPLIT-EPILOGUE burst form (round 6; A/B only until measured): the burst form above with a second
// group of four waves per block (512 threads, one block per CU, two waves per SIMD).  The client phase is the burst
// form's, run by waves 0-3 alone (waves 4-7 wait at the block barrier holding no loads); in the epilogue phase both groups
// work at once -- waves 0-3 the register-held tiles and the first XS LDS-held ones, waves 4-7 the other LDS-held tiles
// (their d is in LDS, readable by any wave after the barrier) -- so the epilogue's optimizer arithmetic issues from two
// waves per SIMD (a VALU op every 2 cycles instead of every 4) while the other group's operand loads and stores run.
// Registers: 256 per wave at two waves per SIMD, so TPB register-held tiles are fewer than the burst form's 8.
// (Waves 4-7 issuing their first tile's operand loads before the barrier keeps 48 more registers live through the
// client phase: 100-190 bytes of scratch per lane at every geometry. Not done.)
template <int OP, int FIN, int EPI, int TPB, int TPB_LDS, int XS>
__global__ void __launch_bounds__(2 * kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
fedavg_tiles_epi_split_f32x4(const RowTableF32 tab, const int K, const int64_t tstride4, f32x4* out, const int64_t b4,
                             const int64_t e4, const float fin_val, const EpiParams E, const int64_t t0,
                             const int64_t t_end) {
    constexpr int CPL = kDefaultTile / (4 * kBlock);
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    constexpr int NT = TPB + TPB_LDS;
    static_assert(XS >= 0 && XS <= TPB_LDS, "split of the LDS-held tiles");
    f32x4 dd[TPB][CPL];
    __shared__ f32x4 staged[TPB_LDS > 0 ? TPB_LDS * CPL * kBlock : 1];
    const FinConst fc = fin_const<FIN>(fin_val);
    const EpiConsts C = epi_consts<EPI>(E);
    if constexpr ((EPI & kEpiTorchSqrt) != 0) rsqrt14_stage();
    if constexpr ((EPI & kEpiTorchSqrtAmd) != 0) rsqrtps_stage(E.rsqrtps);
    const bool helper = __builtin_amdgcn_readfirstlane(threadIdx.x) >= kBlock;  // waves 4-7
    const int tid = threadIdx.x & (kBlock - 1);
    const int64_t t_base = t0 + blockIdx.x;
    const int64_t t_cap = t_end - 1;
    auto operands = [&](EpiIn (&in)[CPL], const int m) __attribute__((always_inline)) {
        const int64_t t = t_base + (int64_t)m * gridDim.x;
        const int64_t tc = t < t_cap ? t : t_cap;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            int64_t i = tc * T4 + tid + c * kBlock;
            i = i < b4 ? b4 : (i >= e4 ? e4 - 1 : i);
            in[c] = epi_load<EPI>(E, i);
        }
    };
    EpiIn cur[CPL], nxt[CPL];
    if (!helper) {  // the client phase: the burst form's, on waves 0-3
        auto sum = [&](f32x4 (&acc)[CPL], const int64_t t) __attribute__((always_inline)) {
            tile_sum_rrem<OP, false, CPL, -1>(acc, tab, K, t * tstride4 + tid, t * T4 + tid, nullptr, b4, e4);
        };
#pragma unroll
        for (int m = 0; m < TPB; ++m) {
            const int64_t t = t_base + (int64_t)m * gridDim.x;
            if (t < t_end) {
                f32x4 acc[CPL];
                sum(acc, t);
                fin_tile_em<FIN, kEmBurst, CPL>(dd[m], acc, fc);
            }
        }
#pragma unroll 1
        for (int m = TPB; m < NT; ++m) {
            const int64_t t = t_base + (int64_t)m * gridDim.x;
            if (t < t_end) {
                f32x4 acc[CPL], r[CPL];
                sum(acc, t);
                fin_tile_em<FIN, kEmBurst, CPL>(r, acc, fc);
#pragma unroll
                for (int c = 0; c < CPL; ++c) staged[((m - TPB) * CPL + c) * kBlock + tid] = r[c];
            }
        }
    }
    __syncthreads();  // the LDS-held d visible to every wave
    auto tile_epilogue = [&](const int64_t t, auto&& d_of) __attribute__((always_inline)) {
        if (t < t_end) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = t * T4 + tid + c * kBlock;
                if (i >= b4 && i < e4) {
                    const f32x4 d = d_of(c);
                    if (out != nullptr && (EPI & 0xFF) != FEDAVG_EPI_ADD_BASE) store4<true>(out + i, d);
                    epilogue4<EPI, kEmBurst>(E, C, i, d, cur[c], out);
                }
            }
        }
    };
    auto rotate = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) cur[c] = nxt[c];
    };
    auto lds_d = [&](const int m) __attribute__((always_inline)) {
        return [&, m](int c) __attribute__((always_inline)) { return staged[((m - TPB) * CPL + c) * kBlock + tid]; };
    };
    if (!helper) {  // the register-held tiles, then LDS-held tiles TPB .. TPB + XS - 1
        constexpr int LAST = TPB + XS;
        operands(cur, 0);
#pragma unroll
        for (int m = 0; m < TPB; ++m) {
            if (m + 1 < LAST) operands(nxt, m + 1);
            tile_epilogue(t_base + (int64_t)m * gridDim.x, [&](int c) __attribute__((always_inline)) { return dd[m][c]; });
            rotate();
        }
#pragma unroll 1
        for (int m = TPB; m < LAST; ++m) {
            if (m + 1 < LAST) operands(nxt, m + 1);
            tile_epilogue(t_base + (int64_t)m * gridDim.x, lds_d(m));
            rotate();
        }
    } else {  // LDS-held tiles TPB + XS .. NT - 1
        operands(cur, TPB + XS);
#pragma unroll 1
        for (int m = TPB + XS; m < NT; ++m) {
            if (m + 1 < NT) operands(nxt, m + 1);
            tile_epilogue(t_base + (int64_t)m * gridDim.x, lds_d(m));
            rotate();
        }
    }
}

template <int OP, int FIN, bool ACC_IN, int EPI, bool PIPE>
__global__ void __launch_bounds__(kBlock) fedavg_tiles_epi_f32x4(const RowTableF32 tab, const int K,
                                                                  const int64_t tstride4, const f32x4* acc_in,
                                                                  f32x4* out, const int64_t b4, const int64_t e4,
                                                                  const float fin_val, const EpiParams E) {
    constexpr int UNROLL = kDefaultUnroll;
    constexpr int CPL = kDefaultTile / (4 * kBlock);
    constexpr int64_t T4 = (int64_t)CPL * kBlock;
    const int64_t t_last = (e4 - 1) / T4;
    const int g0 = PIPE ? (K < UNROLL ? K : UNROLL) : 0;  // clients carried over from the previous tile
    const FinConst fc = fin_const<FIN>(fin_val);
    const EpiConsts C = epi_consts<EPI>(E);
    if constexpr ((EPI & kEpiTorchSqrt) != 0) rsqrt14_stage();
    if constexpr ((EPI & kEpiTorchSqrtAmd) != 0) rsqrtps_stage(E.rsqrtps);
    f32x4 nxt[UNROLL][CPL];
    int64_t t = b4 / T4 + blockIdx.x;
    // kPipeOps (A/B builds: -DFEDAVG_EPI_PIPE2): the next tile's epilogue operands go out with its first clients too,
    // at clamped in-range addresses (a partial edge tile's extra columns are loaded, never used)
#if defined(FEDAVG_EPI_PIPE2)
    constexpr bool kPipeOps = PIPE;
#else
    constexpr bool kPipeOps = false;
#endif
    EpiIn preN[kPipeOps ? CPL : 1];
    auto ops_of = [&](EpiIn (&dst)[kPipeOps ? CPL : 1], const int64_t tt) __attribute__((always_inline)) {
        if constexpr (kPipeOps) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                int64_t i = tt * T4 + threadIdx.x + c * kBlock;
                i = i < b4 ? b4 : (i >= e4 ? e4 - 1 : i);
                dst[c] = epi_load<EPI>(E, i);
            }
        }
    };
    if constexpr (PIPE) {
        if (t <= t_last) {
            const int64_t off = t * tstride4 + threadIdx.x;
#pragma unroll
            for (int j = 0; j < UNROLL; ++j)
                if (j < g0)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) nxt[j][c] = load4<true>(tab.rows[j] + off + c * kBlock);
            ops_of(preN, t);
        }
    }
    for (; t <= t_last; t += gridDim.x) {
        const int64_t off = t * tstride4 + threadIdx.x;
        const int64_t col = t * T4 + threadIdx.x;
        f32x4 acc[CPL];
        int k = 0;
        if constexpr (ACC_IN) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = col + c * kBlock;
                acc[c] = (i >= b4 && i < e4) ? load4<false>(acc_in + i) : f32x4{0, 0, 0, 0};
            }
        } else if constexpr (!PIPE) {
            const f32x4* r = tab.rows[0] + off;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = first4<OP>(load4<true>(r + c * kBlock), tab.w[0]);
            k = 1;
        }
        if constexpr (PIPE) {  // consume the carried group (clients 0 .. g0-1)
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                if (j < g0) {
#pragma unroll
                    for (int c = 0; c < CPL; ++c) {
                        if (!ACC_IN && j == 0) acc[c] = first4<OP>(nxt[0][c], tab.w[0]);
                        else acc[c] = step4<OP>(acc[c], nxt[j][c], tab.w[j]);
                    }
                }
            }
            k = g0;
        }
        for (; k + UNROLL <= K; k += UNROLL) {
            f32x4 v[UNROLL][CPL];
#pragma unroll
            for (int j = 0; j < UNROLL; ++j) {
                const f32x4* r = tab.rows[k + j] + off;
#pragma unroll
                for (int c = 0; c < CPL; ++c) v[j][c] = load4<true>(r + c * kBlock);
            }
#pragma unroll
            for (int j = 0; j < UNROLL; ++j)
#pragma unroll
                for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], v[j][c], tab.w[k + j]);
        }
        for (; k < K; ++k) {
            const f32x4* r = tab.rows[k] + off;
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc[c] = step4<OP>(acc[c], load4<true>(r + c * kBlock), tab.w[k]);
        }
        EpiIn pre[CPL];
        if constexpr (kPipeOps) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) pre[c] = preN[c];
        } else {
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int64_t i = col + c * kBlock;
                if (i >= b4 && i < e4) pre[c] = epi_load<EPI>(E, i);
            }
        }
        if constexpr (PIPE) {
            const int64_t tn = t + gridDim.x;
            if (tn <= t_last) {
                const int64_t offn = tn * tstride4 + threadIdx.x;
#pragma unroll
                for (int j = 0; j < UNROLL; ++j)
                    if (j < g0)
#pragma unroll
                        for (int c = 0; c < CPL; ++c) nxt[j][c] = load4<true>(tab.rows[j] + offn + c * kBlock);
                ops_of(preN, tn);
            }
        }
        f32x4 dv[CPL];
        fin_tile_em<FIN, kEmTile, CPL>(dv, acc, fc);
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int64_t i = col + c * kBlock;
            if (i >= b4 && i < e4) {
                if (out != nullptr && (EPI & 0xFF) != FEDAVG_EPI_ADD_BASE) store4<true>(out + i, dv[c]);
                epilogue4<EPI, kEmTile>(E, C, i, dv[c], pre[c], out);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// FEW-CLIENT fused form on LDS-DMA (round 6): 1-3 client reads, no chained sum.  The per-tile
// form above (the route through round 5) stores each tile's new parameters and states as it finishes -- small writes
// scattered through the read stream, a pattern that ran 67.9 % of 8 TB/s in the epilogue-shaped probe (e_tile2,
// profiles/r04/s2/epi_r2.jsonl) against 76.3 % when a launch's results are held on chip and stored as one chip-wide
// burst (e_burst_r4).  Holding the new p, m, v in registers with the loads in VGPRs ran 53 % (fedavg_tiles_epi_few_f32x4,
// A/B only): at one wave per SIMD a tile's ~50 VALU per element of optimizer arithmetic ran with nothing in flight.
// Here every input goes HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPRs while in flight), so a wave keeps S
// units' loads in flight while it computes:
//   * a UNIT is one wave's 1 KiB piece of every input stream of a tile column (64 lanes x float4): the KC client segments
//     and the NIN operand streams (p, exp_avg, exp_avg_sq ... by optimizer kind) -- G = KC + NIN DMAs, landing at
//     ring[wave][slot][stream][lane], the lane's own element group, so a wave only ever reads what it loaded itself and
//     its own counted `s_waitcnt vmcnt` orders the read (no barriers; MI355X_MICROARCH.md item 7);
//   * a wave runs N units per launch (N / 4 tiles per block, the tiles dealt round-robin as in the burst kernels): units
//     0 .. S-1 are issued at once; unit u is computed from its slot as soon as it lands (d = fin(sum) and the optimizer
//     step, epi_compute), its results kept in VGPRs and the slot refilled with unit u + S; the last S units' results
//     are written back into their slots;
//   * then every result is stored -- the launch's write burst.
// Only the LDS-DMA instructions touch global memory before the burst (the wait counts are exact: vmcnt counts them in
// issue order, G per unit); inputs past the range are read at clamped in-range addresses and never stored.
// Per-element sequence as the per-tile form's (first4 / step4, fin_tile, epi_compute): the bits are the same.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_byte_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// one LDS-DMA of 16 bytes per lane (the wave's 1 KiB lands at lds_dst + lane x 16); nontemporal like every client load.
// M0 carries the LDS base and is written and restored inside the statement (cdna_hip_programming.md, inline asm).
__device__ __forceinline__ void glds16(const void* gsrc, const uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// the wave's LDS reads done before an LDS-DMA into the same bytes is issued: hipcc issues a slot's ds_reads, then the
// refill's DMAs, and waits for the reads only where it uses their values (the compute may be scheduled after the
// DMAs); a DMA that hits in L2 -- a clamped tile re-read -- can then land before a queued read (round 6, session 2:
// one wave-unit of 256 elements wrong in the last, partial launch)
__device__ __forceinline__ void wait_lgkmcnt0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is six bits on gfx950");
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int I, int END, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < END) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, END>(f);
    }
}

// result streams an optimizer kind writes (the EpiIn fields .a .. .d it fills)
template <int EPI>
constexpr int epi_nout() {
    constexpr int KIND = EPI & 0xFF;
    if constexpr (KIND == FEDAVG_EPI_ADD_BASE) return 1;
    if constexpr (KIND == FEDAVG_EPI_SGD || KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_ASGD) return 2;
    if constexpr (KIND == FEDAVG_EPI_RMSPROP) return 4;
    return 3;  // ADAM (no amsgrad on this form), ADAMAX, NADAM, RADAM, RPROP
}

// LDS per block left for the ring beside the epilogue's sqrt table (16 KiB RSQRTPS table, or the AVX-512 path's 512 B)
template <int EPI>
constexpr int epi_dma_ring_bytes() {
    return kLdsBytesPerCu - ((EPI & kEpiTorchSqrtAmd) ? 16 * 1024 : (EPI & kEpiTorchSqrt) ? 1024 : 0);
}
constexpr int kEpiDmaUnits = 16;  // units per wave per launch by default (A/B forms; EpiDmaGeom has the product's)
// ring slots per wave: as many as the LDS holds, with every in-flight DMA countable by vmcnt (<= 63), at most N
template <int EPI, int G, int N = kEpiDmaUnits, int W = 4>
constexpr int epi_dma_slots() {
    const int by_lds = epi_dma_ring_bytes<EPI>() / (W * G * 1024);
    const int by_cnt = 63 / G + 1;
    const int s = by_lds < by_cnt ? by_lds : by_cnt;
    return s < N ? s : N;
}

// TDMA: the AMD hosts' 16 KiB RSQRTPS table staged by LDS-DMA too, each wave a quarter, issued before the units' DMAs
// (so unit 0's wait covers it) and published by one barrier -- instead of rsqrtps_stage's loads, wait and barrier
// ahead of every launch's first DMA.  EM: the epilogue arithmetic's form (kEmFast with one fallback per unit, or kEmElem)
// W: waves per block (one block per CU): 4 -- one wave per SIMD, up to 512 registers each (arch + accumulation VGPRs
// hold the results); 8 -- two waves per SIMD, 256 registers each, the SIMD's VALU issue shared by two instruction
// streams (one wave alone issues a VALU op every 4 cycles, two every 2: MI355X_MICROARCH.md constants table)
template <int OP, int FIN, int EPI, int KC, int NIN, int S, int N, bool TDMA = false, int EM = kEmFast, int W = 4>
__global__ void __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4, W / 4)))
fedavg_tiles_epi_dma_f32x4(const RowTableF32 tab, const int64_t tstride4, f32x4* out, const int64_t b4,
                           const int64_t e4, const float fin_val, const EpiParams E_, const int64_t t0,
                           const int64_t t_end) {
    constexpr int G = KC + NIN;
    static_assert(W == 4 || W == 8, "4 or 8 waves per block");
    constexpr int CPT = 64 / (4 * W);       // float4 columns per lane per tile (4 at W = 4, 2 at W = 8)
    constexpr int64_t T4 = kDefaultTile / 4;  // float4 per tile; a tile is 16 wave pieces of 64 float4
    constexpr int KIND = EPI & 0xFF;
    // RMSprop on this form: its momentum buffer read iff NIN >= 3, centered (grad_avg) iff NIN == 4 -- results p,
    // square_avg (, buffer (, grad_avg)); Adam: amsgrad (max_exp_avg_sq) iff NIN == 4
    constexpr int NOUT = KIND == FEDAVG_EPI_RMSPROP || (KIND == FEDAVG_EPI_ADAM && NIN == 4) ? NIN : epi_nout<EPI>();
    static_assert(KC >= 1 && KC <= 3 && NIN >= 1 && NIN <= 4 && NOUT <= G, "few-client fused form");
    static_assert(KIND != FEDAVG_EPI_RMSPROP || NIN >= 2, "RMSprop reads p and square_avg");
    static_assert(NIN < 4 || KIND == FEDAVG_EPI_ADAM || KIND == FEDAVG_EPI_RMSPROP, "four operand streams");
    static_assert(S >= 1 && S <= N && (S - 1) * G <= 63 && N % CPT == 0, "ring geometry");
    static_assert((int64_t)W * S * G * 1024 <= epi_dma_ring_bytes<EPI>(), "ring fits the CU's LDS");
    __shared__ f32x4 ring[W][S][G][64];
    EpiParams E = E_;
    if constexpr (KIND == FEDAVG_EPI_ADAM) E.amsgrad = NIN == 4;  // the operand streams say which flags are on
    if constexpr (KIND == FEDAVG_EPI_RMSPROP) {
        E.centered = NIN == 4;
        E.has_momentum = NIN >= 3;
    }
    const FinConst fc = fin_const<FIN>(fin_val);
    const EpiConsts C = epi_consts<EPI>(E);
    constexpr bool kTableDma = TDMA && (EPI & kEpiTorchSqrtAmd) != 0;
    if constexpr ((EPI & kEpiTorchSqrt) != 0) rsqrt14_stage();
    if constexpr ((EPI & kEpiTorchSqrtAmd) != 0 && !kTableDma) rsqrtps_stage(E.rsqrtps);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if constexpr (kTableDma) {
#pragma unroll
        for (int j = 0; j < 16 / W; ++j)  // 16 KiB: 16 / W pieces of 1 KiB per wave
            glds16(reinterpret_cast<const uint4*>(E.rsqrtps) + (wave * (16 / W) + j) * 64 + lane,
                   lds_byte_addr(&g_rsqrtps_lds[(wave * (16 / W) + j) * 256]));
    }
    // operand streams in EpiIn order (.a, .b, .c, .d): the parameter (ADD_BASE: the base) and the optimizer states
    const float* opnd[4] = {(EPI & 0xFF) == FEDAVG_EPI_ADD_BASE ? E.base : E.param, E.state1, E.state2, E.state3};
    const int64_t t_first = t0 + blockIdx.x;
    auto tile_of = [&](const int u) __attribute__((always_inline)) {
        const int64_t t = t_first + (int64_t)(u / CPT) * gridDim.x;
        return t < t_end ? t : t_end - 1;
    };
    auto issue = [&](const int u, const int slot) __attribute__((always_inline)) {
        const int64_t t = tile_of(u);
        const int64_t col = (int64_t)(u % CPT) * (W * 64) + threadIdx.x;
#pragma unroll
        for (int k = 0; k < KC; ++k) glds16(tab.rows[k] + t * tstride4 + col, lds_byte_addr(&ring[wave][slot][k][0]));
        int64_t i = t * T4 + col;
        i = i < b4 ? b4 : (i >= e4 ? e4 - 1 : i);  // a partial edge tile: in-range operands, never stored
#pragma unroll
        for (int j = 0; j < NIN; ++j)
            glds16(reinterpret_cast<const f32x4*>(opnd[j]) + i, lds_byte_addr(&ring[wave][slot][KC + j][0]));
    };
    static_for<0, S>([&](auto ic) {
        constexpr int u = decltype(ic)::value;
        issue(u, u);
    });
    EpiIn res[N > S ? N - S : 1];
    static_for<0, N>([&](auto ic) {
        constexpr int u = decltype(ic)::value;
        constexpr int slot = u % S;
        constexpr int issued = S + u < N ? S + u : N;  // units issued before unit u's wait
        wait_vmcnt<(issued - u - 1) * G>();
        if constexpr (kTableDma && u == 0) __builtin_amdgcn_s_barrier();  // every wave's quarter of the table landed
        f32x4 acc = first4<OP>(ring[wave][slot][0][lane], tab.w[0]);
#pragma unroll
        for (int k = 1; k < KC; ++k) acc = step4<OP>(acc, ring[wave][slot][k][lane], tab.w[k]);
        EpiIn in;
        in.a = ring[wave][slot][KC][lane];
        if constexpr (NIN > 1) in.b = ring[wave][slot][KC + 1][lane];
        if constexpr (NIN > 2) in.c = ring[wave][slot][KC + 2][lane];
        if constexpr (NIN > 3) in.d = ring[wave][slot][KC + 3][lane];
        const f32x4 a1[1] = {acc};
        f32x4 d1[1];
        fin_tile<FIN, 1>(d1, a1, fc);
        EpiIn o;
        if constexpr (epi_has_rare<EPI>() && EM == kEmFast) {
            uint32_t slow = 0;
            if constexpr ((EPI & 0xFF) == FEDAVG_EPI_ADAM) slow = C.bc2s.fast ? 0u : 1u;
            if constexpr ((EPI & 0xFF) == FEDAVG_EPI_NADAM) slow = C.bc2.fast ? 0u : 1u;
            if constexpr ((EPI & 0xFF) == FEDAVG_EPI_RADAM) slow = C.bc1.fast ? 0u : 1u;
            o = epi_compute<EPI, kEmFast>(E, C, d1[0], in, slow);
            if (__builtin_expect(wave_any(slow), 0)) {  // every lane: see wave_any
                uint32_t unused = 0;
                o = epi_compute<EPI, kEmElem>(E, C, d1[0], in, unused);
            }
        } else {
            uint32_t unused = 0;
            o = epi_compute<EPI, EM == kEmFast ? kEmElem : EM>(E, C, d1[0], in, unused);
        }
        if constexpr (u < N - S) {
            res[u] = o;
            wait_lgkmcnt0();  // the slot's reads have landed in VGPRs before its refill is issued
            issue(u + S, slot);
        } else {  // held in its slot (its inputs are consumed): entries 0 .. NOUT-1 = .a .. .d
            ring[wave][slot][0][lane] = o.a;
            if constexpr (NOUT > 1) ring[wave][slot][1][lane] = o.b;
            if constexpr (NOUT > 2) ring[wave][slot][2][lane] = o.c;
            if constexpr (NOUT > 3) ring[wave][slot][3][lane] = o.d;
        }
    });
    // the write burst
    static_for<0, N>([&](auto ic) {
        constexpr int u = decltype(ic)::value;
        const int64_t t = t_first + (int64_t)(u / CPT) * gridDim.x;
        const int64_t i = t * T4 + (int64_t)(u % CPT) * (W * 64) + threadIdx.x;
        if (t < t_end && i >= b4 && i < e4) {
            if constexpr (u < N - S) {
                epi_store<EPI>(E, i, res[u], out);
            } else {
                constexpr int slot = u % S;
                EpiIn o;
                o.a = ring[wave][slot][0][lane];
                if constexpr (NOUT > 1) o.b = ring[wave][slot][1][lane];
                if constexpr (NOUT > 2) o.c = ring[wave][slot][2][lane];
                if constexpr (NOUT > 3) o.d = ring[wave][slot][3][lane];
                epi_store<EPI>(E, i, o, out);
            }
        }
    });
}

// the LDS-DMA few-client form for this launch (1-3 client reads, no chained sum, no separate aggregate output):
// NIN operand streams by optimizer kind and flags; false when the form does not carry this kind / flag set
template <int OP, int FIN, int EPI, int KC, int NIN, int N = kEpiDmaUnits, bool TDMA = false, int EM = kEmFast,
          int W = 4>
inline hipError_t launch_epi_dma_n(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    constexpr int S = epi_dma_slots<EPI, KC + NIN, N, W>();
    constexpr int TPB = N * W / 16;  // tiles per block per launch
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, TPB, nl, L.variant & kVariantAnyOrder,
                          [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                              hipExtLaunchKernelGGL((fedavg_tiles_epi_dma_f32x4<OP, FIN, EPI, KC, NIN, S, N, TDMA, EM, W>),
                                                    dim3(nb), dim3(W * 64), 0, s, nullptr, nullptr, flags, L.tab,
                                                    L.tstride4, o, L.b4, L.e4, L.fin_val, E, t0, t_end);
                          });
}

// The product geometry per optimizer kind and client reads: waves per block W, units per wave per launch N, the RSQRTPS
// table by LDS-DMA.  Fused Adam with the AMD-host sqrt, 1e9 params, three interleaved rounds after a 3 s pre-warm, % of
// 8 TB/s, outputs bit-equal (profiles/r06/s6/ab_k*.jsonl; the round-5 per-tile form on the same box 64.5 / 67.7 /
// 67.4 at 1 / 2 / 3 clients):
//   W = 4 (one wave per SIMD), N = 32:  65.6 / 73.1 / 79.2      N = 28: 65.1 / 73.0 / 78.2
//   W = 8 (two per SIMD), N = 12 / 14 / 16 / 18:  74.1 / 74.1 / 73.3 / 73.4  |  73.6 / 74.0 / 74.3 / 74.0  |  74.2 / -- /
//   74.8 / 74.0 (1 / 2 / 3 clients);  N = 16 with the table staged by loads: 72.2 / 74.8 / 78.2
// One wave per SIMD issues a VALU op every 4 cycles; at 1-2 client reads Adam's ~400 instructions per wave-unit
// (4 elements per lane) then take about as long as the unit's 5 KiB of HBM traffic, and two waves per SIMD (issue every
// 2 cycles) win; at 3 reads the unit carries 6 KiB and one wave per SIMD with twice the ring slots (6 against 3) wins.
// N: 16 against 24 / 32 at W = 4 (profiles/r06/s3/, s4/): 68.7 / 72.8 / 74.9 % at 2 clients -- a launch's fixed cost
// (its start, its write burst's drain) over more units; at W = 8, 256 registers per wave hold 13 units' results.
// SGD (momentum) and ADD_BASE, the same sweep (profiles/r06/s8/ab_k*.jsonl, 1 / 2 / 3 clients): W = 4, N = 40: SGD 78.3 /
// 78.9 / 77.1, ADD_BASE 75.4 / 75.3 / 77.3 (N = 32: 77.4 / 78.9 / 77.5, 72.8 / 75.2 / 76.3; N = 16: 69.1 / 75.0 / 75.7,
// 67.3 / 71.3 / 72.3; W = 8, N = 16: 75.9 / 74.3 / 74.7, 72.9 / 75.0 / 74.3) -- lighter arithmetic, fewer result
// registers per unit (8 and 4): one wave per SIMD keeps up, and 40 units fit its registers.
// The other kinds (round 6, later): the ones with a sqrt and a division per element (NAdam, RAdam, Adagrad, RMSprop)
// start from Adam's geometry; Adamax and Rprop 4 waves x 24 units (three result streams per unit: 32 and 40 spill), ASGD
// SGD's.  With the AMD-host sqrt (the pool's hosts, the one measured) a same-process sweep of every geometry per kind
// (profiles/r06/s23/, A/B variant bits 9-11, 1 / 2 / 3 clients, % of 8 TB/s) moved:
//   RAdam 1-2 reads to 4 waves x 40 units, table by DMA: 75.2 / 73.0 -> 76.5 / 78.5 (3 reads stay: 79.6)
//   RMSprop (momentum) 1-2 reads, the same: 73.1 / 74.3 -> 75.2 / 78.3 (3 reads 78.5 against 79.4: kept)
//   Adagrad 2 reads, the same: 72.5 -> 74.1
//   NAdam to 8 waves x 16 units, table by DMA, at every read count: 73.6 / 74.0 / 73.5 -> 74.5 / 74.8 / 75.1
template <int EPI, int KC, int NIN>
struct EpiDmaGeom {
    static constexpr int KIND = EPI & 0xFF;
    static constexpr bool kAdam = KIND == FEDAVG_EPI_ADAM || KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM ||
                                  KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_RMSPROP;
    static constexpr bool kThree = KIND == FEDAVG_EPI_ADAMAX || KIND == FEDAVG_EPI_RPROP;  // light, three streams
    static constexpr bool kAmd = (EPI & kEpiSqrtMask) == kEpiTorchSqrtAmd;
    static constexpr bool kWide = kAmd && KC <= 2 &&
                                  (KIND == FEDAVG_EPI_RADAM || KIND == FEDAVG_EPI_RMSPROP ||
                                   (KIND == FEDAVG_EPI_ADAGRAD && KC == 2));
    static constexpr bool kNadam = kAmd && KIND == FEDAVG_EPI_NADAM;
    // four operand streams (Adam amsgrad, RMSprop centered with momentum): one wave per SIMD, 16 result registers
    // per unit -- 24 units (not swept; RMSprop at 3 reads 16: 24 spill with the IEEE sqrt)
    static constexpr bool kQuad = NIN == 4;
    static constexpr int W = kWide || kQuad ? 4 : kNadam ? 8 : kAdam && KC <= 2 ? 8 : 4;
    // (SGD with its momentum buffer at 3 reads holds 40 units only with 600+ bytes of scratch per lane: 32 there; Adamax
    // and Rprop hold three result streams per unit: 24)
    // (RMSprop with its momentum buffer, IEEE sqrt: 14 / 24 units at 2 / 3 reads, 16 / 32 spill)
    static constexpr bool kRmsMom = KIND == FEDAVG_EPI_RMSPROP && NIN == 3;
    static constexpr int N = kQuad ? (KIND == FEDAVG_EPI_RMSPROP && KC == 3 ? 16 : 24)
                             : kWide ? 40
                             : kNadam ? 16
                             : kThree ? 24
                             : !kAdam ? (KC == 3 ? 32 : 40)
                             : KC == 1 ? 14
                             : KC == 2 ? (kRmsMom ? 14 : 16)
                                       : (kRmsMom ? 24 : 32);
    static constexpr bool TDMA = kWide || kNadam || kQuad || (kAdam && KC != 2);
};

// A/B builds with -DFEDAVG_AB_FEW (torch-mode FIN_DIV, ADD_BASE / SGD, and Adam / NAdam / RAdam / Adagrad / RMSprop with
// the AMD-host sqrt): launch variant bits 9-11 = 1-7 pick another geometry
template <int OP, int FIN, int EPI, int KC, int NIN>
inline hipError_t launch_epi_dma_form(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    constexpr int KIND = EPI & 0xFF;
    constexpr bool kSqrtKind = KIND == FEDAVG_EPI_ADAM || KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM ||
                               KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_RMSPROP;
    if constexpr (kABFew && OP == FEDAVG_OP_TORCH && FIN == FEDAVG_FIN_DIV &&
                  ((kSqrtKind && (EPI & kEpiSqrtMask) == kEpiTorchSqrtAmd) || KIND == FEDAVG_EPI_SGD ||
                   KIND == FEDAVG_EPI_ADD_BASE)) {
        switch ((L.variant >> kVariantLoopShift) & 7) {
            case 1: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 16, false>(L, E, s, nl);
            case 2: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 32, true>(L, E, s, nl);
            case 3: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 12, true, kEmFast, 8>(L, E, s, nl);
            case 4: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 16, true, kEmFast, 8>(L, E, s, nl);
            case 5: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 16, false, kEmFast, 8>(L, E, s, nl);
            case 6: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 24, true>(L, E, s, nl);
            case 7: return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, 40, true>(L, E, s, nl);
            default: break;
        }
    }
    using Geom = EpiDmaGeom<EPI, KC, NIN>;
    return launch_epi_dma_n<OP, FIN, EPI, KC, NIN, Geom::N, Geom::TDMA, kEmFast, Geom::W>(L, E, s, nl);
}

template <int OP, int FIN, int EPI, int KC>
inline hipError_t launch_epi_dma_k(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    constexpr int KIND = EPI & 0xFF;
    const int nin = epi_dma_nin(E, KC);
    if constexpr (KIND == FEDAVG_EPI_ADD_BASE) {
        if (nin == 1) return launch_epi_dma_form<OP, FIN, EPI, KC, 1>(L, E, s, nl);
    } else if constexpr (KIND == FEDAVG_EPI_SGD) {
        if (nin == 1) return launch_epi_dma_form<OP, FIN, EPI, KC, 1>(L, E, s, nl);
        if (nin == 2) return launch_epi_dma_form<OP, FIN, EPI, KC, 2>(L, E, s, nl);
    } else if constexpr (KIND == FEDAVG_EPI_ADAM) {
        if (nin == 3) return launch_epi_dma_form<OP, FIN, EPI, KC, 3>(L, E, s, nl);
        if (nin == 4) return launch_epi_dma_form<OP, FIN, EPI, KC, 4>(L, E, s, nl);
    } else if constexpr (KIND == FEDAVG_EPI_NADAM || KIND == FEDAVG_EPI_RADAM || KIND == FEDAVG_EPI_ADAMAX ||
                         KIND == FEDAVG_EPI_RPROP) {
        if (nin == 3) return launch_epi_dma_form<OP, FIN, EPI, KC, 3>(L, E, s, nl);
    } else if constexpr (KIND == FEDAVG_EPI_ADAGRAD || KIND == FEDAVG_EPI_ASGD) {
        if (nin == 2) return launch_epi_dma_form<OP, FIN, EPI, KC, 2>(L, E, s, nl);
    } else if constexpr (KIND == FEDAVG_EPI_RMSPROP) {
        if (nin == 2) return launch_epi_dma_form<OP, FIN, EPI, KC, 2>(L, E, s, nl);
        if (nin == 3) return launch_epi_dma_form<OP, FIN, EPI, KC, 3>(L, E, s, nl);
        if (nin == 4) return launch_epi_dma_form<OP, FIN, EPI, KC, 4>(L, E, s, nl);
    }
    return hipErrorInvalidValue;
}

template <int OP, int FIN, int EPI>
inline hipError_t launch_epi_dma(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    switch (L.k) {
        case 1: return launch_epi_dma_k<OP, FIN, EPI, 1>(L, E, s, nl);
        case 2: return launch_epi_dma_k<OP, FIN, EPI, 2>(L, E, s, nl);
        case 3: return launch_epi_dma_k<OP, FIN, EPI, 3>(L, E, s, nl);
        default: return hipErrorInvalidValue;
    }
}

// A/B of the burst kernel's client loop (launch variant bits 9-11 = LOOP 1-4), instantiated for one configuration only:
// torch-mode FIN_DIV Adam with the AMD-host sqrt, no chained partial sum (bench.py --epilogue adam on the pool's boxes)
template <int OP, int FIN, bool ACC_IN, int EPI, int TPB_LDS, int LOOP>
inline hipError_t launch_epi_loop_ab(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    const f32x4* ai = reinterpret_cast<const f32x4*>(L.acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, kBurstTiles + TPB_LDS, nl,
                          L.variant & kVariantAnyOrder, [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                              hipExtLaunchKernelGGL(
                                  (fedavg_tiles_epi_burst_f32x4<OP, FIN, ACC_IN, EPI, kBurstTiles, TPB_LDS, LOOP>),
                                  dim3(nb), dim3(kBlock), 0, s, nullptr, nullptr, flags, L.tab, L.k, L.tstride4, ai, o,
                                  L.b4, L.e4, L.fin_val, E, t0, t_end);
                          });
}

template <int OP, int FIN, bool ACC_IN, int EPI, int TPB_LDS>
inline bool epi_loop_ab(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl, hipError_t* err) {
    if constexpr (OP == FEDAVG_OP_TORCH && FIN == FEDAVG_FIN_DIV && !ACC_IN && EPI == (FEDAVG_EPI_ADAM | kEpiTorchSqrtAmd)) {
        switch ((L.variant >> kVariantLoopShift) & 7) {
            case 1: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 1>(L, E, s, nl); return true;
            case 2: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 2>(L, E, s, nl); return true;
            case 3: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 3>(L, E, s, nl); return true;
            case 4: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 4>(L, E, s, nl); return true;
            case 5: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 5>(L, E, s, nl); return true;
            case 6: *err = launch_epi_loop_ab<OP, FIN, ACC_IN, EPI, TPB_LDS, 6>(L, E, s, nl); return true;
            default: return false;
        }
    }
    return false;
}

// one kernel instantiation per optimizer kind: K(EPI) launches the per-tile (PRE) or the burst form.  Product builds
// (fedavg_internal.h kAB): the burst form with 4 (two blocks per CU) or 9 (one block per CU) LDS-held tiles without a
// chained sum, the pipelined per-tile form; A/B builds also the register-only burst form, the burst form over a
// chained sum, the unpipelined per-tile form and the client-loop shapes.
template <int OP, int FIN, int EPI, int TPB, int TPB_LDS, int XS>
inline hipError_t launch_epi_split(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, TPB + TPB_LDS, nl,
                          L.variant & kVariantAnyOrder, [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                              hipExtLaunchKernelGGL((fedavg_tiles_epi_split_f32x4<OP, FIN, EPI, TPB, TPB_LDS, XS>),
                                                    dim3(nb), dim3(2 * kBlock), 0, s, nullptr, nullptr, flags, L.tab,
                                                    L.k, L.tstride4, o, L.b4, L.e4, L.fin_val, E, t0, t_end);
                          });
}

// A/B builds with -DFEDAVG_AB_FEW, torch-mode FIN_DIV Adam with the AMD-host sqrt, 4+ reads without a chained sum, one
// block per CU: launch variant bits 9-11 = 1-5 run the split-epilogue form with (register-held, LDS-held, LDS-held
// finished by waves 0-3) = (4, 9, 4), (4, 9, 5), (3, 9, 4), (4, 9, 3), (5, 9, 3)
template <int OP, int FIN, int EPI>
inline bool epi_split_ab(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl, hipError_t* err) {
    if constexpr (kABFew && OP == FEDAVG_OP_TORCH && FIN == FEDAVG_FIN_DIV && EPI == (FEDAVG_EPI_ADAM | kEpiTorchSqrtAmd)) {
        switch ((L.variant >> kVariantLoopShift) & 7) {
            case 1: *err = launch_epi_split<OP, FIN, EPI, 4, 9, 4>(L, E, s, nl); return true;
            case 2: *err = launch_epi_split<OP, FIN, EPI, 4, 9, 5>(L, E, s, nl); return true;
            case 3: *err = launch_epi_split<OP, FIN, EPI, 3, 9, 4>(L, E, s, nl); return true;
            case 4: *err = launch_epi_split<OP, FIN, EPI, 4, 9, 3>(L, E, s, nl); return true;
            case 5: *err = launch_epi_split<OP, FIN, EPI, 5, 9, 3>(L, E, s, nl); return true;
            default: break;
        }
    }
    return false;
}

template <int OP, int FIN, bool ACC_IN, int EPI>
inline hipError_t launch_epi_k(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    const f32x4* ai = reinterpret_cast<const f32x4*>(L.acc_in);
    f32x4* o = reinterpret_cast<f32x4*>(L.out);
    if constexpr (!ACC_IN) {
        if (L.variant & kVariantEpiDma) return launch_epi_dma<OP, FIN, EPI>(L, E, s, nl);
        if (!(L.variant & (kVariantTileStores | kVariantEpiPrefetch)) && (L.variant & kVariantWideLds)) {
            if constexpr (kABFew && !kAB) {
                hipError_t ab_err = hipSuccess;
                if (epi_split_ab<OP, FIN, EPI>(L, E, s, nl, &ab_err)) return ab_err;
            }
            // Adam at one block per CU (64+ clients: config 5): the split-epilogue form (round 6), unless the public
            // variant asks for the round-5 burst form (kVariantEpiNoSplit)
            if constexpr ((EPI & 0xFF) == FEDAVG_EPI_ADAM) {
                if (!(L.variant & kVariantEpiNoSplit)) return launch_epi_split<OP, FIN, EPI, 4, 9, 4>(L, E, s, nl);
            }
        }
    }
    if constexpr (kAB || !ACC_IN) {
        if (!(L.variant & (kVariantTileStores | kVariantEpiPrefetch))) {  // burst: one launch per grid x TPB tiles
            if constexpr (kAB) {
                hipError_t ab_err = hipSuccess;
                if ((L.variant & kVariantWideLds) &&
                    epi_loop_ab<OP, FIN, ACC_IN, EPI, kBurstEpiLdsTilesWide>(L, E, s, nl, &ab_err))
                    return ab_err;
                if (!(L.variant & (kVariantWideLds | kVariantRegisterTiles)) &&
                    epi_loop_ab<OP, FIN, ACC_IN, EPI, kBurstLdsTiles>(L, E, s, nl, &ab_err))
                    return ab_err;
            }
            if (L.variant & kVariantWideLds)  // one block per CU: 9 more tiles with d in LDS (144 KiB)
                return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid,
                                      kBurstTiles + kBurstEpiLdsTilesWide, nl, L.variant & kVariantAnyOrder,
                                      [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                                          hipExtLaunchKernelGGL(
                                              (fedavg_tiles_epi_burst_f32x4<OP, FIN, ACC_IN, EPI, kBurstTiles,
                                                                            kBurstEpiLdsTilesWide>),
                                              dim3(nb), dim3(kBlock), 0, s, nullptr, nullptr, flags, L.tab, L.k,
                                              L.tstride4, ai, o, L.b4, L.e4, L.fin_val, E, t0, t_end);
                                      });
            if (!kAB || !(L.variant & kVariantRegisterTiles))  // default: 4 more tiles per block with d held in LDS
                return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, kBurstTiles + kBurstLdsTiles,
                                      nl, L.variant & kVariantAnyOrder,
                                      [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                                          hipExtLaunchKernelGGL(
                                              (fedavg_tiles_epi_burst_f32x4<OP, FIN, ACC_IN, EPI, kBurstTiles,
                                                                            kBurstLdsTiles>),
                                              dim3(nb), dim3(kBlock), 0, s, nullptr, nullptr, flags, L.tab, L.k,
                                              L.tstride4, ai, o, L.b4, L.e4, L.fin_val, E, t0, t_end);
                                      });
            if constexpr (kAB)
                return burst_launches(L.b4 / L.tile4, (L.e4 - 1) / L.tile4 + 1, L.grid, kBurstTiles, nl,
                                      L.variant & kVariantAnyOrder, [&](int nb, int64_t t0, int64_t t_end, uint32_t flags) {
                                          hipExtLaunchKernelGGL(
                                              (fedavg_tiles_epi_burst_f32x4<OP, FIN, ACC_IN, EPI, kBurstTiles>), dim3(nb),
                                              dim3(kBlock), 0, s, nullptr, nullptr, flags, L.tab, L.k, L.tstride4, ai, o,
                                              L.b4, L.e4, L.fin_val, E, t0, t_end);
                                      });
        }
    }
    if (kAB && !(L.variant & kVariantEpiPrefetch)) {
        if constexpr (kAB)
            hipLaunchKernelGGL((fedavg_tiles_epi_f32x4<OP, FIN, ACC_IN, EPI, false>), dim3(L.grid), dim3(kBlock), 0, s,
                               L.tab, L.k, L.tstride4, ai, o, L.b4, L.e4, L.fin_val, E);
    } else {
        hipLaunchKernelGGL((fedavg_tiles_epi_f32x4<OP, FIN, ACC_IN, EPI, true>), dim3(L.grid), dim3(kBlock), 0, s, L.tab,
                           L.k, L.tstride4, ai, o, L.b4, L.e4, L.fin_val, E);
    }
    if (nl) ++*nl;
    return hipGetLastError();
}

// the step's sqrt (EpiParams.torch_sqrt, FEDAVG_SQRT_*) as a compile-time epilogue variant
template <int OP, int FIN, bool ACC_IN, int KIND>
inline hipError_t sqrt_mode(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    if (E.torch_sqrt == FEDAVG_SQRT_TORCH_AVX512) return launch_epi_k<OP, FIN, ACC_IN, KIND | kEpiTorchSqrt>(L, E, s, nl);
    if (E.torch_sqrt == FEDAVG_SQRT_TORCH_AMD) return launch_epi_k<OP, FIN, ACC_IN, KIND | kEpiTorchSqrtAmd>(L, E, s, nl);
    return launch_epi_k<OP, FIN, ACC_IN, KIND>(L, E, s, nl);
}

// KINDS: the optimizer kinds this translation unit carries (bit k = kind k; the build splits each (mode,
// finalisation) pair over two units, fedavg_epi_inst.hip); a kind outside it is refused, never run in another form
template <int OP, int FIN, bool ACC_IN, unsigned KINDS = ~0u>
inline hipError_t launch_epi_a(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
#define FEDAVG_EPI_CASE(KIND, CALL)                                                                                    \
    case KIND:                                                                                                       \
        if constexpr ((KINDS >> KIND) & 1u) return CALL<OP, FIN, ACC_IN, KIND>(L, E, s, nl);                         \
        else return hipErrorNotSupported;
    switch (E.kind) {
        FEDAVG_EPI_CASE(FEDAVG_EPI_ADD_BASE, launch_epi_k)
        FEDAVG_EPI_CASE(FEDAVG_EPI_SGD, launch_epi_k)
        FEDAVG_EPI_CASE(FEDAVG_EPI_ADAM, sqrt_mode)
        FEDAVG_EPI_CASE(FEDAVG_EPI_ADAGRAD, sqrt_mode)
        FEDAVG_EPI_CASE(FEDAVG_EPI_RMSPROP, sqrt_mode)
        FEDAVG_EPI_CASE(FEDAVG_EPI_ADAMAX, launch_epi_k)
        FEDAVG_EPI_CASE(FEDAVG_EPI_NADAM, sqrt_mode)
        FEDAVG_EPI_CASE(FEDAVG_EPI_RADAM, sqrt_mode)
        FEDAVG_EPI_CASE(FEDAVG_EPI_RPROP, launch_epi_k)
        FEDAVG_EPI_CASE(FEDAVG_EPI_ASGD, launch_epi_k)
        default:
            return hipErrorInvalidValue;
    }
#undef FEDAVG_EPI_CASE
}

// one (mode, finalisation) pair's entry; product builds carry no chained-sum forms here (launch_epi_step has the
// server step's, fedavg_internal.h epi_direct)
template <int OP, int FIN, unsigned KINDS = ~0u>
inline hipError_t launch_epi_f(const TileLaunch& L, const EpiParams& E, hipStream_t s, uint64_t* nl) {
    if constexpr (kAB)
        return L.acc_in ? launch_epi_a<OP, FIN, true, KINDS>(L, E, s, nl) : launch_epi_a<OP, FIN, false, KINDS>(L, E, s, nl);
    return L.acc_in ? hipErrorNotSupported : launch_epi_a<OP, FIN, false, KINDS>(L, E, s, nl);
}

}  // namespace fedavg
