/* sqrt_probe.c -- diagnostic (not product code): torch CPU's fp32 sqrt, restated.
 *
 * torch 2.10 CPU computes Tensor.sqrt of a contiguous fp32 tensor with MKL VML's vsSqrt (ATen vml.h,
 * IMPLEMENT_VML_MKL(sqrt, Sqrt), VML_HA).  On the AVX-512 path that is NOT the correctly rounded vsqrtps but
 * one Newton step from the CPU's reciprocal-square-root estimate (measured bit-exact in the container over every
 * mantissa of two binades, tools/sqrt_probe.py):
 *     y = rsqrt14(x);  s = x * y;  r = fma(-s, s, x);  sqrt(x) = fma(r, 0.5 * y, s)
 * with inputs below 2^-96 computed at x * 2^64 and scaled back by 2^-32
 * so about 0.5 % of results sit 1 ulp below the correctly rounded one (Adam's exp_avg_sq.sqrt(), torch
 * optim/adam.py:545, and every other torch optimizer's sqrt).
 * The estimate (VRSQRT14PS) depends on the exponent parity and the top 15 mantissa bits only (measured),
 * except x = 4^k exactly (a power of four gives its exact reciprocal root); this program writes that
 * 2 x 2^15 table and checks the table-driven restatement against the instruction itself.
 *
 *   sqrt_probe table OUT.bin            65536 uint32 estimates: parity 0 (x in [1, 2)), then parity 1 ([2, 4))
 *   sqrt_probe check TABLE.bin OUT.bin  restated sqrt of every x in the probe set (see probe_set) with
 *                                       TABLE.bin, written to OUT.bin; prints mismatches against the same
 *                                       restatement with this CPU's own instruction
 */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static uint32_t b_of(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }

/* VRSQRT14PS restated from the table (finite x > 0; 0 -> inf, inf -> 0, NaN / negative -> NaN) */
static float rsqrt14_table(const uint32_t* tab, float x) {
    uint32_t b = b_of(x);
    if (x != x || (b >> 31)) return x != x ? x : (x == 0.0f ? -INFINITY : NAN);
    if (x == 0.0f) return INFINITY;
    if (isinf(x)) return 0.0f;
    int e = (int)((b >> 23) & 0xFF) - 127;
    uint32_t m = b & 0x7FFFFF;
    if ((b >> 23) == 0) {  /* subnormal: normalise */
        int sh = __builtin_clz(m) - 8;
        m = (m << sh) & 0x7FFFFF;
        e = -126 - sh;
    }
    const int p = e & 1;
    const int k = (e - p) / 2;  /* x = 4^k * 2^p * 1.m */
    float y = (p == 0 && m == 0) ? 1.0f : f_of(tab[p * 32768 + (m >> 8)]);
    return ldexpf(y, -k);
}

static float sqrt_restated(float x, float y) {
    if (!(x > 0.0f) || isinf(x)) return sqrtf(x);  /* 0, -0, inf, NaN, negative: vsSqrt's special values */
    const float s = x * y;
    const float r = fmaf(-s, s, x);
    return fmaf(r, 0.5f * y, s);
}

/* probe set: every mantissa of [1, 2) and [2, 4), every subnormal, 1 mantissa in 61 of every other binade,
 * powers of four, specials */
static size_t probe_set(uint32_t* out) {
    size_t n = 0;
    for (uint32_t e = 127; e <= 128; ++e)
        for (uint32_t m = 0; m < (1u << 23); ++m) out[n++] = (e << 23) | m;
    for (uint32_t m = 1; m < (1u << 23); ++m) out[n++] = m;
    for (uint32_t e = 1; e < 255; ++e) {
        if (e == 127 || e == 128) continue;
        for (uint32_t m = e % 61; m < (1u << 23); m += 61) out[n++] = (e << 23) | m;
    }
    const uint32_t sp[] = {0x00000000u, 0x80000000u, 0x7F800000u, 0xFF800000u, 0x7FC00000u, 0xBF800000u, 0x7F7FFFFFu,
                           0x00000001u, 0x3F800000u, 0x40800000u, 0x3E800000u, 0x00800000u};
    for (size_t i = 0; i < sizeof(sp) / 4; ++i) out[n++] = sp[i];
    return n;
}

int main(int argc, char** argv) {
    if (argc >= 3 && !strcmp(argv[1], "table")) {
        FILE* f = fopen(argv[2], "wb");
        if (!f) return 3;
        for (int p = 0; p < 2; ++p)
            for (uint32_t i = 0; i < (1u << 15); i += 16) {
                float xs[16], ys[16];
                for (int j = 0; j < 16; ++j) xs[j] = f_of(((uint32_t)(p + 127) << 23) | ((i + j) << 8) | 0x80u);
                _mm512_storeu_ps(ys, _mm512_rsqrt14_ps(_mm512_loadu_ps(xs)));
                if (fwrite(ys, 4, 16, f) != 16) return 4;
            }
        fclose(f);
        return 0;
    }
    if (argc >= 4 && !strcmp(argv[1], "check")) {
        uint32_t* tab = malloc(65536 * 4);
        FILE* f = fopen(argv[2], "rb");
        if (!f || fread(tab, 4, 65536, f) != 65536) return 5;
        fclose(f);
        uint32_t* xs = malloc((size_t)64 << 22);  /* 64 Mi values */
        const size_t n = probe_set(xs);
        float* res = malloc(n * 4);
        size_t est_mism = 0, sqrt_mism = 0;
        for (size_t i = 0; i < n; i += 16) {
            float xv[16], yv[16];
            const size_t c = n - i < 16 ? n - i : 16;
            float xo[16];
            for (size_t j = 0; j < 16; ++j) {
                xo[j] = f_of(xs[j < c ? i + j : i]);
                xv[j] = (xo[j] > 0.0f && xo[j] < 0x1p-96f) ? xo[j] * 0x1p64f : xo[j];  /* the tiny-input scaling */
            }
            _mm512_storeu_ps(yv, _mm512_rsqrt14_ps(_mm512_loadu_ps(xv)));
            for (size_t j = 0; j < c; ++j) {
                const float yt = rsqrt14_table(tab, xv[j]);
                if (b_of(yt) != b_of(yv[j]) && xv[j] > 0.0f && !isinf(xv[j])) ++est_mism;
                const float sc = xv[j] != xo[j] ? 0x1p-32f : 1.0f;
                const float a = sqrt_restated(xv[j], yt) * sc, b = sqrt_restated(xv[j], yv[j]) * sc;
                if (b_of(a) != b_of(b)) ++sqrt_mism;
                res[i + j] = a;
            }
        }
        FILE* o = fopen(argv[3], "wb");
        if (!o || fwrite(res, 4, n, o) != n) return 6;
        fclose(o);
        printf("{\"probe_values\": %zu, \"estimate_mismatches_vs_instruction\": %zu, "
               "\"sqrt_mismatches_vs_instruction\": %zu}\n", n, est_mism, sqrt_mism);
        return 0;
    }
    fprintf(stderr, "usage: sqrt_probe table OUT | check TABLE OUT\n");
    return 2;
}
