/* sqrt_probe2.c -- diagnostic (not product code): which sequence does torch CPU's fp32 sqrt run on THIS host?
 * (tools/sqrt_probe.c restates the AVX-512 path of MKL vsSqrt; MKL dispatches by CPU, so another host -- e.g. the
 * GPU pool's AMD EPYC -- may run another code path.)  Reads the probe inputs (uint32 bit patterns) and torch's
 * results, and counts mismatches of candidate sequences:
 *   est  = rsqrt14 (VRSQRT14PS) | rsqrtps (VRSQRTPS, 12-bit, the AVX2 estimate)
 *   nr1  s = x*y; r = fma(-s, s, x); sqrt = fma(r, 0.5*y, s)            (one Newton step on the root)
 *   nr1n s = x*y; h = 0.5*y; sqrt = s + (x - s*s)*h without fma
 *   nry  y' = y * (1.5 - 0.5*x*y*y) [fma forms], then nr1 with y'         (Newton on the reciprocal root first)
 *   nry2 y' as in nry; sqrt = x * y'
 * and writes, for the estimate(s) that depend on the top k mantissa bits only, k.
 *   sqrt_probe2 IN_X.bin IN_TORCH.bin       prints one JSON line */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static uint32_t b_of(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }

static void est16(int which, const float* x, float* y) {
    if (which == 0) _mm512_storeu_ps(y, _mm512_rsqrt14_ps(_mm512_loadu_ps(x)));
    else {
        _mm256_storeu_ps(y, _mm256_rsqrt_ps(_mm256_loadu_ps(x)));
        _mm256_storeu_ps(y + 8, _mm256_rsqrt_ps(_mm256_loadu_ps(x + 8)));
    }
}

static float cand(int c, float x, float y) {
    if (!(x > 0.0f) || isinf(x)) return sqrtf(x);
    const float h = 0.5f * y;
    switch (c) {
        case 0: { const float s = x * y; const float r = fmaf(-s, s, x); return fmaf(r, h, s); }
        case 1: { const float s = x * y; const float r = x - s * s; return s + r * h; }
        case 2: {
            const float t = fmaf(-(x * y), y, 1.0f);            /* 1 - x y^2 */
            const float y1 = fmaf(0.5f * y, t, y);              /* y + y/2 (1 - x y^2) */
            const float s = x * y1; const float r = fmaf(-s, s, x); return fmaf(r, 0.5f * y1, s);
        }
        case 3: {
            const float t = fmaf(-(x * y), y, 1.0f);
            const float y1 = fmaf(0.5f * y, t, y);
            return x * y1;
        }
    }
    return NAN;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    fseek(f, 0, SEEK_END);
    const size_t n = (size_t)ftell(f) / 4;
    fseek(f, 0, SEEK_SET);
    uint32_t* xb = malloc(n * 4);
    float* t = malloc(n * 4);
    if (fread(xb, 4, n, f) != n) return 4;
    fclose(f);
    f = fopen(argv[2], "rb");
    if (!f || fread(t, 4, n, f) != n) return 5;
    fclose(f);
    size_t mism[2][4] = {{0}};
    size_t mism_scaled[2][4] = {{0}};
    for (size_t i = 0; i < n; i += 16) {
        float xv[16], yv[2][16], xs[16], ys[2][16];
        const size_t c = n - i < 16 ? n - i : 16;
        for (size_t j = 0; j < 16; ++j) {
            xv[j] = f_of(xb[j < c ? i + j : i]);
            xs[j] = xv[j] < 0x1p-96f ? xv[j] * 0x1p64f : xv[j];
        }
        for (int e = 0; e < 2; ++e) { est16(e, xv, yv[e]); est16(e, xs, ys[e]); }
        for (size_t j = 0; j < c; ++j) {
            const uint32_t tb = b_of(t[i + j]);
            const int tnan = t[i + j] != t[i + j];
            for (int e = 0; e < 2; ++e)
                for (int k = 0; k < 4; ++k) {
                    const float r = cand(k, xv[j], yv[e][j]);
                    if (!((r != r && tnan) || b_of(r) == tb)) ++mism[e][k];
                    const int tiny = xv[j] < 0x1p-96f && xv[j] > 0.0f;
                    float rs = cand(k, xs[j], ys[e][j]);
                    if (tiny) rs *= 0x1p-32f;
                    if (!((rs != rs && tnan) || b_of(rs) == tb)) ++mism_scaled[e][k];
                }
        }
    }
    /* estimate structure: over [1, 4), the smallest k such that the estimate depends on the top k mantissa bits */
    int kdep[2] = {23, 23};
    for (int e = 0; e < 2; ++e) {
        for (int k = 8; k <= 23; ++k) {
            int ok = 1;
            for (int p = 0; p < 2 && ok; ++p)
                for (uint32_t m = 1; m < (1u << 23) && ok; m += 16) {
                    float xv[16], yv[16], x0[16], y0[16];
                    for (int j = 0; j < 16; ++j) {
                        xv[j] = f_of(((uint32_t)(p + 127) << 23) | (m + j < (1u << 23) ? m + j : m));
                        uint32_t mm = ((m + j < (1u << 23) ? m + j : m) >> (23 - k)) << (23 - k);
                        x0[j] = f_of(((uint32_t)(p + 127) << 23) | (mm ? mm : 1));
                    }
                    est16(e, xv, yv);
                    est16(e, x0, y0);
                    for (int j = 0; j < 16; ++j)
                        if (b_of(yv[j]) != b_of(y0[j])) { ok = 0; break; }
                }
            if (ok) { kdep[e] = k; break; }
        }
    }
    printf("{\"values\": %zu, \"rsqrt14\": {\"nr1\": %zu, \"nr1_nofma\": %zu, \"nry\": %zu, \"nry_mul\": %zu}, "
           "\"rsqrtps\": {\"nr1\": %zu, \"nr1_nofma\": %zu, \"nry\": %zu, \"nry_mul\": %zu}, "
           "\"rsqrt14_scaled\": {\"nr1\": %zu, \"nr1_nofma\": %zu, \"nry\": %zu, \"nry_mul\": %zu}, "
           "\"rsqrtps_scaled\": {\"nr1\": %zu, \"nr1_nofma\": %zu, \"nry\": %zu, \"nry_mul\": %zu}, "
           "\"estimate_top_bits\": {\"rsqrt14\": %d, \"rsqrtps\": %d}}\n",
           n, mism[0][0], mism[0][1], mism[0][2], mism[0][3], mism[1][0], mism[1][1], mism[1][2], mism[1][3],
           mism_scaled[0][0], mism_scaled[0][1], mism_scaled[0][2], mism_scaled[0][3],
           mism_scaled[1][0], mism_scaled[1][1], mism_scaled[1][2], mism_scaled[1][3], kdep[0], kdep[1]);
    return 0;
}
