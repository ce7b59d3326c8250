/* div_const_check.c -- test helper (not product code): the constant-divisor quotient of the plain kernels' FIN_DIV
 * (nvflare_amd/csrc/fedavg_tiles.h div_const: r = RN(1/b); q = RN(a r); e = fma(-q, b, a); RN(q + e r)) against the
 * IEEE quotient a / b, on the host, for every dividend significand of [1, 2) and each divisor given on the command
 * line (scaled into [1, 2): away from underflow and overflow only the significands matter).  Prints the number of
 * mismatches per divisor.   gcc -O2 -ffp-contract=off -mfma tests/div_const_check.c -o div_const_check -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float from_bits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t to_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main(int argc, char** argv) {
    long total = 0;
    for (int i = 1; i < argc; ++i) {
        const float b0 = strtof(argv[i], NULL);
        const float b = from_bits((to_bits(b0) & 0x7FFFFFu) | 0x3F800000u);
        const float r = 1.0f / b;
        long bad = 0;
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            const float a = from_bits(0x3F800000u | m);
            const float q = a * r;
            const float e = fmaf(-q, b, a);
            const float q1 = fmaf(e, r, q);
            const float ref = a / b;
            bad += to_bits(q1) != to_bits(ref);
        }
        printf("%.9g %ld\n", (double)b, bad);
        total += bad;
    }
    return total ? 1 : 0;
}
