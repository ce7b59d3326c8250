/* rsqrtps_dump.c -- diagnostic (not product code): this CPU's RSQRTPS and RCPPS estimates (the approximate SSE
 * instructions inside MKL's SSE4.2 / AVX vsSqrt kernels, whose bits differ between CPU vendors) over every fp32 in
 * [1, 4), written as run-length pairs (first input bit pattern of a run, estimate bits) so a whole binade pair
 * fits in a few hundred KiB.
 *   rsqrtps_dump OUT_RSQRT.bin OUT_RCP.bin       (gcc -O2 -msse2 tools/rsqrtps_dump.c -o rsqrtps_dump) */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static int dump(const char* path, int rcp) {
    FILE* f = fopen(path, "wb");
    if (!f) return 1;
    uint32_t prev = 0xFFFFFFFFu, runs = 0;
    for (uint32_t b = 0x3F800000u; b < 0x40800000u; b += 4) {
        float x[4];
        uint32_t in[4] = {b, b + 1, b + 2, b + 3}, out[4];
        memcpy(x, in, 16);
        __m128 v = _mm_loadu_ps(x);
        __m128 r = rcp ? _mm_rcp_ps(v) : _mm_rsqrt_ps(v);
        memcpy(out, &r, 16);
        for (int j = 0; j < 4; ++j) {
            if (out[j] != prev) {
                uint32_t pair[2] = {in[j], out[j]};
                fwrite(pair, 4, 2, f);
                prev = out[j];
                ++runs;
            }
        }
    }
    fclose(f);
    printf("{\"file\": \"%s\", \"runs\": %u}\n", path, runs);
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: rsqrtps_dump OUT_RSQRT.bin OUT_RCP.bin\n");
        return 2;
    }
    return dump(argv[1], 0) || dump(argv[2], 1);
}
