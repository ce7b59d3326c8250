// Exhaustive check (TEST TOOL): gfx950's hardware fp32 -> bfloat16 conversion (v_cvt_pk_bf16_f32, what
// `(__bf16)x` compiles to) against c10::BFloat16's round_to_nearest_even bit recipe
// (c10/util/BFloat16.h: NaN -> 0x7FC0, else (u + 0x7FFF + ((u >> 16) & 1)) >> 16) for all 2^32 fp32 bit
// patterns.  fedavg_narrow.hip relies on the two agreeing for every non-NaN input; NaN inputs must map to
// some NaN (payloads are not part of the contract).  Built with the product's flags (denormals kept).
//
//   hipcc -O3 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 tools/bf16_cvt_probe.hip -o tools/bf16_cvt_probe
//   ./tools/bf16_cvt_probe            -> one JSON line; exit status 0 iff no mismatch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint16_t c10_rne(uint32_t u) {
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__global__ void probe(unsigned long long* counts, uint32_t* first_bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long bad = 0, nan_ok = 0, nan_bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const uint32_t u = (uint32_t)i;
        float x = __uint_as_float(u);
        asm volatile("" : "+v"(x));
        const __bf16 h = (__bf16)x;
        uint16_t hw;
        __builtin_memcpy(&hw, &h, 2);
        if ((u & 0x7fffffffu) > 0x7f800000u) {
            const bool is_nan = (hw & 0x7fffu) > 0x7f80u;
            nan_ok += is_nan;
            nan_bad += !is_nan;
        } else if (hw != c10_rne(u)) {
            ++bad;
            atomicCAS(first_bad, 0xffffffffu, u);
        }
    }
    atomicAdd(&counts[0], bad);
    atomicAdd(&counts[1], nan_ok);
    atomicAdd(&counts[2], nan_bad);
}

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)

int main() {
    unsigned long long* d_counts;
    uint32_t* d_first;
    CHECK(hipMalloc(&d_counts, 3 * sizeof(unsigned long long)));
    CHECK(hipMalloc(&d_first, sizeof(uint32_t)));
    CHECK(hipMemset(d_counts, 0, 3 * sizeof(unsigned long long)));
    CHECK(hipMemset(d_first, 0xff, sizeof(uint32_t)));
    hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, d_counts, d_first);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long c[3];
    uint32_t first;
    CHECK(hipMemcpy(c, d_counts, sizeof(c), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&first, d_first, sizeof(first), hipMemcpyDeviceToHost));
    printf("{\"tool\": \"bf16_cvt_probe\", \"inputs\": 4294967296, \"non_nan_mismatches\": %llu, "
           "\"nan_inputs_to_nan\": %llu, \"nan_inputs_to_non_nan\": %llu, \"first_mismatch\": \"0x%08x\"}\n",
           c[0], c[1], c[2], first);
    (void)hipFree(d_counts);
    (void)hipFree(d_first);
    return (c[0] == 0 && c[2] == 0) ? 0 : 1;
}
