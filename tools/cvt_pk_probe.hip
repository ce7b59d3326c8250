// Exhaustive check (TEST TOOL): gfx950's packed fp32 -> 16-bit conversions v_cvt_pk_bf16_f32 and v_cvt_pk_f16_f32,
// which fedavg_narrow.hip's pack2 uses for two elements at once, against the per-element roundings the other 16-bit
// kernels use (bits16): c10::BFloat16's round_to_nearest_even recipe (as tools/bf16_cvt_probe.hip) and
// v_cvt_f16_f32 ((_Float16)x).  Every one of the 2^32 fp32 bit patterns goes through both halves of the packed
// instruction (low half x with a different value in the high half, and the reverse); non-NaN results must be equal
// bit for bit, NaN inputs must give some NaN.  Built with the product's flags (denormals kept).
//
//   hipcc -O3 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 tools/cvt_pk_probe.hip -o tools/cvt_pk_probe
//   ./tools/cvt_pk_probe            -> one JSON line; exit status 0 iff no mismatch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint16_t c10_rne(uint32_t u) {
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ uint16_t f16_one(float x) {
    asm volatile("" : "+v"(x));
    const _Float16 h = (_Float16)x;
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
}

__device__ __forceinline__ bool nan32(uint32_t u) { return (u & 0x7fffffffu) > 0x7f800000u; }

// counts: [0] bf16 non-NaN mismatches, [1] bf16 NaN -> non-NaN, [2] f16 non-NaN mismatches, [3] f16 NaN -> non-NaN
__global__ void probe(unsigned long long* counts, uint32_t* first_bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long c[4] = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const uint32_t u = (uint32_t)i, v = u ^ 0x9e3779b9u;
        const float x = __uint_as_float(u), y = __uint_as_float(v);
        uint32_t b0, b1, h0, h1;
        asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(b0) : "v"(x), "v"(y));
        asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(b1) : "v"(y), "v"(x));
        asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h0) : "v"(x), "v"(y));
        asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h1) : "v"(y), "v"(x));
        const uint16_t bx[2] = {(uint16_t)(b0 & 0xffffu), (uint16_t)(b1 >> 16)};
        const uint16_t hx[2] = {(uint16_t)(h0 & 0xffffu), (uint16_t)(h1 >> 16)};
        const uint16_t bref = c10_rne(u), href = f16_one(x);
        for (int p = 0; p < 2; ++p) {
            if (nan32(u)) {
                c[1] += (bx[p] & 0x7fffu) <= 0x7f80u;
                c[3] += (hx[p] & 0x7fffu) <= 0x7c00u;
            } else {
                if (bx[p] != bref) {
                    ++c[0];
                    atomicCAS(first_bad, 0xffffffffu, u);
                }
                if (hx[p] != href) {
                    ++c[2];
                    atomicCAS(first_bad, 0xffffffffu, u);
                }
            }
        }
    }
    for (int k = 0; k < 4; ++k) atomicAdd(&counts[k], c[k]);
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
    CHECK(hipMalloc(&d_counts, 4 * sizeof(unsigned long long)));
    CHECK(hipMalloc(&d_first, sizeof(uint32_t)));
    CHECK(hipMemset(d_counts, 0, 4 * sizeof(unsigned long long)));
    CHECK(hipMemset(d_first, 0xff, sizeof(uint32_t)));
    hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, d_counts, d_first);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long c[4];
    uint32_t first;
    CHECK(hipMemcpy(c, d_counts, sizeof(c), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&first, d_first, sizeof(first), hipMemcpyDeviceToHost));
    printf("{\"tool\": \"cvt_pk_probe\", \"inputs\": 4294967296, \"positions\": 2, \"bf16_non_nan_mismatches\": %llu, "
           "\"bf16_nan_to_non_nan\": %llu, \"f16_non_nan_mismatches\": %llu, \"f16_nan_to_non_nan\": %llu, "
           "\"first_mismatch\": \"0x%08x\"}\n",
           c[0], c[1], c[2], c[3], first);
    (void)hipFree(d_counts);
    (void)hipFree(d_first);
    return (c[0] == 0 && c[1] == 0 && c[2] == 0 && c[3] == 0) ? 0 : 1;
}
