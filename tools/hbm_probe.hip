// hbm_probe.hip -- diagnostic only (not part of the product library): the achievable HBM read and
// copy bandwidth on this device, as the ceiling the FedAvg kernel's roofline fraction is read against.
//   read:  every lane streams float4 loads over a buffer and folds them into one value per lane
//          (written once, so the loads stay live);
//   copy:  float4 copy kernel (the guide's 6.29 TB/s reference measurement shape).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hbm_probe.hip -o tools/build/libhbm_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) probe_read(const f32x4* __restrict__ src, int64_t n4, f32x4* __restrict__ sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
        f32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += v[u];
    }
    for (; i < n4; i += stride) acc += src[i];
    sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) probe_copy(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
}

extern "C" {
// mode 0: read (nt), 1: read (temporal), 2: copy kernel (dst = second half), 3: hipMemcpyAsync D2D
int probe_run(int mode, void* buf, size_t bytes, int blocks, int reps, float* ms_out) {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f32x4* sink = nullptr;
    if (hipMalloc(&sink, (size_t)blocks * 256 * sizeof(f32x4)) != hipSuccess) return 2;
    const int64_t n4 = (int64_t)(bytes / 16);
    auto launch = [&]() {
        switch (mode) {
            case 0:
                hipLaunchKernelGGL((probe_read<8, true>), dim3(blocks), dim3(256), 0, s, (const f32x4*)buf, n4, sink);
                break;
            case 1:
                hipLaunchKernelGGL((probe_read<8, false>), dim3(blocks), dim3(256), 0, s, (const f32x4*)buf, n4, sink);
                break;
            case 2:
                hipLaunchKernelGGL(probe_copy, dim3(blocks), dim3(256), 0, s, (const f32x4*)buf, (f32x4*)buf + n4 / 2,
                                   n4 / 2);
                break;
            default:
                hipMemcpyAsync((char*)buf + bytes / 2, buf, bytes / 2, hipMemcpyDeviceToDevice, s);
        }
    };
    launch();
    hipEventRecord(a, s);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    *ms_out = ms / reps;
    hipFree(sink);
    hipEventDestroy(a);
    hipEventDestroy(b);
    hipStreamDestroy(s);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
}
