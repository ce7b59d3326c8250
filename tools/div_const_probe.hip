// div_const_probe.hip -- diagnostic (not product code): is the quotient by a launch-constant divisor b, computed as
//     r = RN(1 / b);  q = RN(a r);  e = fma(-q, b, a);  q' = RN(q + e r)          (Markstein's correction)
// the correctly rounded a / b?  Away from underflow and overflow the answer depends on the significands of a and b
// only (scaling a or b by a power of two scales every intermediate exactly), so every significand of a in [1, 2)
// (2^23 dividends) is checked against the IEEE division (v_div_scale / v_div_fmas / v_div_fixup) for each divisor
// significand b in [1, 2) of a list.  The product guards the rest: its fast path runs only where a and q have
// exponent fields in [27, 227] and b in [2^-60, 2^60] (fedavg_tiles.h div_const).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/div_const_probe.hip -o tools/build/libdiv_const_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) div_probe(const float* __restrict__ bs, int nb, unsigned long long* __restrict__ bad,
                                                 uint32_t* __restrict__ first_bad) {
    const float b = bs[blockIdx.y];
    const float r = 1.0f / b;
    unsigned long long mism = 0;
    uint32_t fb = 0xFFFFFFFFu;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // one dividend significand per thread
    if (i < (1u << 23)) {
        const float a = __uint_as_float(0x3F800000u | i);
        const float q = a * r;
        const float e = __builtin_fmaf(-q, b, a);
        const float q1 = __builtin_fmaf(e, r, q);
        const float ref = a / b;
        if (__float_as_uint(q1) != __float_as_uint(ref)) {
            mism = 1;
            fb = 0x3F800000u | i;
        }
    }
    if (mism) {
        atomicAdd(bad + blockIdx.y, mism);
        atomicMin(first_bad + blockIdx.y, fb);
    }
}

extern "C" int div_probe_run(const float* host_b, int nb, unsigned long long* host_bad, uint32_t* host_first) {
    float* d_b;
    unsigned long long* d_bad;
    uint32_t* d_first;
    if (hipMalloc(&d_b, nb * 4) || hipMalloc(&d_bad, nb * 8) || hipMalloc(&d_first, nb * 4)) return 1;
    (void)hipMemcpy(d_b, host_b, nb * 4, hipMemcpyHostToDevice);
    (void)hipMemset(d_bad, 0, nb * 8);
    (void)hipMemset(d_first, 0xFF, nb * 4);
    for (int b0 = 0; b0 < nb; b0 += 256) {
        const int n = nb - b0 < 256 ? nb - b0 : 256;
        hipLaunchKernelGGL(div_probe, dim3((1u << 23) / 256, n), dim3(256), 0, 0, d_b + b0, n, d_bad + b0, d_first + b0);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    (void)hipMemcpy(host_bad, d_bad, nb * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(host_first, d_first, nb * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_b);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
