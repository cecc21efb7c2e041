// tdoa_probe.hip -- the shader clock under VALU load (bench.py's gpu_clock_mhz).
//
// Boxes of the pool run the same build several percent apart (DESIGN.md,
// round 5: k_p1k_lean 31.5 vs 29.3 us), and the chip's clock under load is
// power-limited, not the 2.4 GHz boost.  bench.py runs this probe right after
// its timed region so the line records the clock the box held: every CU's
// waves run independent FMA chains (the load the GCC-PHAT kernels put on the
// SIMDs) for about `ms` milliseconds, and each wave reads s_memtime (shader
// clock) and s_memrealtime (the chip's constant 100 MHz clock) at both ends.
// Clock = median over waves of d(memtime) / d(memrealtime) x 100 MHz.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "tdoa.h"
#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

constexpr int PROBE_THREADS = 256;

__global__ void __launch_bounds__(PROBE_THREADS) k_clock_probe(unsigned long long ticks, float seed,
                                                               unsigned long long *out, float *sink)
{
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        a[i] = seed + (float)(threadIdx.x + i);
    unsigned long long r1 = r0;
    do {
#pragma unroll 4
        for (int it = 0; it < 64; it++)
#pragma unroll
            for (int i = 0; i < 8; i++)
                a[i] = __builtin_fmaf(a[i], 0.999999f, 1e-7f);
        r1 = __builtin_amdgcn_s_memrealtime();
    } while (r1 - r0 < ticks);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++)
        s += a[i];
    if (s == 12345.0f)  // keeps the chains live; never true in practice
        sink[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (PROBE_THREADS / 64) + threadIdx.x / 64;
        out[2 * w] = c1 - c0;
        out[2 * w + 1] = r1 - r0;
    }
}

}  // namespace

extern "C" int tdoa_gpu_clock_mhz(int device, void *stream, double ms, double *mhz)
{
    if (!mhz || !(ms > 0.0) || ms > 100.0)
        return tdoa_set_error(-1, "tdoa_gpu_clock_mhz: mhz must be non-null, 0 < ms <= 100");
    if (hipSetDevice(device) != hipSuccess)
        return tdoa_set_error(-2, "tdoa_gpu_clock_mhz: hipSetDevice failed");
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        return tdoa_set_error(-2, "tdoa_gpu_clock_mhz: no CU count");
    // four workgroups of four waves per CU: four waves per SIMD
    const int blocks = 4 * cus, waves = blocks * (PROBE_THREADS / 64);
    unsigned long long *d_out = nullptr;
    float *d_sink = nullptr;
    if (hipMalloc(&d_out, sizeof(unsigned long long) * 2 * waves) != hipSuccess ||
        hipMalloc(&d_sink, sizeof(float) * PROBE_THREADS) != hipSuccess) {
        (void)hipFree(d_out);
        return tdoa_set_error(-2, "tdoa_gpu_clock_mhz: hipMalloc failed");
    }
    hipStream_t st = (hipStream_t)stream;
    const unsigned long long ticks = (unsigned long long)(ms * 1e5);  // 100 MHz
    hipLaunchKernelGGL(k_clock_probe, dim3((unsigned)blocks), dim3(PROBE_THREADS), 0, st, ticks, 1.0f, d_out,
                       d_sink);
    std::vector<unsigned long long> h(2 * (size_t)waves);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(h.data(), d_out, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
    if (e != hipSuccess)
        return tdoa_set_error(-2, "tdoa_gpu_clock_mhz: probe launch failed");
    std::vector<double> f;
    f.reserve(waves);
    for (int w = 0; w < waves; w++)
        if (h[2 * w + 1] > 0)
            f.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 100.0);
    if (f.empty())
        return tdoa_set_error(-2, "tdoa_gpu_clock_mhz: no samples");
    std::nth_element(f.begin(), f.begin() + f.size() / 2, f.end());
    *mhz = f[f.size() / 2];
    return 0;
}
