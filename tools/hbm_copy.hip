// hbm_copy.hip -- achievable-HBM calibration for the roofline denominator
// (SURVEY.md 8(d)): a 16-B-per-lane streaming copy over
// buffers far larger than the 256 MiB Infinity Cache, timed with HIP events.
//
//   hbm_copy [MiB per buffer, default 1024] [iterations, default 20]
//
// Prints one JSON line: bytes moved per launch (read + write), the average
// launch time and the achieved GB/s.  Run it under
//   rocprofv3 --kernel-trace --stats -- ./hbm_copy
// so the rocprof average of k_copy16 can be set beside the event figure.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

// grid-stride copy, 16 B per lane per access, four accesses in flight per lane
__global__ void __launch_bounds__(256) k_copy16(const v4u *__restrict__ src, v4u *__restrict__ dst,
                                                size_t n16)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        v4u a = __builtin_nontemporal_load(src + i);
        v4u b = __builtin_nontemporal_load(src + i + stride);
        v4u c = __builtin_nontemporal_load(src + i + 2 * stride);
        v4u d = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2 * stride);
        __builtin_nontemporal_store(d, dst + i + 3 * stride);
    }
    for (; i < n16; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// the same copy with default-policy loads and stores (nt stores are not
// write-through on gfx950, and the plain form is the guide's float4 copy)
__global__ void __launch_bounds__(256) k_copy16p(const v4u *__restrict__ src, v4u *__restrict__ dst,
                                                 size_t n16)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const v4u a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride)
        dst[i] = src[i];
}

// read-only sweep (sum of words), the bound of a read-dominated kernel
__global__ void __launch_bounds__(256) k_read16(const v4u *__restrict__ src, size_t n16, unsigned *sink)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const v4u a = __builtin_nontemporal_load(src + i);
        acc += a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u)  // practically never: keeps the loads alive
        sink[0] = acc;
}

__global__ void k_fill(v4u *p, size_t n16)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v4u{(unsigned)i, (unsigned)(i * 3), (unsigned)(i * 7), (unsigned)(i * 11)};
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 1024;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    if (mib < 16 || mib > 16384 || iters < 1 || iters > 1000) {
        fprintf(stderr, "usage: hbm_copy [16..16384 MiB] [1..1000 iterations]\n");
        return 2;
    }
    const size_t bytes = mib << 20, n16 = bytes / 16;
    v4u *a = nullptr, *b = nullptr;
    unsigned *sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, n16);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, b, n16);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const dim3 grid(cus * 8), block(256);  // 8 x 256-thread workgroups per CU
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms_copy = 0.f, ms_copyp = 0.f, ms_read = 0.f;
    const dim3 gridp(cus * 4);  // plain copy: 4 x 256-thread workgroups per CU
    for (int pass = 0; pass < 2; pass++) {  // pass 0: warm-up (clocks, translations)
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; i++)  // alternate directions: no buffer stays cached
            hipLaunchKernelGGL(k_copy16, grid, block, 0, 0, (i & 1) ? b : a, (i & 1) ? a : b, n16);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_copy, e0, e1));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; i++)
            hipLaunchKernelGGL(k_copy16p, gridp, block, 0, 0, (i & 1) ? b : a, (i & 1) ? a : b, n16);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_copyp, e0, e1));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; i++)
            hipLaunchKernelGGL(k_read16, grid, block, 0, 0, (i & 1) ? b : a, n16, sink);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_read, e0, e1));
    }
    CK(hipGetLastError());
    const double t_copy = ms_copy / 1e3 / iters, t_read = ms_read / 1e3 / iters, t_copyp = ms_copyp / 1e3 / iters;
    printf("{\"kernel\": \"k_copy16\", \"mib_per_buffer\": %zu, \"iterations\": %d, \"grid\": %u, "
           "\"copy_bytes_per_launch\": %zu, \"copy_us\": %.3f, \"copy_gbs\": %.1f, "
           "\"copy_plain_kernel\": \"k_copy16p\", \"copy_plain_grid\": %u, \"copy_plain_us\": %.3f, "
           "\"copy_plain_gbs\": %.1f, "
           "\"read_kernel\": \"k_read16\", \"read_bytes_per_launch\": %zu, \"read_us\": %.3f, "
           "\"read_gbs\": %.1f}\n",
           mib, iters, grid.x, 2 * bytes, t_copy * 1e6, 2.0 * bytes / t_copy / 1e9, gridp.x, t_copyp * 1e6,
           2.0 * bytes / t_copyp / 1e9, bytes, t_read * 1e6, (double)bytes / t_read / 1e9);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
