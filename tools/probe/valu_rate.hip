// valu_rate.hip -- SIMD issue-rate / latency probe (diagnostic only): cycles
// (s_memtime) per wave64 VALU instruction per SIMD for packed fp32 FMA / add,
// scalar fp32 FMA and 32-bit integer adds, with C independent chains per wave
// at 1, 2 and 4 waves per SIMD (one workgroup of 4 * W waves per CU, every CU).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND, int C>
__global__ void __launch_bounds__(1024) k_rate(float *out, unsigned long long *cyc, int iters)
{
    const int t = threadIdx.x;
    f2 a[C];
    float s[C];
    int u[C];
#pragma unroll
    for (int i = 0; i < C; i++) {
        a[i] = f2{(float)(t + i), (float)(t - i)};
        s[i] = (float)(t * i);
        u[i] = t + i;
    }
    const f2 m = f2{1.0001f, 0.9999f}, c = f2{0.5f, 0.25f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < iters; k++) {
#pragma unroll
        for (int r = 0; r < 128 / C; r++)
#pragma unroll
            for (int i = 0; i < C; i++) {
                if (KIND == 0)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "v"(c));
                else if (KIND == 1)
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                else if (KIND == 2)
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[i]) : "v"(m.x), "v"(c.x));
                else
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(t));
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0;
#pragma unroll
    for (int i = 0; i < C; i++)
        acc += a[i].x + a[i].y + s[i] + (float)u[i];
    out[blockIdx.x * blockDim.x + t] = acc;
    if ((t & 63) == 0)
        cyc[blockIdx.x * 16 + (t >> 6)] = t1 - t0;
}

template <int KIND, int C>
void run(int cus, float *out, unsigned long long *cyc, const char *name)
{
    const int iters = 100;
    for (int w = 1; w <= 4; w *= 2) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL((k_rate<KIND, C>), dim3(cus), dim3(256 * w), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
        }
        unsigned long long h[16];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        unsigned long long mx = 0;
        for (int i = 0; i < 4 * w; i++)
            mx = h[i] > mx ? h[i] : mx;
        const double insts = (double)iters * 128;  // per wave
        printf("%-13s chains %2d waves/SIMD %d: %.2f cycles per instruction per SIMD\n", name, C, w,
               (double)mx / (insts * w));
    }
}

int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    unsigned long long *cyc;
    (void)hipMalloc(&out, sizeof(float) * cus * 1024);
    (void)hipMalloc(&cyc, sizeof(unsigned long long) * cus * 16);
    run<0, 1>(cus, out, cyc, "v_pk_fma_f32");
    run<0, 4>(cus, out, cyc, "v_pk_fma_f32");
    run<0, 16>(cus, out, cyc, "v_pk_fma_f32");
    run<0, 32>(cus, out, cyc, "v_pk_fma_f32");
    run<1, 1>(cus, out, cyc, "v_pk_add_f32");
    run<1, 16>(cus, out, cyc, "v_pk_add_f32");
    run<2, 1>(cus, out, cyc, "v_fma_f32");
    run<2, 16>(cus, out, cyc, "v_fma_f32");
    run<3, 1>(cus, out, cyc, "v_add_u32");
    run<3, 16>(cus, out, cyc, "v_add_u32");
    return 0;
}
