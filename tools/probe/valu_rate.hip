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
    long long q[C];
#pragma unroll
    for (int i = 0; i < C; i++) {
        q[i] = (long long)t * (i + 3);
        a[i] = f2{(float)(t + i), (float)(t - i)};
        s[i] = (float)(t * i);
        u[i] = t + i;
    }
    const f2 m = f2{1.0001f, 0.9999f}, c = f2{0.5f, 0.25f};
    const unsigned long long msk = __builtin_amdgcn_ballot_w64((t & 8) != 0);
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
                else if (KIND == 3)
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(t));
                else if (KIND == 4)  // lane-half exchange of two registers
                    asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(s[i]), "+v"(u[i]));
                else if (KIND == 5)
                    asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(s[i]), "+v"(u[i]));
                else if (KIND == 6)  // DPP-sourced add (row_ror:8)
                    asm volatile("v_add_f32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(s[i]) : "v"(c.x));
                else if (KIND == 7)
                    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(s[i]) : "v"(c.x), "s"(msk));
                else if (KIND == 10)  // DPP move (row_ror:8)
                    asm volatile("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(s[i]));
                else if (KIND == 11)  // lane-select by a per-lane bit: v_bfi (mask in a VGPR)
                    asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(u[i]) : "v"(t), "v"(u[(i + 1) % C]));
                else if (KIND == 8)  // complex product by an SGPR constant (the c_mul_s pair)
                    asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[0,1]\n\tv_pk_fma_f32 %0, %0, %1, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "+v"(a[i]) : "s"(m));
                else if (KIND == 12) {  // 64-bit multiply-add of 32-bit operands
                    unsigned long long cy;
                    asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q[i]), "=s"(cy) : "v"(t), "v"(u[i]));
                } else if (KIND == 13)
                    asm volatile("v_mad_i32_i24 %0, %0, %1, %2" : "+v"(u[i]) : "v"(t), "v"(u[(i + 1) % C]));
                else if (KIND == 14)
                    asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(t));
                else if (KIND == 15)
                    asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) % C]));
                else if (KIND == 16) {  // 64-bit compare (VCC)
                    asm volatile("v_cmp_gt_i64_e32 vcc, %0, %1" : : "v"(q[i]), "v"(q[(i + 1) % C]) : "vcc");
                } else if (KIND == 17)
                    asm volatile("v_lshlrev_b64 %0, 9, %0" : "+v"(q[i]));
                else  // a VALU op followed by s_nop 0 (the inline-asm boundary padding)
                    asm volatile("v_pk_add_f32 %0, %0, %1\n\ts_nop 0" : "+v"(a[i]) : "v"(c));
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0;
#pragma unroll
    for (int i = 0; i < C; i++)
        acc += a[i].x + a[i].y + s[i] + (float)u[i] + (float)q[i];
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
    run<0, 16>(cus, out, cyc, "v_pk_fma_f32");
    run<18, 16>(cus, out, cyc, "pk_fma+s_mov");
    run<19, 16>(cus, out, cyc, "2pk_fma+s_mov");
    run<20, 16>(cus, out, cyc, "pk_fma sgpr");
    run<2, 16>(cus, out, cyc, "v_fma_f32");
    return 0;
    run<3, 16>(cus, out, cyc, "v_add_u32");
    run<12, 16>(cus, out, cyc, "v_mad_i64_i32");
    run<13, 16>(cus, out, cyc, "v_mad_i32_i24");
    run<14, 16>(cus, out, cyc, "v_mul_lo_u32");
    run<15, 16>(cus, out, cyc, "v_lshl_add_u64");
    run<16, 16>(cus, out, cyc, "v_cmp_gt_i64");
    run<17, 16>(cus, out, cyc, "v_lshlrev_b64");
    return 0;
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
    run<7, 8>(cus, out, cyc, "cndmask_e64");
    run<10, 8>(cus, out, cyc, "v_mov_dpp");
    run<11, 8>(cus, out, cyc, "v_bfi_b32");
    return 0;
    run<4, 8>(cus, out, cyc, "permlane32");
    run<5, 8>(cus, out, cyc, "permlane16");
    run<6, 8>(cus, out, cyc, "v_add_f32_dpp");
    run<7, 8>(cus, out, cyc, "v_cndmask");
    run<8, 8>(cus, out, cyc, "pk_mul+pk_fma");
    run<9, 8>(cus, out, cyc, "pk_add+s_nop");
    return 0;
}
