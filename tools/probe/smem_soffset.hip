// Probe (diagnostic, round 6): scalar loads that carry BOTH an SGPR offset and
// an immediate offset (`s_load_dword sD, s[B:B+1], sOFF offset:IMM`, the SMEM
// SOE + IMM form), which hipcc emits for a kernel-argument array indexed by a
// wave-uniform runtime value.  k_frame16's F16_RNG_SCALAR build reads its
// compact ranges kp.wc_lo / wc_w / wc_off that way and gets wrong offsets for
// some pairs (tests/test_gpu_bench_path.py, DESIGN.md "the two unexplained
// failures").  Three forms, each checked against the host:
//   asm_global   inline asm on a global buffer
//   asm_kernarg  inline asm on the kernarg segment pointer
//   compiled     a byval struct's byte / u16 arrays at a readfirstlane index
// Scalar loads only; every result leaves through a vector store.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

struct Args {
    uint8_t pad[284];
    uint16_t off16[32];  // at 284, as tdoa_kparams::wc_off
    uint8_t lo8[32];     // at 348
    uint8_t w8[32];      // at 380
    int32_t words[64];   // at 412
};

template <int IMM>
__device__ __forceinline__ uint32_t sload_soe(const void *base, uint32_t soff)
{
    uint32_t r;
    asm volatile("s_load_dword %0, %1, %2 offset:%3\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(r)
                 : "s"(base), "s"(soff), "i"(IMM));
    return r;
}

__global__ void k_probe(Args a, const uint32_t *gbuf, uint32_t *out, int n)
{
    const int lane = threadIdx.x;
    for (int i = 0; i < n; i++) {
        const uint32_t soff = (uint32_t)__builtin_amdgcn_readfirstlane(4 * i);
        // asm on a global buffer: gbuf[k] = k; address gbuf + soff + 16
        const uint32_t g = sload_soe<16>(gbuf, soff);
        // asm on the kernarg segment: a.words at kernarg + 412 + soff
        const uint32_t k = sload_soe<412>((const void *)__builtin_amdgcn_kernarg_segment_ptr(), soff);
        // compiled: byval arrays at a wave-uniform runtime index
        const int p = __builtin_amdgcn_readfirstlane(i);
        const uint32_t c = (uint32_t)a.lo8[p] | (uint32_t)a.w8[p] << 8 | (uint32_t)a.off16[p] << 16;
        if (lane == 0) {
            out[4 * i] = g;
            out[4 * i + 1] = k;
            out[4 * i + 2] = c;
            out[4 * i + 3] = (uint32_t)a.words[p];
        }
    }
}

int main()
{
    const int n = 28;
    Args a{};
    for (int i = 0; i < 32; i++) {
        a.off16[i] = (uint16_t)(1000 + 37 * i);
        a.lo8[i] = (uint8_t)(3 * i + 1);
        a.w8[i] = (uint8_t)(100 + i);
    }
    for (int i = 0; i < 64; i++)
        a.words[i] = 0x5000 + i;
    uint32_t hg[256], hout[4 * n];
    for (int i = 0; i < 256; i++)
        hg[i] = 0xA000 + i;
    uint32_t *dg, *dout;
    if (hipMalloc(&dg, sizeof hg) != hipSuccess || hipMalloc(&dout, sizeof hout) != hipSuccess)
        return 2;
    hipMemcpy(dg, hg, sizeof hg, hipMemcpyHostToDevice);
    hipMemset(dout, 0xFF, sizeof hout);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, a, dg, dout, n);
    if (hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost) != hipSuccess)
        return 3;
    int bad[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const uint32_t eg = 0xA000 + 4 + i;  // gbuf + 4 i + 16 bytes
        const uint32_t ek = 0x5000 + i;
        const uint32_t ec = (uint32_t)a.lo8[i] | (uint32_t)a.w8[i] << 8 | (uint32_t)a.off16[i] << 16;
        const uint32_t e[4] = {eg, ek, ec, ek};
        for (int f = 0; f < 4; f++)
            if (hout[4 * i + f] != e[f]) {
                if (bad[f] < 4)
                    printf("form %d index %d: got 0x%x expected 0x%x\n", f, i, hout[4 * i + f], e[f]);
                bad[f]++;
            }
    }
    printf("{\"asm_global_bad\": %d, \"asm_kernarg_bad\": %d, \"compiled_bad\": %d, \"compiled_words_bad\": %d, "
           "\"indices\": %d}\n",
           bad[0], bad[1], bad[2], bad[3], n);
    return 0;
}
