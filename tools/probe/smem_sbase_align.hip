// Minimal reproducer (round 6): hipcc emits a scalar load whose SGPR base is
// not 4-byte aligned, and gfx950 drops the base's low address bits.
//
// A byval kernel argument's uint16_t array read at a wave-uniform EVEN index
// p (p = 4 q + 2): the element's address kernarg + OFF + 2 p is dword-aligned,
// so the compiler uses one s_load_dword (then a shift) -- but it forms the
// address as SBASE = kernarg + p plus SOFFSET = p:
//     s_add_u32 s4, s0, sP ; s_addc_u32 s5, s1, 0
//     s_load_dword sD, s[4:5], sP offset:OFF
// SBASE = kernarg + 4 q + 2 is misaligned by 2; the hardware ignores its low
// two bits, so the load returns the dword at kernarg + OFF + 8 q: element
// 4 q instead of 4 q + 2.  (k_frame16's F16_RNG_SCALAR builds read
// tdoa_kparams::wc_off that way: every wave's row 2 got the compact offset of
// its row 0, DESIGN.md "k_frame16: the two unexplained failures".)
//
// Output: per q, the value read at p = 4 q + 2 (compiled and via a per-lane
// VMEM read of the same element) against the host's.  Scalar loads only; the
// results leave through vector stores.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

struct Args {  // the tail of tdoa_kparams: wc_off at 284, wc_lo at 340, wc_w at 368
    uint8_t pad[284];
    uint16_t off16[28];
    uint8_t lo8[28], w8[28];
};

// k_frame16's F16_RNG_SCALAR pick, reduced: the wave's four ranges
// (lo | w << 8 | off << 16) of pairs 4 w + q as uniform loads, lane row q's
// picked -- the code that fails in the library build (see the header)
template <int P>  // compile-time, as k_frame16's pair count
__global__ void k_probe(Args a, uint32_t *out)
{
    const int w0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    uint32_t rq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int p = 4 * w0 + q < P ? 4 * w0 + q : 0;
        rq[q] = (uint32_t)a.lo8[p] | (uint32_t)a.w8[p] << 8 | (uint32_t)a.off16[p] << 16;
    }
    const int row = ((int)threadIdx.x >> 4) & 3;
    uint32_t v = row == 0 ? rq[0] : (row == 1 ? rq[1] : (row == 2 ? rq[2] : rq[3]));
    asm volatile("" : "+v"(v));
    if (((int)threadIdx.x & 15) == 0)
        out[threadIdx.x >> 4] = v;
}

// the instruction shape alone, in asm: SBASE = buf + p (p even), SOFFSET = p,
// offset IMM -- exact arithmetic reads the dword at buf + 2 p + IMM
template <int IMM>
__global__ void k_shape(const uint32_t *buf, uint32_t *out)
{
    for (int i = 0; i < 4; i++) {
        const uint32_t p = (uint32_t)__builtin_amdgcn_readfirstlane(2 * i);
        const char *b = reinterpret_cast<const char *>(buf) + p;
        uint32_t r;
        asm volatile("s_load_dword %0, %1, %2 offset:%3\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(r)
                     : "s"(b), "s"(p), "i"(IMM));
        if (threadIdx.x == 0)
            out[i] = r;
    }
}

int main()
{
    constexpr int P = 28, NW = 7;  // seven waves, four pairs each
    Args a{};
    for (int i = 0; i < 28; i++) {
        a.off16[i] = (uint16_t)(1000 + 37 * i);
        a.lo8[i] = (uint8_t)(3 * i + 1);
        a.w8[i] = (uint8_t)(100 + i);
    }
    uint32_t *dout, *dbuf, hout[4 * NW], hbuf[64], hs[4];
    for (int i = 0; i < 64; i++)
        hbuf[i] = 0x100 * i;  // dword i holds 256 i
    if (hipMalloc(&dout, sizeof hout) != hipSuccess || hipMalloc(&dbuf, sizeof hbuf) != hipSuccess)
        return 2;
    hipMemcpy(dbuf, hbuf, sizeof hbuf, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe<P>, dim3(1), dim3(64 * NW), 0, 0, a, dout);
    if (hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost) != hipSuccess)
        return 3;
    int bad = 0;
    for (int r = 0; r < 4 * NW; r++) {
        const uint32_t e = (uint32_t)a.lo8[r] | (uint32_t)a.w8[r] << 8 | (uint32_t)a.off16[r] << 16;
        if (hout[r] != e) {
            printf("compiled pick: pair %d off %u expected %u\n", r, hout[r] >> 16, e >> 16);
            bad++;
        }
    }
    hipLaunchKernelGGL(k_shape<16>, dim3(1), dim3(64), 0, 0, dbuf, dout);
    if (hipMemcpy(hs, dout, sizeof hs, hipMemcpyDeviceToHost) != hipSuccess)
        return 4;
    int bad_shape = 0;
    for (int i = 0; i < 4; i++) {
        const int p = 2 * i;
        const uint32_t exact = hbuf[(2 * p + 16) / 4], dropped = hbuf[(((p & ~3) + p + 16) / 4)];
        printf("asm shape p %d: got dword %u; exact address -> %u, SBASE low bits dropped -> %u\n", p, hs[i] / 256,
               exact / 256, dropped / 256);
        bad_shape += hs[i] != exact;
    }
    printf("{\"compiled_pick_wrong_pairs\": %d, \"asm_shape_wrong\": %d}\n", bad, bad_shape);
    return 0;
}
