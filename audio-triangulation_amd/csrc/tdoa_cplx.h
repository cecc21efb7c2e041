// tdoa_cplx.h -- packed-fp32 complex arithmetic for gfx950 (one f2 = one
// 64-bit VGPR pair = re, im).  The compiler does not fold the re/im swaps of
// "* i" and the conjugations of complex code into the VOP3P op_sel / neg
// modifiers of v_pk_add_f32 / v_pk_fma_f32 (it materialises them with v_mov +
// v_xor), so the primitives below pin one packed instruction each:
//   op_sel[i]    picks the dword of source i that feeds the LOW result,
//   op_sel_hi[i] the dword that feeds the HIGH result (default 1 = high),
//   neg_lo / neg_hi negate source i's input to the low / high result.
// Used by the GCC-PHAT kernels (tdoa_phat1024.hip, tdoa_p1k_w64.hip, tdoa_phat_r16.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "tdoa_fft32.h"

namespace {

__device__ __forceinline__ f2 v_xx(f2 a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ f2 v_yy(f2 a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ f2 v_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

#ifdef TDOA_ASM_MUL_S
// products by compile-time twiddles in an SGPR pair as pinned asm pairs
// (tdoa_phat_r16.hip, whose scheduling measured better with them)
#define TDOA_PK_MUL_S(name, mods1, mods2)                                                  \
    __device__ __forceinline__ f2 name(f2 a, f2 w)                                         \
    {                                                                                      \
        f2 t, r;                                                                           \
        asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]" mods1 "\n\t"                         \
            "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1]" mods2             \
            : "=v"(r), "=&v"(t)                                                            \
            : "v"(a), "s"(w));                                                             \
        return r;                                                                          \
    }
TDOA_PK_MUL_S(c_mul_s, "", " neg_lo:[0,1,0]")
TDOA_PK_MUL_S(c_mulconj_s, "", " neg_hi:[0,0,1]")
TDOA_PK_MUL_S(c_negmul_s, " neg_lo:[0,1] neg_hi:[0,1]", " neg_hi:[0,1,0]")
TDOA_PK_MUL_S(c_negmulconj_s, " neg_lo:[0,1] neg_hi:[0,1]", " neg_lo:[0,1,0] neg_hi:[0,1,1]")
#undef TDOA_PK_MUL_S
#else
// products by compile-time twiddles (SGPR-pair constants) as plain packed-vector
// code: splats become op_sel, so each is still v_pk_mul + v_pk_fma, but the
// post-RA scheduler sees them and fills the packed-result hazard slots
__device__ __forceinline__ f2 c_mul_s(f2 a, f2 w) { return v_fma(v_yy(a), f2{-w.y, w.x}, v_xx(a) * w); }
__device__ __forceinline__ f2 c_mulconj_s(f2 a, f2 w) { return v_fma(v_yy(a), f2{w.y, w.x}, v_xx(a) * f2{w.x, -w.y}); }
__device__ __forceinline__ f2 c_negmul_s(f2 a, f2 w) { return c_mul_s(a, f2{-w.x, -w.y}); }
__device__ __forceinline__ f2 c_negmulconj_s(f2 a, f2 w) { return c_mulconj_s(a, f2{-w.x, -w.y}); }
#endif

#define TDOA_PK(name, mnemonic, mods)                                      \
    __device__ __forceinline__ f2 name(f2 a, f2 b)                         \
    {                                                                      \
        f2 r;                                                              \
        asm(mnemonic " %0, %1, %2 " mods : "=v"(r) : "v"(a), "v"(b));      \
        return r;                                                          \
    }
// a + conj(b), a - conj(b)
TDOA_PK(c_addconj, "v_pk_add_f32", "neg_hi:[0,1]")
TDOA_PK(c_subconj, "v_pk_add_f32", "neg_lo:[0,1]")
// a - i b = (a.x + b.y, a.y - b.x);  a + i b = (a.x - b.y, a.y + b.x)
TDOA_PK(c_add_mi, "v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]")
TDOA_PK(c_add_i, "v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]")
// -i (a - b) = (a.y - b.y, b.x - a.x);  i (a - b) = (b.y - a.y, a.x - b.x)
TDOA_PK(c_sub_mi, "v_pk_add_f32", "op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]")
TDOA_PK(c_sub_i, "v_pk_add_f32", "op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[1,0] neg_hi:[0,1]")
// conj(a + i b) = (a.x - b.y, -a.y - b.x);  conj(a - i b) = (a.x + b.y, b.x - a.y)
TDOA_PK(c_conj_add_i, "v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[1,1]")
TDOA_PK(c_conj_add_mi, "v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[1,0]")
#undef TDOA_PK

// a * w
__device__ __forceinline__ f2 c_mul(f2 a, f2 w)
{
    f2 t, r;
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r), "=&v"(t)
        : "v"(a), "v"(w));
    return r;
}
// a * conj(w)
__device__ __forceinline__ f2 c_mulconj(f2 a, f2 w)
{
    f2 t, r;
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,0,1]"
        : "=v"(r), "=&v"(t)
        : "v"(a), "v"(w));
    return r;
}
// conj(a) * b
__device__ __forceinline__ f2 c_conjmul(f2 a, f2 b)
{
    f2 t, r;
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,1,0]"
        : "=v"(r), "=&v"(t)
        : "v"(a), "v"(b));
    return r;
}
// -i x = (x.y, -x.x);  i x = (-x.y, x.x)
__device__ __forceinline__ f2 c_mi(f2 x)
{
    f2 r;
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ f2 c_i(f2 x)
{
    f2 r;
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_lo:[0,1]" : "=v"(r) : "v"(x));
    return r;
}

// x / sqrt(|x|^2 + e2): |x|^2 + e2 as two fma (no clamp instruction; a zero
// bin stays 0, and for every other bin of an integer frame e2 is far below the
// fp32 resolution of |x|^2), rsq, scale.  Plain vector code: the splat {r, r}
// folds into op_sel_hi (no copy), and the compiler sees the rsq result's
// wait state (the pinned-asm form carried an unconditional s_nop 0)
__device__ __forceinline__ f2 c_unit(f2 x, float e2)
{
#ifdef TDOA_ASM_MUL_S
    // k_frame16 (tdoa_phat_r16.hip) keeps the pinned form, which measured
    // faster there (4.09 vs 4.10 ms per config-3 step, 110.0 vs 112.3 ms per
    // config-4 step, together with its DIF twiddles); the asm multiply opens
    // with s_nop 0 because the compiler does not pad a transcendental result
    // ahead of inline asm
    const float m = __builtin_fmaf(x.x, x.x, __builtin_fmaf(x.y, x.y, e2));
    f2 rr;
    rr.x = __builtin_amdgcn_rsqf(m);
    f2 y;
#ifndef TDOA_UNIT_NOP
#define TDOA_UNIT_NOP "s_nop 0\n\t"  // the trans-use wait state (tools/co_audit.py checks it)
#endif
    asm(TDOA_UNIT_NOP "v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(y) : "v"(x), "v"(rr));
    return y;
#else
    const float r = __builtin_amdgcn_rsqf(__builtin_fmaf(x.x, x.x, __builtin_fmaf(x.y, x.y, e2)));
    return x * f2{r, r};
#endif
}

// W_32^k = e^{-2 pi i k / 32}, k = 1..7 (the others by symmetry)
__device__ __forceinline__ f2 w32c(int k)
{
    constexpr float C[8] = {1.0f,         0.98078528f, 0.92387953f, 0.83146961f,
                            0.70710678f,  0.55557023f, 0.38268343f, 0.19509032f};
    return f2{C[k], -C[8 - k]};
}

// (a - b) * W_32^{+-k}: the twiddle of one radix-2 DIF butterfly
template <bool INV>
__device__ __forceinline__ f2 dif_tw(f2 a, f2 b, int k)
{
    if (k == 0)
        return a - b;
    if (k == 8)
        return INV ? c_sub_i(a, b) : c_sub_mi(a, b);
    if (k < 8)
        return INV ? c_mulconj_s(a - b, w32c(k)) : c_mul_s(a - b, w32c(k));
    // W^k = -conj(W^{16-k})
    return INV ? c_mul_s(b - a, w32c(16 - k)) : c_mulconj_s(b - a, w32c(16 - k));
}
// x * W_32^{+-k} (no subtraction)
template <bool INV>
__device__ __forceinline__ f2 tw_only(f2 x, int k)
{
    if (k == 0)
        return x;
    if (k == 8)
        return INV ? c_i(x) : c_mi(x);
    if (k < 8)
        return INV ? c_mulconj_s(x, w32c(k)) : c_mul_s(x, w32c(k));
    return INV ? c_negmul_s(x, w32c(16 - k)) : c_negmulconj_s(x, w32c(16 - k));
}

// cos / sin (2 pi q / 32), q = 0..16, in double: the FMA butterfly constants
// below are rounded once from their exact quotients
__device__ constexpr double COS32D[17] = {
    1.0, 0.98078528040323043, 0.92387953251128674, 0.83146961230254524, 0.70710678118654752,
    0.55557023301960218, 0.38268343236508977, 0.19509032201612826, 0.0, -0.19509032201612826,
    -0.38268343236508977, -0.55557023301960218, -0.70710678118654752, -0.83146961230254524,
    -0.92387953251128674, -0.98078528040323043, -1.0};
__device__ __forceinline__ f2 v_sw(f2 a) { return __builtin_shufflevector(a, a, 1, 0); }

// DIT butterfly (a, b) <- (a + W b, a - W b), W = W_32^{+-q} (q compile-time
// after unrolling), in three packed FMAs for a non-trivial W (Goedecker's
// tangent form; the swaps fold into op_sel):
//   |Re W| >= |Im W|: W b = c (b + i tau b), tau = Im W / Re W, c = Re W
//       u = fma(swap(b), (-tau, tau), b);  a +- c u
//   otherwise:       W b = i s (b - i kap b), kap = Re W / Im W, s = Im W
//       u = fma(swap(b), (kap, -kap), b);  a +- i s u = fma(swap(u), (-+s, +-s), a)
// W = 1 and W = -+i are one packed add each.
template <bool INV>
__device__ __forceinline__ void bfly_dit(f2 &a, f2 &b, int q)
{
    const f2 t = a;
    if (q == 0) {
        a = t + b;
        b = t - b;
        return;
    }
    if (q == 8) {  // W = -i (forward), +i (inverse)
        a = INV ? c_add_i(t, b) : c_add_mi(t, b);
        b = INV ? c_add_mi(t, b) : c_add_i(t, b);
        return;
    }
    // sin(2 pi q / 32) = cos(2 pi (8 - q) / 32); forward Im W = -sin
    const double wr = COS32D[q], si = COS32D[q < 8 ? 8 - q : q - 8];
    const double im = INV ? si : -si;
    if (__builtin_fabs(wr) >= __builtin_fabs(im)) {
        const float tau = (float)(im / wr), c = (float)wr;
        const f2 u = v_fma(v_sw(b), f2{-tau, tau}, b);
        a = v_fma(u, f2{c, c}, t);
        b = v_fma(u, f2{-c, -c}, t);
    } else {
        const float kap = (float)(wr / im), s = (float)im;
        const f2 u = v_fma(v_sw(b), f2{kap, -kap}, b);
        a = v_fma(v_sw(u), f2{-s, s}, t);
        b = v_fma(v_sw(u), f2{s, -s}, t);
    }
}

// Radix-2 DIT DFT-32 with FMA butterflies, natural order in and out (the
// input bit reversal is register renaming).  HALF_ZERO: inputs 16..31 are
// zero, so the first stage is a copy.  34 non-trivial butterflies at three
// packed FMAs: 194 instructions (162 with HALF_ZERO) against the DIF form's
// 228 (197).
template <bool INV, bool HALF_ZERO>
__device__ __forceinline__ void fft32d(f2 (&x)[32])
{
    f2 v[32];
#pragma unroll
    for (int i = 0; i < 32; i++)
        v[i] = x[brev5(i)];
#pragma unroll
    for (int g = 0; g < 32; g += 2) {
        if (HALF_ZERO)
            v[g + 1] = v[g];
        else
            bfly_dit<INV>(v[g], v[g + 1], 0);
    }
#pragma unroll
    for (int m = 4; m <= 32; m *= 2)
#pragma unroll
        for (int g = 0; g < 32; g += m)
#pragma unroll
            for (int j = 0; j < m / 2; j++)
                bfly_dit<INV>(v[g + j], v[g + j + m / 2], j * (32 / m));
#pragma unroll
    for (int k = 0; k < 32; k++)
        x[k] = v[k];
}

// In-place radix-2 DIF DFT-32 on packed primitives: natural-order input, X[k]
// ends in v[brev5(k)].  HALF_ZERO: inputs 16..31 are zero.
template <bool INV, bool HALF_ZERO>
__device__ __forceinline__ void fft32p(f2 (&v)[32])
{
#pragma unroll
    for (int span = 16; span >= 1; span >>= 1) {
#pragma unroll
        for (int start = 0; start < 32; start += 2 * span) {
#pragma unroll
            for (int j = 0; j < span; j++) {
                const int k = j * (16 / span);
                if (HALF_ZERO && span == 16) {
                    v[j + 16] = tw_only<INV>(v[j], k);
                } else {
                    const f2 a = v[start + j], b = v[start + j + span];
                    v[start + j] = a + b;
                    v[start + j + span] = dif_tw<INV>(a, b, k);
                }
            }
        }
    }
}

// LDS read the backend does not merge into ds_read2_b64 (a volatile
// access; volatile reads stay in order among themselves only): two
// ds_read_b64 take 4 LDS cycles, one ds_read2_b64 8, and ds_read2 banks by
// (a/4) mod 32 (MI355X_MICROARCH.md LDS table)
__device__ __forceinline__ f2 lds_rd(const f2 *p)
{
    typedef __attribute__((address_space(3))) f2 lds_f2;
    return *(const volatile lds_f2 *)(const lds_f2 *)p;
}
__device__ __forceinline__ uint32_t lds_rd_u32(const uint32_t *p)
{
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    return *(const volatile lds_u32 *)(const lds_u32 *)p;
}

// half exchange of two complex registers across lane bit 5 (vdst = a: lanes
// 32-63 of a <-> lanes 0-31 of b) / lane bit 4 (odd rows of a <-> even rows of b).
// The components go through scalar copies: __builtin_bit_cast of an
// ext_vector element (a.y) reads element 0 with this compiler.
template <bool X32>
__device__ __forceinline__ void pswap(f2 &a, f2 &b)
{
    const float ax = a.x, ay = a.y, bx = b.x, by = b.y;
    const unsigned uax = __float_as_uint(ax), uay = __float_as_uint(ay), ubx = __float_as_uint(bx),
                   uby = __float_as_uint(by);
    const auto rx = X32 ? __builtin_amdgcn_permlane32_swap(uax, ubx, false, false)
                        : __builtin_amdgcn_permlane16_swap(uax, ubx, false, false);
    const auto ry = X32 ? __builtin_amdgcn_permlane32_swap(uay, uby, false, false)
                        : __builtin_amdgcn_permlane16_swap(uay, uby, false, false);
    const unsigned r0 = rx[0], r1 = rx[1], r2 = ry[0], r3 = ry[1];
    a = f2{__uint_as_float(r0), __uint_as_float(r2)};
    b = f2{__uint_as_float(r1), __uint_as_float(r3)};
}
__device__ __forceinline__ void pswap32(f2 &a, f2 &b) { pswap<true>(a, b); }
__device__ __forceinline__ void pswap16(f2 &a, f2 &b) { pswap<false>(a, b); }

}  // namespace
