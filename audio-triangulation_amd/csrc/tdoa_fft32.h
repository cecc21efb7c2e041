// tdoa_fft32.h -- register-resident DFT-32 and DPP (max, first index)
// reductions shared by the GCC-PHAT kernels (tdoa_gcc_phat.hip,
// tdoa_phat1024.hip).  Internal linkage: each TU compiles its own copy with its
// own floating-point flags.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 cmulf(f2 a, f2 b)
{
    return f2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ f2 conjf2(f2 a) { return f2{a.x, -a.y}; }
__device__ __forceinline__ f2 times_i(f2 a) { return f2{-a.y, a.x}; }
__device__ __forceinline__ f2 times_mi(f2 a) { return f2{a.y, -a.x}; }

// cos / sin (2 pi k / 32), k = 0..15
__device__ constexpr float COS32[16] = {
    1.0f,         0.98078528f,  0.92387953f,  0.83146961f, 0.70710678f,  0.55557023f,
    0.38268343f,  0.19509032f,  0.0f,         -0.19509032f, -0.38268343f, -0.55557023f,
    -0.70710678f, -0.83146961f, -0.92387953f, -0.98078528f};
__device__ constexpr float SIN32[16] = {
    0.0f,        0.19509032f, 0.38268343f, 0.55557023f, 0.70710678f, 0.83146961f,
    0.92387953f, 0.98078528f, 1.0f,        0.98078528f, 0.92387953f, 0.83146961f,
    0.70710678f, 0.55557023f, 0.38268343f, 0.19509032f};

// t * W_32^k (forward, W = e^{-2 pi i/32}) or * W_32^{-k} (inverse)
template <bool INV>
__device__ __forceinline__ f2 tw32(f2 t, int k)
{
    if (k == 0)
        return t;
    if (k == 8)
        return INV ? times_i(t) : times_mi(t);
    return cmulf(t, f2{COS32[k], INV ? SIN32[k] : -SIN32[k]});
}

__device__ constexpr int brev5(int k)
{
    return ((k & 1) << 4) | ((k & 2) << 2) | (k & 4) | ((k & 8) >> 2) | ((k & 16) >> 4);
}

// In-place radix-2 DIF DFT-32: natural-order input, X[k] ends in v[brev5(k)].
// HALF_ZERO: inputs 16..31 are zero.
template <bool INV, bool HALF_ZERO>
__device__ __forceinline__ void fft32(f2 (&v)[32])
{
#pragma unroll
    for (int span = 16; span >= 1; span >>= 1) {
#pragma unroll
        for (int start = 0; start < 32; start += 2 * span) {
#pragma unroll
            for (int j = 0; j < span; j++) {
                const int k = j * (16 / span);
                if (HALF_ZERO && span == 16) {
                    v[j + 16] = tw32<INV>(v[j], k);
                } else {
                    const f2 a = v[start + j], b = v[start + j + span];
                    v[start + j] = a + b;
                    v[start + j + span] = tw32<INV>(a - b, k);
                }
            }
        }
    }
}


// (max value, first index) combine through one DPP lane move (no LDS round
// trip).  Lanes whose row is outside ROWMASK keep their own value (old = src).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void dpp_argmax(float &v, int &i)
{
    const int vb = __builtin_bit_cast(int, v);
    const float ov =
        __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(vb, vb, CTRL, ROWMASK, 0xF, false));
    const int oi = __builtin_amdgcn_update_dpp(i, i, CTRL, ROWMASK, 0xF, false);
    if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}
// within each 16-lane row: xor 1, xor 2 (quad_perm), half-row mirror, row mirror
__device__ __forceinline__ void row_argmax(float &v, int &i)
{
    dpp_argmax<0xB1, 0xF>(v, i);
    dpp_argmax<0x4E, 0xF>(v, i);
    dpp_argmax<0x141, 0xF>(v, i);
    dpp_argmax<0x140, 0xF>(v, i);
}
// whole wave -> lane 63 (row_bcast:15 into rows 1, 3; row_bcast:31 into rows 2, 3)
__device__ __forceinline__ void wave_argmax_to63(float &v, int &i)
{
    row_argmax(v, i);
    dpp_argmax<0x142, 0xA>(v, i);
    dpp_argmax<0x143, 0xC>(v, i);
}
// each 32-lane half-wave -> its lane 31 / 63
__device__ __forceinline__ void half_argmax_to31(float &v, int &i)
{
    row_argmax(v, i);
    dpp_argmax<0x142, 0xA>(v, i);
}

// ---- (max, first index) by keys: a float as a signed-int key with the same
// order (-0.0 folded to +0.0 first, so equal floats give equal keys; no NaN
// reaches these), reduced by DPP-fused v_max_i32 / v_min_i32 within rows and
// v_permlane16/32_swap across rows; then the smallest index among the lanes
// holding the maximum.  Every lane of the half-wave / wave receives both.
__device__ __forceinline__ int fkey(float v)
{
    const int b = __builtin_bit_cast(int, v + 0.0f);
    return b ^ ((b >> 31) & 0x7FFFFFFF);
}
__device__ __forceinline__ float fkey_value(int k) { return __builtin_bit_cast(float, k ^ ((k >> 31) & 0x7FFFFFFF)); }

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
template <bool MAX>
__device__ __forceinline__ int row_reduce(int v)  // every lane of each 16-lane row
{
    auto op = [](int a, int b) { return MAX ? imax(a, b) : imin(a, b); };
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));   // xor 1
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));   // xor 2
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));  // half-row mirror
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));  // row mirror
    return v;
}
template <bool MAX>
__device__ __forceinline__ int half_reduce(int v)  // rows (0, 1) and (2, 3): each 32-lane half
{
    v = row_reduce<MAX>(v);
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return MAX ? imax(v, imax((int)r[0], (int)r[1])) : imin(v, imin((int)r[0], (int)r[1]));
}
template <bool MAX>
__device__ __forceinline__ int wave_reduce(int v)
{
    v = half_reduce<MAX>(v);
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return MAX ? imax(v, imax((int)r[0], (int)r[1])) : imin(v, imin((int)r[0], (int)r[1]));
}
// key: the lane's best key (INT_MIN: none), idx: its first index (INT_MAX: none)
__device__ __forceinline__ void half_argmax_key(int &key, int &idx)
{
    const int mk = half_reduce<true>(key);
    idx = half_reduce<false>(key == mk ? idx : INT_MAX);
    key = mk;
}
__device__ __forceinline__ void wave_argmax_key(int &key, int &idx)
{
    const int mk = wave_reduce<true>(key);
    idx = wave_reduce<false>(key == mk ? idx : INT_MAX);
    key = mk;
}

}  // namespace
