// tdoa_keys.h -- exact (value, first index) maxima as one unsigned 64-bit key
// reduced across a wave by DPP moves (no LDS round trips); shared by the
// DIRECT matrix-core kernel (tdoa_direct.hip) and the streaming update
// (tdoa_stream.hip).  Internal linkage per TU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

// ---- DPP wave reductions (no LDS round trips): the butterfly of
// tdoa_fft32.h -- xor 1, xor 2, half-row mirror, row mirror, then
// row_bcast:15 into rows 1, 3 and row_bcast:31 into rows 2, 3 -- leaves the
// result in lane 63 (and, without the last step, each half-wave's in lanes 31 / 63)
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int v)
{
    return __builtin_amdgcn_update_dpp(v, v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ void dpp_sum_step(int &x)
{
    x += __builtin_amdgcn_update_dpp(0, x, CTRL, RM, 0xF, false);
}
// sum over each aligned group of `width` lanes (4 .. 64, uniform): the group's
// last lane holds it (every lane of the group for width <= 16)
__device__ __forceinline__ int group_sum_dpp(int x, int width)
{
    dpp_sum_step<0xB1, 0xF>(x);
    dpp_sum_step<0x4E, 0xF>(x);
    if (width > 4)
        dpp_sum_step<0x141, 0xF>(x);
    if (width > 8)
        dpp_sum_step<0x140, 0xF>(x);
    if (width > 16)
        dpp_sum_step<0x142, 0xA>(x);
    if (width > 32)
        dpp_sum_step<0x143, 0xC>(x);
    return x;
}
template <int CTRL, int RM>
__device__ __forceinline__ void dpp_umax_step(uint64_t &k)
{
    const uint32_t lo = (uint32_t)dpp_i<CTRL, RM>((int)(uint32_t)k);
    const uint32_t hi = (uint32_t)dpp_i<CTRL, RM>((int)(uint32_t)(k >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    k = o > k ? o : k;
}
// unsigned 64-bit max of the wave -> lane 63
__device__ __forceinline__ uint64_t wave_umax_dpp(uint64_t k)
{
    dpp_umax_step<0xB1, 0xF>(k);
    dpp_umax_step<0x4E, 0xF>(k);
    dpp_umax_step<0x141, 0xF>(k);
    dpp_umax_step<0x140, 0xF>(k);
    dpp_umax_step<0x142, 0xA>(k);
    dpp_umax_step<0x143, 0xC>(k);
    return k;
}
__device__ __forceinline__ uint64_t lane63_u64(uint64_t k)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

// Exact int64 (value, first index) maxima as one unsigned key: |score| <=
// N * 2^30 <= 2^42 (N <= 4096) and |L| <= 28 * 2^42 < 2^47, so
// key = (v + 2^47) << IB | (2^IB - 1 - index) orders by value, then by the
// smaller index, in 48 + IB <= 64 bits.  Argmax: index = lag slot (IB = 7,
// correlations.c:20-23 keeps the first maximum); grid: index = the tuple's
// first cell or the tuple index (IB = 16, callers check < 65536) -- tuple
// order is first-cell order, so the smallest cell among equal L is the first
// row-major argmax of vga_heatmap.h:99-108.
constexpr int64_t KEY_BIAS = (int64_t)1 << 47;
template <int IB>
__device__ __forceinline__ uint64_t vkey(int64_t v, int idx)
{
    return ((uint64_t)(v + KEY_BIAS) << IB) | (uint64_t)((1 << IB) - 1 - idx);
}
template <int IB>
__device__ __forceinline__ int64_t key_value(uint64_t k)
{
    return (int64_t)(k >> IB) - KEY_BIAS;
}
template <int IB>
__device__ __forceinline__ int key_index(uint64_t k)
{
    return (1 << IB) - 1 - (int)(k & ((1u << IB) - 1));
}

}  // namespace
