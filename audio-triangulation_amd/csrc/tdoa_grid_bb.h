// tdoa_grid_bb.h -- the exact branch-and-bound grid solve of one frame by one
// wave (vga_heatmap.h:99-108: max L over cells, first row-major argmax),
// shared by k_grid_bb (tdoa_grid.hip) and the streaming update
// (tdoa_stream.hip).  See DESIGN.md "k_grid_bb".
//
// The distinct tuples are regrouped by the 8 x 8 block of cells their first
// cell lies in (entries of <= 64 tuples, host table, build_bb_tiles); an
// entry's bound is the sum over pairs, in the pair order of L itself, of the
// weighted-score maximum over the entry's lag range for that pair.  Addition
// (float or int64) is monotone in each operand, so the bound is >= the L of
// every tuple of the entry, computed exactly as the exhaustive scan computes it
// (0 + w_0 + w_1 + ...).  The wave evaluates the entry with the largest bound,
// then every entry whose bound is not below the best L found so far; an entry
// whose bound is below it cannot hold a tuple that reaches the maximum, so the
// result (max L, smallest tuple index among equal L) is the exhaustive scan's,
// bit for bit.  Worst case (flat scores): every entry is evaluated.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>

#include "tdoa_fft32.h"
#include "tdoa_internal.h"

namespace tdoa_bb {

// diagnostic build only (TDOA_DIAG): s_memtime cycles per phase accumulated
// per wave -- [1] bounds, [2] seed reduction + seed evaluation, [3] the other
// evaluations, [4] evaluation count (k_grid_bb adds [0] frame loads, [5] frames)
#ifdef TDOA_DIAG
#define BB_T0() unsigned long long bb_t_ = __builtin_amdgcn_s_memtime()
#define BB_MARK(k)                                                 \
    do {                                                           \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
        bbacc[k] += n_ - bb_t_;                                    \
        bb_t_ = n_;                                                \
    } while (0)
#define BB_COUNT(k) (bbacc[k] += 1)
#else
#define BB_T0() \
    do {        \
    } while (0)
#define BB_MARK(k) \
    do {           \
    } while (0)
#define BB_COUNT(k) ((void)0)
#endif

template <typename T> __device__ __forceinline__ T lowest();
template <> __device__ __forceinline__ int64_t lowest<int64_t>() { return INT64_MIN; }
template <> __device__ __forceinline__ float lowest<float>() { return -INFINITY; }

template <typename T> __device__ __forceinline__ T vmax(T a, T b);
template <> __device__ __forceinline__ float vmax<float>(float a, float b) { return fmaxf(a, b); }
template <> __device__ __forceinline__ int64_t vmax<int64_t>(int64_t a, int64_t b) { return a > b ? a : b; }

__device__ __forceinline__ float readlane(float v, int l)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ int64_t readlane(int64_t v, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <typename T>
__device__ __forceinline__ void better(T &bv, int &bu, T ov, int ou)
{
    if (ov > bv || (ov == bv && ou < bu)) {
        bv = ov;
        bu = ou;
    }
}

// (max, first index) across the wave by DPP lane moves -> lane 63 (the
// __shfl_xor butterfly was a chain of twelve LDS round trips per reduction):
// xor 1, xor 2, half-row mirror, row mirror, row_bcast:15, row_bcast:31.
// Lanes without a source keep their own value (old = src).
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_mov(int v)
{
    return __builtin_amdgcn_update_dpp(v, v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ float dpp_mov(float v)
{
    return __builtin_bit_cast(float, dpp_mov<CTRL, RM>(__builtin_bit_cast(int, v)));
}
template <int CTRL, int RM>
__device__ __forceinline__ int64_t dpp_mov(int64_t v)
{
    const uint32_t lo = (uint32_t)dpp_mov<CTRL, RM>((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)dpp_mov<CTRL, RM>((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int CTRL, int RM, typename T>
__device__ __forceinline__ void dpp_better(T &v, int &i)
{
    better<T>(v, i, dpp_mov<CTRL, RM>(v), dpp_mov<CTRL, RM>(i));
}
// the wave's (max, first index) to every lane (float: by keys, tdoa_fft32.h;
// v is never NaN here)
template <typename T>
__device__ __forceinline__ void wave_best(T &v, int &i)
{
    if constexpr (sizeof(T) == 4) {
        int k = fkey(v);
        wave_argmax_key(k, i);
        v = fkey_value(k);
        return;
    }
    dpp_better<0xB1, 0xF>(v, i);
    dpp_better<0x4E, 0xF>(v, i);
    dpp_better<0x141, 0xF>(v, i);
    dpp_better<0x140, 0xF>(v, i);
    dpp_better<0x142, 0xA>(v, i);
    dpp_better<0x143, 0xC>(v, i);
    v = readlane(v, 63);
    i = __builtin_amdgcn_readlane(i, 63);
}

// One frame, one wave.  Wl: the frame's weighted scores [P][K] in LDS (written
// by this wave before the call); M8: a [128] LDS scratch row of this wave;
// tiles / rng: the entry table (LDS or global).  Returns the max L (best) and
// its tuple index in first-cell order (bu, INT_MAX when no L exceeded the
// lowest value).  Every lane returns the same pair.
template <typename T, int TWC, int JT>
__device__ __forceinline__ void solve_wave(const tdoa_kparams &kp, const T *Wl, T *M8,
                                           const int32_t *tiles, const uint16_t *rng, int lane,
                                           T &best_out, int &bu_out, unsigned long long (&bbacc)[8])
{
    (void)bbacc;
    BB_T0();
    const int P = kp.P, K = kp.K, NT = kp.bb_NT, TW = kp.TW;
    const T low = lowest<T>();
    // entry bounds, lane-strided, in L's own pair order
    T bt[JT];
#pragma unroll
    for (int j = 0; j < JT; j++)
        bt[j] = (lane + 64 * j < NT) ? (T)0 : low;
    if (P <= 8) {  // few pairs: a direct range loop
#pragma unroll
        for (int j = 0; j < JT; j++) {
            const int t = lane + 64 * j;
            if (t < NT) {
                T b = 0;
                for (int p = 0; p < P; p++) {
                    const int r = rng[t * P + p], lo = r & 0xFF, hi = r >> 8;
                    const T *w = Wl + p * K;
                    T m = w[lo];
                    for (int k = lo + 1; k <= hi; k++)
                        m = vmax<T>(m, w[k]);
                    b += m;
                }
                bt[j] = b;
            }
        }
    } else {
        // many pairs: per pair the 8-wide running maxima M8[k] = max w[k..k+7]
        // (clamped to K - 1); a range of width <= 16 is max(M8[lo],
        // M8[max(lo, hi - 7)]) -- independent reads, not a dependent chain.
        // (Four pairs' rows per sync measured no faster: the pass is bound
        // by LDS issue, not by its round trips.)
        for (int p = 0; p < P; p++) {
            const T *w = Wl + p * K;
            wave_lds_sync();  // previous pair's M8 reads come first
            for (int k = lane; k < K; k += 64) {
                T m = w[k];
#pragma unroll
                for (int d = 1; d < 8; d++)
                    m = vmax<T>(m, w[k + d < K ? k + d : K - 1]);
                M8[k] = m;
            }
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < JT; j++) {
                const int t = lane + 64 * j;
                if (t < NT) {
                    const int r = rng[t * P + p], lo = r & 0xFF, hi = r >> 8;
                    T m = M8[lo];
                    for (int k = lo + 8; k + 7 < hi; k += 8)  // ranges wider than 16
                        m = vmax<T>(m, M8[k]);
                    m = vmax<T>(m, M8[hi - 7 > lo ? hi - 7 : lo]);
                    bt[j] += m;
                }
            }
        }
    }
    BB_MARK(1);
    // seed: the entry of largest bound (first on ties; NaN bounds never win)
    T sv = low;
    int st = 0;
#pragma unroll
    for (int j = 0; j < JT; j++)
        if (bt[j] > sv) {
            sv = bt[j];
            st = lane + 64 * j;
        }
    wave_best<T>(sv, st);
    const int seed = st;

    T best = low;
    int bu = INT_MAX;
    // evaluate one entry: one tuple per lane; only L > lowest is recorded (the
    // exhaustive scan never records an L equal to its start value)
    auto eval = [&](int t) {
        BB_COUNT(4);
        const int start = tiles[2 * t], cnt = tiles[2 * t + 1];
        T L = low;
        int ui = INT_MAX;
        if (lane < cnt) {
            const int u = start + lane;
            L = 0;
#pragma unroll
            for (int tw = 0; tw < TWC; tw++) {
                if (tw < TW) {
                    const uint32_t word = kp.bb_tuples[(size_t)u * TW + tw];
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const int p = 4 * tw + b;
                        if (p < P)
                            L += Wl[p * K + ((word >> (8 * b)) & 0xFFu)];
                    }
                }
            }
            ui = kp.bb_uidx[u];
        }
        const bool win = L > low && (L > best || (L == best && ui < bu));
        if (__ballot(win) == 0)
            return;
        T v = win ? L : low;
        int vi = win ? ui : INT_MAX;
        wave_best<T>(v, vi);
        best = v;
        bu = vi;
    };
    if (NT > 0)
        eval(seed);
    BB_MARK(2);
#pragma unroll
    for (int j = 0; j < JT; j++) {
        const int t = lane + 64 * j;
        uint64_t mask = __ballot(t < NT && t != seed && !(bt[j] < best));
        while (mask) {
            const int l = __builtin_ctzll(mask);
            mask &= mask - 1;
            if (!(readlane(bt[j], l) < best))  // the best may have risen since
                eval(l + 64 * j);
        }
    }
    BB_MARK(3);
    best_out = best;
    bu_out = bu;
}

}  // namespace tdoa_bb
