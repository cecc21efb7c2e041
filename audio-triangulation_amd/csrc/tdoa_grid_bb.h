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

// many pairs, P % 4 == 0: the bounds' queries unguarded (see solve_wave)
#ifndef BB_Q4
#define BB_Q4 1
#endif
// the evaluations' loads and gathers unguarded (see solve_wave)
#ifndef BB_EV
#define BB_EV 1
#endif

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

// row stride of the grouped levels (P > 8): 8 lags per lane, 12 or 16 lanes
__host__ __device__ constexpr int bb_row(int K) { return K <= 96 ? 96 : 128; }
// row stride of the frame's scores in LDS: K, or K rounded up to 16 B for many
// pairs (P > 8), whose level build then reads a lane's 16 scores as four
// aligned 16-B reads and whose compact chunks expand by one 16-B store each
__host__ __device__ constexpr int bb_ks(int P, int K) { return P > 8 ? (K + 3) & ~3 : K; }
// the frame's scores per wave, padded to 16 B: the levels follow them
__host__ __device__ constexpr int bb_pk(int P, int K) { return (P * bb_ks(P, K) + 3) & ~3; }

// LDS scratch elements per wave after the frame's scores: the sparse table's
// levels 1, 2, 3 [3][P][K] (P <= 8, bb_pk apart), or the same levels of four
// pairs at a time [3][4][row] otherwise
__host__ __device__ constexpr int bb_scratch(int P, int K)
{
    return P <= 8 ? 3 * bb_pk(P, K) : 3 * 4 * bb_row(K);
}

// the level-j sparse table: S_j[i] = max w[i .. i + 2^j - 1], so the maximum
// over a range of width n, 2^j <= n < 2^(j+1), is exactly
// max(S_j[lo], S_j[hi + 1 - 2^j]) -- two independent reads.  The host encodes
// every (entry, pair) range as that query (bb_query, tdoa_capi.cpp: offset of
// the first window from the scores, distance of the second); a window never
// crosses its pair's row, both lie inside [lo, hi].  Tables with a range wider
// than 15 lags take the exhaustive k_grid (kp.bb_wide; configs 3 / 4: <= 11 / 15).
template <typename T>
__device__ __forceinline__ T bb_range_max(const T *Wl, uint32_t q)
{
    const int o1 = (int)(q & 0x1FFFu), dl = (int)(q >> 13);
    return vmax<T>(Wl[o1], Wl[o1 + dl]);
}

// One frame, one wave.  Wl: the frame's weighted scores [P][KS] in LDS (written
// by this wave before the call), followed by bb_scratch(P, K) scratch
// elements (16-B aligned); qt: the entries' range queries [NT][P];
// tiles: the entry table (global: an entry index is wave-uniform).  Returns the max L (best) and
// its tuple index in first-cell order (bu, INT_MAX when no L exceeded the
// lowest value).  Every lane returns the same pair.
template <typename T, int TWC, int JT>
__device__ __forceinline__ void solve_wave(const tdoa_kparams &kp, T *Wl, const int32_t *tiles,
                                           const uint16_t *qt, int lane, T &best_out, int &bu_out,
                                           unsigned long long (&bbacc)[8])
{
    (void)bbacc;
    BB_T0();
    const int P = kp.P, K = kp.K, NT = kp.bb_NT, TW = kp.TW, PKp = bb_pk(P, K), KS = bb_ks(P, K);
    const T low = lowest<T>();
    // entry bounds, lane-strided, in L's own pair order
    T bt[JT];
#pragma unroll
    for (int j = 0; j < JT; j++)
        bt[j] = (lane + 64 * j < NT) ? (T)0 : low;
    // TWC <= 2 instantiations take TW <= 2 tables (P <= 8, tdoa_grid.hip), the
    // others P > 8: one path per instantiation
    if constexpr (TWC <= 2) {
        // few pairs: levels 1, 2, 3 of every pair in three wave-synced passes
        // (the range loop they replace issued n dependent reads per range: 69 %
        // of a config-3 wave)
        const int PK = P * K;
        T *S2 = Wl + PKp, *S4 = S2 + PKp, *S8 = S4 + PKp;
        for (int i = lane; i < PK; i += 64)
            S2[i] = vmax<T>(Wl[i], Wl[i + 1 < PK ? i + 1 : i]);
        wave_lds_sync();
        for (int i = lane; i < PK; i += 64)
            S4[i] = vmax<T>(S2[i], S2[i + 2 < PK ? i + 2 : i]);
        wave_lds_sync();
        for (int i = lane; i < PK; i += 64)
            S8[i] = vmax<T>(S4[i], S4[i + 4 < PK ? i + 4 : i]);
        wave_lds_sync();
#if BB_Q4
        if (NT > 0) {
            // every lane and pair slot reads (entry clamped to NT - 1, pair to
            // P - 1), an entry's windows all before its first max; the sum
            // takes p < P
#pragma unroll
            for (int j = 0; j < JT; j++) {
                T wa[8], wb[8];
                const int t = lane + 64 * j < NT ? lane + 64 * j : NT - 1;
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    const uint32_t q = qt[t * P + (p < P ? p : P - 1)];
                    const int o1 = (int)(q & 0x1FFFu), dl = (int)(q >> 13);
                    wa[p] = Wl[o1];
                    wb[p] = Wl[o1 + dl];
                }
                __builtin_amdgcn_sched_barrier(0);
                T b = 0;
#pragma unroll
                for (int p = 0; p < 8; p++)
                    if (p < P)  // bounds summed in L's own pair order
                        b += vmax<T>(wa[p], wb[p]);
                bt[j] = lane + 64 * j < NT ? b : low;
            }
        }
        if (false)
#endif
#pragma unroll
        for (int j = 0; j < JT; j++) {
            const int t = lane + 64 * j;
            if (t < NT) {
                T mp[8];
#pragma unroll
                for (int p = 0; p < 8; p++)
                    if (p < P)
                        mp[p] = bb_range_max<T>(Wl, qt[t * P + p]);
                T b = 0;
#pragma unroll
                for (int p = 0; p < 8; p++)
                    if (p < P)  // bounds summed in L's own pair order
                        b += mp[p];
                bt[j] = b;
            }
        }
    } else {
        // many pairs: the same levels, four pairs per wave sync (all P pairs'
        // levels would take 3 P K scratch elements per wave: occupancy).  Lane
        // 16 g + q builds lags k = 8q .. 8q + 7 of pair p0 + g at levels 1, 2, 3
        // from 15 reads (14 + 12 + 8 maxima, six 16-B stores).  Round 2's
        // 8-wide maxima alone answered ranges narrower than 8 with
        // max w[lo .. lo + 7] -- valid but loose bounds: 3.03 entry evaluations
        // per config-4 frame against 1.87 with exact ones
        const int RW = bb_row(K), gq = lane >> 4, q8 = 8 * (lane & 15);
        T *G = Wl + PKp;  // [3][4][RW]
#if BB_Q4
        // P % 4 == 0: every lane queries (lanes past NT repeat entry NT - 1 and
        // are masked after the loop), with no per-pair guard, so a group's
        // query words and range reads issue together instead of one pair's
        // round trip after another; the next group's words are requested a
        // group ahead
        const bool q4 = (P & 3) == 0 && NT > 0;
        int tq[JT];
#pragma unroll
        for (int j = 0; j < JT; j++)
            tq[j] = lane + 64 * j < NT ? lane + 64 * j : NT - 1;
        uint2 qn[JT];
        if (q4) {
#pragma unroll
            for (int j = 0; j < JT; j++) {
                qn[j] = *reinterpret_cast<const uint2 *>(qt + tq[j] * P);
                bt[j] = (T)0;
            }
        }
#endif
        for (int p0 = 0; p0 < P; p0 += 4) {
            wave_lds_sync();  // the previous group's level reads come first
            if (p0 + gq < P && q8 < RW) {
                const T *w = Wl + (p0 + gq) * KS;
                T x[16];
                // lags q8 .. q8 + 15 as aligned 16-B reads (KS and q8 multiples
                // of 4; past the row's K lags they read the next row or the
                // levels: windows there are never queried, a query's windows lie
                // inside its range)
                constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
                for (int v = 0; v < 16 / PER; v++) {
                    const uint4 u = *reinterpret_cast<const uint4 *>(w + q8 + v * PER);
                    __builtin_memcpy(&x[v * PER], &u, 16);
                }
                // in place, each level stored as soon as it is built (few live values)
                T *dst = G + gq * RW + q8;
#pragma unroll
                for (int d = 0; d < 14; d++)
                    x[d] = vmax<T>(x[d], x[d + 1]);
#pragma unroll
                for (int d = 0; d < 8; d++)
                    dst[d] = x[d];
#pragma unroll
                for (int d = 0; d < 12; d++)
                    x[d] = vmax<T>(x[d], x[d + 2]);
#pragma unroll
                for (int d = 0; d < 8; d++)
                    dst[4 * RW + d] = x[d];
#pragma unroll
                for (int d = 0; d < 8; d++)
                    x[d] = vmax<T>(x[d], x[d + 4]);
#pragma unroll
                for (int d = 0; d < 8; d++)
                    dst[8 * RW + d] = x[d];
            }
            wave_lds_sync();
#if BB_Q4
            if (q4) {
                uint2 qc[JT];
#pragma unroll
                for (int j = 0; j < JT; j++) {
                    qc[j] = qn[j];
                    if (p0 + 4 < P)
                        qn[j] = *reinterpret_cast<const uint2 *>(qt + tq[j] * P + p0 + 4);
                }
                // every window read issued before the first max (the scheduler
                // otherwise waits on each range's two reads in turn)
                T wa[JT][4], wb[JT][4];
#pragma unroll
                for (int j = 0; j < JT; j++)
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        const uint32_t q = ((g < 2 ? qc[j].x : qc[j].y) >> (16 * (g & 1))) & 0xFFFFu;
                        const int o1 = (int)(q & 0x1FFFu), dl = (int)(q >> 13);
                        wa[j][g] = Wl[o1];
                        wb[j][g] = Wl[o1 + dl];
                    }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < JT; j++)
#pragma unroll
                    for (int g = 0; g < 4; g++)  // bounds summed in L's own pair order
                        bt[j] += vmax<T>(wa[j][g], wb[j][g]);
                continue;
            }
#endif
#pragma unroll
            for (int j = 0; j < JT; j++) {
                const int t = lane + 64 * j;
                if (t < NT) {
                    // the group's four queries in one 8-B read (P % 4 == 0: aligned)
                    uint32_t qg[4];
                    if ((P & 3) == 0) {
                        const uint2 qq = *reinterpret_cast<const uint2 *>(qt + t * P + p0);
                        qg[0] = qq.x & 0xFFFFu;
                        qg[1] = qq.x >> 16;
                        qg[2] = qq.y & 0xFFFFu;
                        qg[3] = qq.y >> 16;
                    } else {
#pragma unroll
                        for (int g = 0; g < 4; g++)
                            qg[g] = p0 + g < P ? qt[t * P + p0 + g] : 0u;
                    }
                    T mp[4];
#pragma unroll
                    for (int g = 0; g < 4; g++)
                        if (p0 + g < P)
                            mp[g] = bb_range_max<T>(Wl, qg[g]);
#pragma unroll
                    for (int g = 0; g < 4; g++)
                        if (p0 + g < P)  // bounds summed in L's own pair order
                            bt[j] += mp[g];
                }
            }
        }
#if BB_Q4
        if (q4)
#pragma unroll
            for (int j = 0; j < JT; j++)
                if (lane + 64 * j >= NT)
                    bt[j] = low;
#endif
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
    // an entry's evaluation in two halves: fetch (its tuple words and indices,
    // one tuple per lane, from L2) and consume (the gathers, L, the wave's
    // best).  Only L > lowest is recorded (the exhaustive scan never records an
    // L equal to its start value).
    struct Pre {
        uint32_t w[TWC];
        int ui, cnt;
    };
#if BB_EV
    // unguarded: the entry's (start, count) as one uniform load, every lane's
    // words and index requested at once (lanes past the count load the
    // entry's first tuple; their L is masked), and every gather issued before
    // the first add -- guarded, each load or gather was its own round trip
    auto fetch = [&](int t, Pre &pr) {
        const int2 tc = *reinterpret_cast<const int2 *>(tiles + 2 * t);
        pr.cnt = tc.y;
        const int u = tc.x + (lane < tc.y ? lane : 0);
#pragma unroll
        for (int tw = 0; tw < TWC; tw++)
            pr.w[tw] = kp.bb_tuples[(size_t)u * TW + (tw < TW ? tw : TW - 1)];
        const int ui = kp.bb_uidx[u];
        pr.ui = lane < tc.y ? ui : INT_MAX;
    };
    auto consume = [&](const Pre &pr) {
        BB_COUNT(4);
        T g[4 * TWC];
#pragma unroll
        for (int p = 0; p < 4 * TWC; p++)  // pairs past P read row 0 (not summed)
            g[p] = Wl[(p < P ? p * KS : 0) + ((pr.w[p >> 2] >> (8 * (p & 3))) & 0xFFu)];
        __builtin_amdgcn_sched_barrier(0);
        T L = 0;
        if (P == 4 * TWC) {
#pragma unroll
            for (int p = 0; p < 4 * TWC; p++)
                L += g[p];
        } else {
#pragma unroll
            for (int p = 0; p < 4 * TWC; p++)
                if (p < P)
                    L += g[p];
        }
        L = lane < pr.cnt ? L : low;
#else
    auto fetch = [&](int t, Pre &pr) {
        const int start = tiles[2 * t];
        pr.cnt = tiles[2 * t + 1];
        pr.ui = INT_MAX;
        if (lane < pr.cnt) {
            const int u = start + lane;
#pragma unroll
            for (int tw = 0; tw < TWC; tw++)
                if (tw < TW)
                    pr.w[tw] = kp.bb_tuples[(size_t)u * TW + tw];
            pr.ui = kp.bb_uidx[u];
        }
    };
    auto consume = [&](const Pre &pr) {
        BB_COUNT(4);
        T L = low;
        if (lane < pr.cnt) {
            L = 0;
#pragma unroll
            for (int tw = 0; tw < TWC; tw++) {
                if (tw < TW) {
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const int p = 4 * tw + b;
                        if (p < P)
                            L += Wl[p * KS + ((pr.w[tw] >> (8 * b)) & 0xFFu)];
                    }
                }
            }
        }
#endif
        const int ui = pr.ui;
        const bool win = L > low && (L > best || (L == best && ui < bu));
        if (__ballot(win) == 0)
            return;
        T v = win ? L : low;
        int vi = win ? ui : INT_MAX;
        wave_best<T>(v, vi);
        best = v;
        bu = vi;
    };
    Pre pa, pb;
    if (NT > 0) {
        fetch(seed, pa);
        consume(pa);
    }
    BB_MARK(2);
    // the other entries whose bound is not below the best, in entry order,
    // software-pipelined by one: the next candidate's words are in flight
    // while this one is consumed (the buffers alternate: a register copy of a
    // pending load would wait for it).  A candidate is re-checked against the
    // best before it is consumed -- the best may have risen since.
    uint64_t mk[JT];
#pragma unroll
    for (int j = 0; j < JT; j++)
        mk[j] = __ballot(lane + 64 * j < NT && lane + 64 * j != seed && !(bt[j] < best));
    auto pop = [&]() -> int {  // straight-line (an early return indexed mk in scratch)
        int r = -1;
#pragma unroll
        for (int j = 0; j < JT; j++) {
            const bool take = r < 0 && mk[j] != 0;
            if (take)
                r = __builtin_ctzll(mk[j]) + 64 * j;
            mk[j] = take ? mk[j] & (mk[j] - 1) : mk[j];
        }
        return r;
    };
    auto bound_of = [&](int t) -> T {
        T b = low;
#pragma unroll
        for (int j = 0; j < JT; j++)
            if ((t >> 6) == j)
                b = readlane(bt[j], t & 63);
        return b;
    };
    int cur = pop();
    if (cur >= 0)
        fetch(cur, pa);
    while (cur >= 0) {
        int nx = pop();
        if (nx >= 0)
            fetch(nx, pb);
        if (!(bound_of(cur) < best))
            consume(pa);
        cur = nx;
        if (cur < 0)
            break;
        nx = pop();
        if (nx >= 0)
            fetch(nx, pa);
        if (!(bound_of(cur) < best))
            consume(pb);
        cur = nx;
    }
    BB_MARK(3);
    best_out = best;
    bu_out = bu;
}

}  // namespace tdoa_bb
