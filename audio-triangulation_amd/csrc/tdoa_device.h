// tdoa_device.h -- device phases shared by the engines' kernels:
// staging + integer prep, argmax + lag prior + gate, grid solve.
// Included by exactly one TU per engine (internal linkage), so every engine
// compiles these with its own floating-point flags.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>

#include "tdoa_internal.h"

#ifndef TDOA_GRID_MARK
#define TDOA_GRID_MARK(i) \
    do {                  \
    } while (0)
#endif

namespace {

// 16-B chunk k (8 int16 samples) of row `row` of a frame batch: int16 rows, or
// the streaming batch's 8-bit rows (kp.frames_u8) widened from 8 bytes
__device__ __forceinline__ uint4 frame_chunk(const tdoa_kparams &kp, const int16_t *frames, int64_t row, int k)
{
    if (kp.frames_u8) {
        const uint2 b = reinterpret_cast<const uint2 *>(reinterpret_cast<const uint8_t *>(frames) +
                                                        row * kp.N)[k];
        return make_uint4(__builtin_amdgcn_perm(0u, b.x, 0x0C010C00u), __builtin_amdgcn_perm(0u, b.x, 0x0C030C02u),
                          __builtin_amdgcn_perm(0u, b.y, 0x0C010C00u), __builtin_amdgcn_perm(0u, b.y, 0x0C030C02u));
    }
    return reinterpret_cast<const uint4 *>(frames + row * kp.N)[k];
}

// a streaming slot's frame in the capture ring (kp.frame_ring): its stream's
// bytes (dma_sampler.c:17-23 round-robin), the absolute index of the frame's
// first sample and that sample's ring index
struct RingSlot {
    const uint8_t *cap;
    int64_t t0, j;
};
__device__ __forceinline__ RingSlot ring_slot(const tdoa_kparams &kp, int64_t slot)
{
    RingSlot r;
    r.cap = kp.frame_ring + (size_t)kp.frame_ids[slot] * kp.ring_len * kp.M;
    r.t0 = kp.frame_end[slot] - kp.N;
    r.j = kp.frame_ring_at[slot];
    return r;
}

// chunk k (8 samples) of mic m of that frame: samples j + 8k + i (wrapping at
// ring_len), zero before the stream's first sample -- the bytes the trigger
// scanned (k_stream_trigger_p)
__device__ __forceinline__ uint4 ring_chunk(const tdoa_kparams &kp, const RingSlot &rs, int m, int k)
{
    const int M = kp.M;
    const int64_t cl = kp.ring_len;
    const uint8_t *cap = rs.cap + m;
    const int64_t t0 = rs.t0 + 8 * k;  // absolute index of sample 8k
    int64_t j = rs.j + 8 * k;
    if (j >= cl)
        j -= cl;
    uint32_t b[8];
    if (M == 3 && t0 >= 0 && j + 10 <= cl) {  // the 28 bytes read stay in the ring
        // three mics (config 5): the 22 bytes holding the chunk in two wide
        // loads (7 aligned dwords), shifted to the sample's byte, then every
        // third byte (eight byte loads per chunk bound the staging on the
        // texture units)
        // (the word pointer by pointer arithmetic: an integer-to-pointer cast
        // loses the global address space, and flat loads' waits drain LDS too)
        const uint8_t *ab = cap + j * 3;
        const uint32_t sh = (uint32_t)((uintptr_t)ab & 3u);
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(ab - sh);
        uint32_t w[7];
#pragma unroll
        for (int d = 0; d < 7; d++)
            w[d] = wp[d];
        uint32_t x[6];
#pragma unroll
        for (int d = 0; d < 6; d++)
            x[d] = __builtin_amdgcn_alignbyte(w[d + 1], w[d], sh);
        // sample i is byte 3i of x: 0, 3 | 6, 9 | 12, 15 | 18, 21
        return make_uint4(__builtin_amdgcn_perm(0u, x[0], 0x0C030C00u),
                          __builtin_amdgcn_perm(x[2], x[1], 0x0C050C02u),
                          __builtin_amdgcn_perm(x[3], x[3], 0x0C030C00u),
                          __builtin_amdgcn_perm(x[5], x[4], 0x0C050C02u));
    }
    if (t0 >= 0 && j + 8 <= cl) {
#pragma unroll
        for (int i = 0; i < 8; i++)
            b[i] = cap[(j + i) * M];
    } else {  // the ring's end or the stream's start: sample by sample
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int64_t ji = j + i >= cl ? j + i - cl : j + i;
            b[i] = t0 + i < 0 ? 0u : (uint32_t)cap[ji * M];
        }
    }
    return make_uint4(b[0] | b[1] << 16, b[2] | b[3] << 16, b[4] | b[5] << 16, b[6] | b[7] << 16);
}


__device__ __forceinline__ uint4 ring_chunk(const tdoa_kparams &kp, int64_t slot, int m, int k)
{
    return ring_chunk(kp, ring_slot(kp, slot), m, k);
}

struct NoBetween {
    __device__ void operator()() const {}
};

// Three mics (config 5's streaming batch), a thread's CH chunks c0 + nt i at
// once: every chunk's slot records are requested first, then every chunk's
// ring words, then the bytes are picked -- two dependent round trips after the
// batch count.  Chunk by chunk (ring_chunk), each chunk's record loads and word
// loads sat under the chunk's own branch and were waited on in turn: six round
// trips for three chunks.  between() runs once the records are requested and
// before their values are used (the EMA states' loads go there: their stream
// ids were requested with the records).  Chunks >= nchunk read chunk nchunk - 1's
// words and come back zero; the rare chunks that start before the stream or
// wrap the ring take ring_chunk's byte path.
template <int CH, typename Between>
__device__ __forceinline__ void ring_chunks3(const tdoa_kparams &kp, int64_t f0, int c0, int nt, int nchunk, int cpr,
                                             uint4 (&v)[CH], Between between)
{
    const int64_t cl = kp.ring_len;
    int sid[CH];
    int64_t fe[CH], fa[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
        const int c = c0 + nt * i < nchunk ? c0 + nt * i : nchunk - 1;
        const int64_t slot = f0 + (c / cpr) / 3;
        sid[i] = kp.frame_ids[slot];
        fe[i] = kp.frame_end[slot];
        fa[i] = kp.frame_ring_at[slot];
    }
    between();
    uint32_t wd[CH][7], sh[CH];
    bool fast[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
        const int c = c0 + nt * i < nchunk ? c0 + nt * i : nchunk - 1;
        const int r = c / cpr, k = c - r * cpr, m = r - (r / 3) * 3;
        const int64_t t0 = fe[i] - kp.N + 8 * k;
        int64_t j = fa[i] + 8 * k;
        if (j >= cl)
            j -= cl;
        fast[i] = t0 >= 0 && j + 10 <= cl;
        // (a slow chunk reads its stream's first words instead: in bounds, unused)
        const uint8_t *ab = kp.frame_ring + (size_t)sid[i] * cl * 3 + m + (fast[i] ? j : 0) * 3;
        sh[i] = (uint32_t)((uintptr_t)ab & 3u);
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(ab - sh[i]);
#pragma unroll
        for (int d = 0; d < 7; d++)
            wd[i][d] = wp[d];
    }
    // every chunk's words requested before the first pick waits on any (the
    // scheduler otherwise pulled chunk 0's picks, and a full wait, ahead of
    // chunks 1 and 2's address arithmetic)
    __builtin_amdgcn_sched_barrier(0);
    // (the picks unconditional: under the chunk's branch, the compiler sank the
    // chunk's loads into it, one round trip per chunk again)
#pragma unroll
    for (int i = 0; i < CH; i++) {
        const int c = c0 + nt * i;
        uint32_t x[6];
#pragma unroll
        for (int d = 0; d < 6; d++)
            x[d] = __builtin_amdgcn_alignbyte(wd[i][d + 1], wd[i][d], sh[i]);
        // sample s is byte 3 s of the aligned words (ring_chunk's fast path)
        uint4 q = make_uint4(__builtin_amdgcn_perm(0u, x[0], 0x0C030C00u), __builtin_amdgcn_perm(x[2], x[1], 0x0C050C02u),
                             __builtin_amdgcn_perm(x[3], x[3], 0x0C030C00u), __builtin_amdgcn_perm(x[5], x[4], 0x0C050C02u));
        if (!fast[i] && c < nchunk) {
            // the records read again (rare path): holding them across the
            // word loads cost registers the kernel does not have (an opaque
            // slot index: not merged with the first loads)
            const int r = c / cpr, k = c - r * cpr;
            int64_t slot = f0 + r / 3;
            asm volatile("" : "+v"(slot));
            q = ring_chunk(kp, slot, r - (r / 3) * 3, k);
        }
        v[i] = c < nchunk ? q : make_uint4(0, 0, 0, 0);
    }
}

typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), c,
                                  false);
}

// (x0, x1) int16 pair -> (x0 >> 8, x1 >> 8): signed high bytes (v_pk_ashrrev_i16)
__device__ __forceinline__ uint32_t hi8(uint32_t x)
{
    v2s v = __builtin_bit_cast(v2s, x);
    const v2s sh = {8, 8};
    v = v >> sh;
    return __builtin_bit_cast(uint32_t, v);
}
// (x0 & 255, x1 & 255): unsigned low bytes; x = hi*256 + lo exactly
__device__ __forceinline__ uint32_t lo8(uint32_t x) { return x & 0x00FF00FFu; }

// words (b[2q], b[2q+1]) and (b[2q+2], b[2q+3]) -> (b[2q+1], b[2q+2])
__device__ __forceinline__ uint32_t odd_pair(uint32_t next, uint32_t cur)
{
    return __builtin_amdgcn_alignbit(next, cur, 16);
}

// rolling_buffer.c:65-66, buffer.c:16, buffer.c:8-9 for one sample
__device__ __forceinline__ uint32_t prep_sample(uint32_t x16, uint32_t off16, int32_t w)
{
    const uint32_t y = (x16 - off16) & 0xFFFFu;                    // (int16)(x - off)
    const int32_t z = (int32_t)(int16_t)(uint16_t)((y << 8) & 0xFFFFu);  // x <<= 8
    const int32_t t = z * w;                                         // (int32)x * W[i]
    return (uint32_t)(t >> 15) & 0xFFFFu;                            // (int16)(tmp >> 15)
}

__device__ __forceinline__ uint32_t prep_word(uint32_t v, uint32_t off16, uint32_t wv)
{
    const int32_t w0 = (int32_t)(int16_t)(wv & 0xFFFFu);
    const int32_t w1 = (int32_t)(int16_t)(wv >> 16);
    return prep_sample(v & 0xFFFFu, off16, w0) | (prep_sample(v >> 16, off16, w1) << 16);
}

__device__ __forceinline__ int sum_word(uint32_t v)
{
    return (int)(int16_t)(v & 0xFFFFu) + (int)(int16_t)(v >> 16);
}

struct Smem {
    uint32_t *X;      // [F*M][RS] packed int16 pairs
    int64_t *scores;  // [F*P][K]
    int *sums;        // [F*M]
    int *best;        // [F*P]
    int64_t *redv;    // [nwaves]
    int *redi;        // [nwaves]
};

__device__ __forceinline__ Smem carve(char *smem, const tdoa_kparams &kp, int nwaves)
{
    Smem s;
    size_t o = 0;
    s.X = (uint32_t *)(smem + o);
    o += (size_t)kp.F * kp.M * kp.RS * 4;
    o = (o + 15) & ~(size_t)15;
    s.scores = (int64_t *)(smem + o);
    o += (size_t)kp.F * kp.P * kp.K * 8;
    o = (o + 15) & ~(size_t)15;
    s.redv = (int64_t *)(smem + o);
    o += (size_t)nwaves * 8 * 8;
    s.sums = (int *)(smem + o);
    o += (size_t)kp.F * kp.M * 4;
    s.best = (int *)(smem + o);
    o += (size_t)kp.F * kp.P * 4;
    s.redi = (int *)(smem + o);
    return s;
}

size_t smem_bytes(const tdoa_kparams &kp, int nwaves)
{
    size_t o = (size_t)kp.F * kp.M * kp.RS * 4;
    o = (o + 15) & ~(size_t)15;
    o += (size_t)kp.F * kp.P * kp.K * 8;
    o = (o + 15) & ~(size_t)15;
    o += (size_t)nwaves * 8 * 8;
    o += (size_t)kp.F * kp.M * 4;
    o += (size_t)kp.F * kp.P * 4;
    o += (size_t)nwaves * 8 * 4;
    return (o + 15) & ~(size_t)15;
}

// ------------------------------------------------------------------ stage
template <bool PREPARED>
__device__ void stage_frames(const tdoa_kparams &kp, const Smem &sm, const int16_t *__restrict__ frames,
                             int64_t f0, int nf)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int rows = nf * kp.M, NW = kp.N / 2, padw = kp.PADW, RS = kp.RS;
    for (int i = tid; i < rows * 2 * padw; i += nt) {
        const int r = i / (2 * padw), k = i - r * 2 * padw;
        sm.X[r * RS + (k < padw ? k : NW + k)] = 0u;
    }
    for (int i = tid; i < rows; i += nt)
        sm.sums[i] = 0;
    __syncthreads();

    const int cpr = kp.N / 8;  // 16-byte chunks per row
    const uint4 *src = reinterpret_cast<const uint4 *>(frames + f0 * kp.M * kp.N);
    const int nchunk = rows * cpr;
    const int width = cpr < 64 ? cpr : 64;  // lanes of one wave that share a row
    for (int c0 = 0; c0 < nchunk; c0 += nt) {
        const int c = c0 + tid;
        const bool ok = c < nchunk;
        uint4 v = make_uint4(0, 0, 0, 0);
        int r = 0;
        if (ok) {
            r = c / cpr;
            const int k = c - r * cpr;
            if (kp.frame_ring) {  // streaming batch: frame f0 + r / M from its stream's ring
                const int fl = r / kp.M, m = r - fl * kp.M;
                v = ring_chunk(kp, f0 + fl, m, k);
            } else if (kp.frames_u8) {
                v = frame_chunk(kp, frames, f0 * kp.M + r, k);
            } else {
                v = src[c];
            }
            *reinterpret_cast<uint4 *>(&sm.X[r * RS + padw + 4 * k]) = v;
        }
        if (!PREPARED) {
            int s = sum_word(v.x) + sum_word(v.y) + sum_word(v.z) + sum_word(v.w);
            for (int m = 1; m < width; m <<= 1)
                s += __shfl_xor(s, m, 64);
            if (ok && (tid & (width - 1)) == 0)
                atomicAdd(&sm.sums[r], s);
        }
    }
    __syncthreads();
    if (PREPARED)
        return;
    const uint4 *win = reinterpret_cast<const uint4 *>(kp.window);
    for (int c = tid; c < nchunk; c += nt) {
        const int r = c / cpr, k = c - r * cpr;
        // floor mean: int64 `total >> BITS` == int32 arithmetic shift here
        const uint32_t off16 = (uint32_t)(sm.sums[r] >> kp.log2N) & 0xFFFFu;
        uint4 *p = reinterpret_cast<uint4 *>(&sm.X[r * RS + padw + 4 * k]);
        uint4 v = *p;
        const uint4 w = win[k];
        v.x = prep_word(v.x, off16, w.x);
        v.y = prep_word(v.y, off16, w.y);
        v.z = prep_word(v.z, off16, w.z);
        v.w = prep_word(v.w, off16, w.w);
        *p = v;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ xcorr
// One work item = (frame f, pair p, lag tile t, segment g): 16 lags
// s0..s0+15 (s0 even) over words [g*SEGW, (g+1)*SEGW) of the a-row.
//   even lag s0+2e : a-word w . b-word (w + h + e)               (h = s0/2)
//   odd  lag s0+2e+1: a-word w . (b[2(w+h+e)+1], b[2(w+h+e)+2])
// The b-side words sit in an 8-slot register ring (slot (r+e)&7 holds
// q = w+h+e at unrolled step r), split into hi/lo byte pairs.
__device__ void xcorr_phase(const tdoa_kparams &kp, const Smem &sm, int nf)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int NSEG = kp.NSEG, T = kp.T, P = kp.P;
    const int total = nf * P * T * NSEG;
    for (int base = 0; base < total; base += nt) {
        const int item = base + tid;
        const bool valid = item < total;
        const int it = valid ? item : 0;
        const int g = it % NSEG;
        int rest = it / NSEG;
        const int t = rest % T;
        rest /= T;
        const int p = rest % P;
        const int f = rest / P;
        const uint32_t *A = sm.X + (f * kp.M + kp.pair_i[p]) * kp.RS + kp.PADW;
        const uint32_t *Bw = sm.X + (f * kp.M + kp.pair_j[p]) * kp.RS + kp.PADW;
        const int s0 = kp.sbase + TDOA_LT * t;
        const int h = s0 / 2;
        const int w0 = g * TDOA_SEGW;

        uint32_t EH[TDOA_LT2], EL[TDOA_LT2], OH[TDOA_LT2], OL[TDOA_LT2];
        int aEH[TDOA_LT2], aEL[TDOA_LT2], aOH[TDOA_LT2], aOL[TDOA_LT2];
        uint32_t last;
        {
            uint32_t raw[TDOA_LT2 + 1];
#pragma unroll
            for (int e = 0; e <= TDOA_LT2; e++)
                raw[e] = Bw[w0 + h + e];
#pragma unroll
            for (int e = 0; e < TDOA_LT2; e++) {
                EH[e] = hi8(raw[e]);
                EL[e] = lo8(raw[e]);
                const uint32_t o = odd_pair(raw[e + 1], raw[e]);
                OH[e] = hi8(o);
                OL[e] = lo8(o);
                aEH[e] = aEL[e] = aOH[e] = aOL[e] = 0;
            }
            last = raw[TDOA_LT2];
        }
        for (int wb = 0; wb < TDOA_SEGW; wb += TDOA_LT2) {
#pragma unroll
            for (int r = 0; r < TDOA_LT2; r++) {
                const int w = w0 + wb + r;
                const uint32_t a = A[w];
#pragma unroll
                for (int e = 0; e < TDOA_LT2; e++) {
                    const int sl = (r + e) & (TDOA_LT2 - 1);
                    aEH[e] = dot2(a, EH[sl], aEH[e]);
                    aEL[e] = dot2(a, EL[sl], aEL[e]);
                    aOH[e] = dot2(a, OH[sl], aOH[e]);
                    aOL[e] = dot2(a, OL[sl], aOL[e]);
                }
                const uint32_t nb = Bw[w + h + TDOA_LT2 + 1];
                EH[r] = hi8(last);
                EL[r] = lo8(last);
                const uint32_t o = odd_pair(nb, last);
                OH[r] = hi8(o);
                OL[r] = lo8(o);
                last = nb;
            }
        }
        // widen (hi*256 + lo), sum the NSEG segments of this (f, p, t)
        int64_t vals[TDOA_LT];
#pragma unroll
        for (int e = 0; e < TDOA_LT2; e++) {
            vals[2 * e] = (int64_t)aEH[e] * 256 + aEL[e];
            vals[2 * e + 1] = (int64_t)aOH[e] * 256 + aOL[e];
        }
        for (int m = 1; m < NSEG; m <<= 1) {
#pragma unroll
            for (int u = 0; u < TDOA_LT; u++)
                vals[u] += __shfl_xor(vals[u], m, 64);
        }
        if (valid && g == 0) {
            int64_t *dst = sm.scores + (f * P + p) * kp.K + kp.S;
#pragma unroll
            for (int u = 0; u < TDOA_LT; u++) {
                const int s = s0 + u;
                if (s >= -kp.S && s <= kp.S)
                    dst[s] = vals[u];
            }
        }
    }
    __syncthreads();
}

// -------------------------------------------------- argmax + lag prior + gate
// One wave per (frame, pair): first strictly-greater lag (correlations.c:20-23),
// then weighted = score * scale[|s - best|] (correlations.c:26-33: for int64
// scores (int64)((float)score * scale), truncating; float scores stay float).
__device__ __forceinline__ void store_score(const tdoa_kout &o, size_t i, int64_t raw, int64_t w)
{
    if (o.scores)
        o.scores[i] = raw;
    if (o.weighted)
        o.weighted[i] = w;
}
__device__ __forceinline__ void store_score(const tdoa_kout &o, size_t i, float raw, float w)
{
    if (o.scores_f)
        o.scores_f[i] = raw;
    if (o.weighted_f)
        o.weighted_f[i] = w;
}
__device__ __forceinline__ int64_t apply_prior(int64_t v, float scale)
{
    const float x = (float)v * scale;
    return (int64_t)x;
}
__device__ __forceinline__ float apply_prior(float v, float scale) { return v * scale; }

template <typename T> __device__ __forceinline__ T lowest();
template <> __device__ __forceinline__ int64_t lowest<int64_t>() { return INT64_MIN; }
template <> __device__ __forceinline__ float lowest<float>() { return -INFINITY; }

template <typename T>
__device__ void argmax_prior_phase(const tdoa_kparams &kp, T *scores, int *bestlag,
                                   const tdoa_kout &out, int64_t f0, int nf,
                                   const float *prior_tab = nullptr)
{
    const float *prior = prior_tab ? prior_tab : kp.prior;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P;
    for (int fp = wave; fp < nf * P; fp += nwaves) {
        T *sc = scores + fp * K;
        const int k1 = lane, k2 = lane + 64;
        const T v1 = k1 < K ? sc[k1] : lowest<T>();
        const T v2 = k2 < K ? sc[k2] : lowest<T>();
        T bv = v1;
        int bk = k1;
        if (v2 > bv) {
            bv = v2;
            bk = k2;
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const T ov = __shfl_xor(bv, m, 64);
            const int ok = __shfl_xor(bk, m, 64);
            if (ov > bv || (ov == bv && ok < bk)) {
                bv = ov;
                bk = ok;
            }
        }
        const size_t gbase = (size_t)(f0 * P + fp) * K;
        if (k1 < K) {
            const int d = k1 > bk ? k1 - bk : bk - k1;
            const T wv = apply_prior(v1, prior[d]);
            sc[k1] = wv;
            store_score(out, gbase + k1, v1, wv);
        }
        if (k2 < K) {
            const int d = k2 > bk ? k2 - bk : bk - k2;
            const T wv = apply_prior(v2, prior[d]);
            sc[k2] = wv;
            store_score(out, gbase + k2, v2, wv);
        }
        if (lane == 0) {
            bestlag[fp] = bk - kp.S;
            out.lags[f0 * P + fp] = bk - kp.S;
        }
    }
    __syncthreads();
    if (out.gate) {
        for (int f = tid; f < nf; f += blockDim.x) {
            int tot = 0;
            for (int p = 0; p < P; p++) {
                const int b = bestlag[f * P + p];
                tot += b * b;
            }
            out.gate[f0 + f] = tot > 4 ? 1 : 0;
        }
    }
}

// ------------------------------------------------------------- grid solve
// All F frames of the workgroup in one sweep over the distinct lag tuples:
// every tuple word is loaded once and scored for each frame, then one
// (max L, first tuple) reduction per frame.  Tuples are in first-cell order,
// so the smallest tuple index among the maxima carries the first row-major
// argmax cell of vga_heatmap.h:99-108.
#define TDOA_FMAX 8
template <typename T>
__device__ __forceinline__ void better(T &bv, int &bu, T ov, int ou)
{
    if (ov > bv || (ov == bv && ou < bu)) {
        bv = ov;
        bu = ou;
    }
}

__device__ __forceinline__ void store_max(const tdoa_kout &o, int64_t i, int64_t v)
{
    if (o.max_L)
        o.max_L[i] = v;
}
__device__ __forceinline__ void store_max(const tdoa_kout &o, int64_t i, float v)
{
    if (o.max_Lf)
        o.max_Lf[i] = v;
}

template <typename T, int FMAX = TDOA_FMAX, int TWC = (TDOA_MAX_PAIRS + 3) / 4>
__device__ void grid_phase_t(const tdoa_kparams &kp, const T *scores, T *redv, int *redi,
                             const tdoa_kout &out, int64_t f0, int nf,
                             const uint32_t *tuples = nullptr, const int32_t *cells = nullptr,
                             uint32_t omask = 0xFFFFFFFFu)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int nt = blockDim.x;
    const int K = kp.K, P = kp.P, TW = kp.TW, U = kp.U;
    const uint32_t *tup = tuples ? tuples : kp.tuples;
    T bv[FMAX];
    int bu[FMAX];
#pragma unroll
    for (int f = 0; f < FMAX; f++) {
        bv[f] = lowest<T>();
        bu[f] = INT_MAX;
    }
    // UNR tuples in flight per thread; each thread's u still increases, so a
    // strict '>' keeps its first maximum
    constexpr int UNR = TWC == 1 ? 4 : 1;
    for (int u0 = tid; u0 < U; u0 += UNR * nt) {
        uint32_t wd[UNR][TWC];
#pragma unroll
        for (int r = 0; r < UNR; r++) {
            const int u = u0 + r * nt;
#pragma unroll
            for (int tw = 0; tw < TWC; tw++)
                wd[r][tw] = (u < U && tw < TW) ? tup[u * TW + tw] : 0u;
        }
#pragma unroll
        for (int r = 0; r < UNR; r++) {
            const int u = u0 + r * nt;
            if (u >= U)
                break;
            T L[FMAX];
#pragma unroll
            for (int f = 0; f < FMAX; f++)
                L[f] = 0;
#pragma unroll
            for (int tw = 0; tw < TWC; tw++) {
                const uint32_t word = wd[r][tw];
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int p = 4 * tw + b;
                    if (p < P) {
                        const int idx = p * K + ((word >> (8 * b)) & 0xFFu);
#pragma unroll
                        for (int f = 0; f < FMAX; f++)
                            if (f < nf)
                                L[f] += scores[f * P * K + idx];
                    }
                }
            }
#pragma unroll
            for (int f = 0; f < FMAX; f++)
                if (L[f] > bv[f]) {
                    bv[f] = L[f];
                    bu[f] = u;
                }
        }
    }
    TDOA_GRID_MARK(8);
#pragma unroll
    for (int f = 0; f < FMAX; f++) {
        if (f < nf) {
            for (int m = 32; m >= 1; m >>= 1)
                better(bv[f], bu[f], __shfl_xor(bv[f], m, 64), __shfl_xor(bu[f], m, 64));
            if (lane == 0) {
                redv[wave * FMAX + f] = bv[f];
                redi[wave * FMAX + f] = bu[f];
            }
        }
    }
    __syncthreads();
    TDOA_GRID_MARK(9);
    if (tid < nf && ((omask >> tid) & 1u)) {  // omask: the frames whose outputs are written
        const int f = tid;
        T v = redv[f];
        int ui = redi[f];
        for (int w = 1; w < nwaves; w++)
            better(v, ui, redv[w * FMAX + f], redi[w * FMAX + f]);
        if (ui < 0 || ui >= U)  // only if every L compared false (NaN scores)
            ui = 0;
        const int cell = cells ? cells[ui] : kp.tuple_cell[ui];
        const int64_t fi = f0 + f;
        if (out.cell)
            out.cell[fi] = cell;
        store_max(out, fi, v);
        if (out.xy) {
            const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
            out.xy[2 * fi] = (float)(cx - kp.half_w) / kp.grid_scale;
            out.xy[2 * fi + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
        }
    }
}

template <int TWC>
__device__ void grid_phase(const tdoa_kparams &kp, const Smem &sm, const tdoa_kout &out,
                           int64_t f0, int nf)
{
    if (!out.cell && !out.xy && !out.max_L && !out.max_Lf)
        return;
    grid_phase_t<int64_t, TDOA_FMAX, TWC>(kp, sm.scores, sm.redv, sm.redi, out, f0, nf);
}


}  // namespace
