// tdoa_kernels.hip -- gfx950 kernels of the TDOA hot path.
//
// k_direct: one launch runs, for F frames per workgroup,
//   stage      coalesced 16-B loads of int16 [M][N] rows into LDS, per-row
//              floor-mean DC removal (rolling_buffer.c:64-66), <<8 int16 wrap
//              (buffer.c:13-16), Q15 window (buffer.c:4-11), in place
//   xcorr      exact int64 cross-correlation for every pair and lag
//              (correlations.c:9-18) with packed v_dot2_i32_i16: one operand
//              is split into a signed high byte and an unsigned low byte so
//              every int32 partial is exact; partials widen to int64 once
//   argmax     first strictly-greater lag (correlations.c:20-23), wave shuffle
//   prior      (int64)((float)score * scale[|s-best|]) (correlations.c:26-33)
//   gate       sum_p best^2 > 4 (sample_compute.h:124-134)
//   grid       L = sum_p corr_p[LUT_p] max pass (vga_heatmap.h:99-108) over
//              the distinct lag tuples of the grid, first row-major argmax
// k_average: the EMA of correlations.c:38-63 for S independent streams.
//
// Built with -ffp-contract=off: the float steps must round exactly as the
// reference's IEEE host build does.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

#ifdef TDOA_DIAG
// Diagnostic build only (libtdoa_diag.so): per-workgroup phase stamps.
#define TDOA_DIAG_SLOTS 8
__device__ unsigned long long g_diag[1 << 20];
#define DIAG_STAMP(i)                                                   \
    do {                                                                \
        if (threadIdx.x == 0)                                           \
            g_diag[(size_t)blockIdx.x * TDOA_DIAG_SLOTS + (i)] =        \
                __builtin_amdgcn_s_memtime();                           \
    } while (0)
#else
#define DIAG_STAMP(i) \
    do {              \
    } while (0)
#endif

namespace {

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
            v = src[c];
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
                                   const tdoa_kout &out, int64_t f0, int nf)
{
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
            const T wv = apply_prior(v1, kp.prior[d]);
            sc[k1] = wv;
            store_score(out, gbase + k1, v1, wv);
        }
        if (k2 < K) {
            const int d = k2 > bk ? k2 - bk : bk - k2;
            const T wv = apply_prior(v2, kp.prior[d]);
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

template <typename T>
__device__ void grid_phase_t(const tdoa_kparams &kp, const T *scores, T *redv, int *redi,
                             const tdoa_kout &out, int64_t f0, int nf)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P, TW = kp.TW, U = kp.U;
    T bv[TDOA_FMAX];
    int bu[TDOA_FMAX];
#pragma unroll
    for (int f = 0; f < TDOA_FMAX; f++) {
        bv[f] = lowest<T>();
        bu[f] = INT_MAX;
    }
    for (int u = tid; u < U; u += blockDim.x) {
        T L[TDOA_FMAX];
#pragma unroll
        for (int f = 0; f < TDOA_FMAX; f++)
            L[f] = 0;
        for (int tw = 0; tw < TW; tw++) {
            const uint32_t word = kp.tuples[u * TW + tw];
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int p = 4 * tw + b;
                if (p < P) {
                    const int idx = p * K + ((word >> (8 * b)) & 0xFFu);
#pragma unroll
                    for (int f = 0; f < TDOA_FMAX; f++)
                        if (f < nf)
                            L[f] += scores[f * P * K + idx];
                }
            }
        }
#pragma unroll
        for (int f = 0; f < TDOA_FMAX; f++)
            if (L[f] > bv[f]) {  // u increases per thread: strict > keeps the first
                bv[f] = L[f];
                bu[f] = u;
            }
    }
#pragma unroll
    for (int f = 0; f < TDOA_FMAX; f++) {
        if (f < nf) {
            for (int m = 32; m >= 1; m >>= 1)
                better(bv[f], bu[f], __shfl_xor(bv[f], m, 64), __shfl_xor(bu[f], m, 64));
            if (lane == 0) {
                redv[wave * TDOA_FMAX + f] = bv[f];
                redi[wave * TDOA_FMAX + f] = bu[f];
            }
        }
    }
    __syncthreads();
    if (tid < nf) {
        const int f = tid;
        T v = redv[f];
        int ui = redi[f];
        for (int w = 1; w < nwaves; w++)
            better(v, ui, redv[w * TDOA_FMAX + f], redi[w * TDOA_FMAX + f]);
        const int cell = kp.tuple_cell[ui];
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

__device__ void grid_phase(const tdoa_kparams &kp, const Smem &sm, const tdoa_kout &out,
                           int64_t f0, int nf)
{
    if (!out.cell && !out.xy && !out.max_L && !out.max_Lf)
        return;
    grid_phase_t<int64_t>(kp, sm.scores, sm.redv, sm.redi, out, f0, nf);
}

template <bool PREPARED>
__global__ void __launch_bounds__(1024) k_direct(tdoa_kparams kp, tdoa_kout out,
                                                 const int16_t *__restrict__ frames, int64_t B)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Smem sm = carve(smem, kp, blockDim.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kp.F;
    const int nf = (int)((B - f0) < kp.F ? (B - f0) : kp.F);
    DIAG_STAMP(0);
    stage_frames<PREPARED>(kp, sm, frames, f0, nf);
    DIAG_STAMP(1);
    xcorr_phase(kp, sm, nf);
    DIAG_STAMP(2);
    argmax_prior_phase<int64_t>(kp, sm.scores, sm.best, out, f0, nf);
    __syncthreads();
    DIAG_STAMP(3);
    grid_phase(kp, sm, out, f0, nf);
    DIAG_STAMP(4);
}

// --------------------------------------------------------------- EMA
// correlations.c:38-63 for stream s (one workgroup per stream):
//   est = (int64)((float)est + (float)(fresh - est) * decay); best = first max
__global__ void __launch_bounds__(256) k_average(tdoa_kparams kp, int64_t *__restrict__ est,
                                                 const int64_t *__restrict__ fresh,
                                                 const float *__restrict__ decay,
                                                 int32_t *__restrict__ best, tdoa_kout out,
                                                 int do_grid)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int64_t *W = (int64_t *)smem;                   // [P][K]
    int64_t *redv = W + kp.P * kp.K;                // [4]
    int *redi = (int *)(redv + 4);                  // [4]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int64_t s = blockIdx.x;
    const int K = kp.K, P = kp.P;
    const float dec = decay[s];
    for (int p = wave; p < P; p += nwaves) {
        int64_t *e = est + ((size_t)s * P + p) * K;
        const int64_t *fr = fresh + ((size_t)s * P + p) * K;
        int64_t bv = INT64_MIN;
        int bk = INT_MAX;
        for (int k = lane; k < 128; k += 64) {
            if (k < K) {
                const int64_t ev = e[k];
                const float delta = (float)(fr[k] - ev) * dec;
                const float sum = (float)ev + delta;
                const int64_t nv = (int64_t)sum;
                e[k] = nv;
                W[p * K + k] = nv;
                if (nv > bv) {
                    bv = nv;
                    bk = k;
                }
            }
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const int64_t ov = __shfl_xor(bv, m, 64);
            const int ok = __shfl_xor(bk, m, 64);
            if (ov > bv || (ov == bv && ok < bk)) {
                bv = ov;
                bk = ok;
            }
        }
        if (lane == 0)
            best[s * P + p] = bk - kp.S;
    }
    __syncthreads();
    if (!do_grid)
        return;
    int64_t bv = INT64_MIN;
    int bu = INT_MAX;
    for (int u = tid; u < kp.U; u += blockDim.x) {
        int64_t L = 0;
        for (int tw = 0; tw < kp.TW; tw++) {
            const uint32_t word = kp.tuples[u * kp.TW + tw];
            for (int b = 0; b < 4; b++) {
                const int p = 4 * tw + b;
                if (p < P)
                    L += W[p * K + ((word >> (8 * b)) & 0xFFu)];
            }
        }
        if (L > bv) {
            bv = L;
            bu = u;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const int64_t ov = __shfl_xor(bv, m, 64);
        const int ou = __shfl_xor(bu, m, 64);
        if (ov > bv || (ov == bv && ou < bu)) {
            bv = ov;
            bu = ou;
        }
    }
    if (lane == 0) {
        redv[wave] = bv;
        redi[wave] = bu;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < nwaves; w++)
            if (redv[w] > bv || (redv[w] == bv && redi[w] < bu)) {
                bv = redv[w];
                bu = redi[w];
            }
        const int cell = kp.tuple_cell[bu];
        if (out.cell)
            out.cell[s] = cell;
        if (out.max_L)
            out.max_L[s] = bv;
        if (out.xy) {
            out.xy[2 * s] = (float)(cell % kp.grid_W - kp.half_w) / kp.grid_scale;
            out.xy[2 * s + 1] = (float)(kp.half_h - cell / kp.grid_W) / kp.grid_scale;
        }
    }
}

// ------------------------------------------------ per-frame reference ops
// op 0: rolling_buffer.c:43-71  linearise ring from head, floor-mean DC, power
// op 1: buffer.c:13-18          x <<= 8 (int16 wrap)
// op 2: buffer.c:4-11           x = (int16)((int32)x * W[i] >> 15)
__global__ void __launch_bounds__(256) k_ref_buffer(int op, int16_t *__restrict__ buf,
                                                    const int16_t *__restrict__ ring, int head,
                                                    int64_t *__restrict__ power,
                                                    const int16_t *__restrict__ window, int n,
                                                    int log2n)
{
    __shared__ int tot;
    __shared__ unsigned long long pw;
    const int tid = threadIdx.x;
    if (op == 0) {
        if (tid == 0) {
            tot = 0;
            pw = 0;
        }
        __syncthreads();
        int s = 0;
        for (int i = tid; i < n; i += blockDim.x)
            s += ring[(head + i) & (n - 1)];
        atomicAdd(&tot, s);
        __syncthreads();
        const uint32_t off16 = (uint32_t)(tot >> log2n) & 0xFFFFu;
        long long p = 0;
        for (int i = tid; i < n; i += blockDim.x) {
            const uint32_t x = (uint32_t)(uint16_t)ring[(head + i) & (n - 1)];
            const int16_t y = (int16_t)(uint16_t)((x - off16) & 0xFFFFu);
            buf[i] = y;
            p += (long long)y * y;
        }
        atomicAdd(&pw, (unsigned long long)p);
        __syncthreads();
        if (tid == 0)
            *power = (int64_t)pw;
    } else if (op == 1) {
        for (int i = tid; i < n; i += blockDim.x)
            buf[i] = (int16_t)(uint16_t)(((uint32_t)(uint16_t)buf[i] << 8) & 0xFFFFu);
    } else {
        for (int i = tid; i < n; i += blockDim.x) {
            const int32_t t = (int32_t)buf[i] * (int32_t)window[i];
            buf[i] = (int16_t)(uint16_t)((uint32_t)(t >> 15) & 0xFFFFu);
        }
    }
}

// ================================================================ GCC-PHAT
// One workgroup (N'/4 threads, N' = N) per frame.  With L = 2N (zero-padded
// linear correlation) every mic's real FFT_L is one complex FFT_N' of
// z[n] = x[2n] + i x[2n+1] (z = 0 for n >= N/2) plus a split step; every
// pair's real inverse FFT_L is one complex inverse FFT_N' of
// Y[k] = (R[k] + R*[N'-k]) + i (R[k] - R*[N'-k]) e^{+2 pi i k / L},
// R = conj(X_i) X_j / max(|X_i^* X_j|, eps)   (PHAT),
// y = IFFT(Y)/L  ->  r[2n] = Re y[n], r[2n+1] = Im y[n].
// FFTs: Stockham autosort radix-4 (+ one radix-2 pass when log2 N' is odd)
// in LDS, all M (then P) transforms of the frame advanced together.
// Input samples are the same integer prep as DIRECT (DC, <<8, Q15 window),
// scaled by 2^-15.

struct cf {
    float x, y;
};
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf cconj(cf a) { return {a.x, -a.y}; }
__device__ __forceinline__ cf mul_i(cf a) { return {-a.y, a.x}; }      // * i
__device__ __forceinline__ cf mul_mi(cf a) { return {a.y, -a.x}; }    // * -i

template <bool INV>
__device__ __forceinline__ void fft4(cf &v0, cf &v1, cf &v2, cf &v3)
{
    const cf a = cadd(v0, v2), b = csub(v0, v2), c = cadd(v1, v3);
    const cf d = INV ? mul_i(csub(v1, v3)) : mul_mi(csub(v1, v3));
    v0 = cadd(a, c);
    v1 = cadd(b, d);
    v2 = csub(a, c);
    v3 = csub(b, d);
}

__device__ __forceinline__ cf ldtw(const float *tw, int k) { return {tw[2 * k], tw[2 * k + 1]}; }

// One Stockham radix-4 pass (Ns = size of finished sub-transforms) over nb
// buffers of length n; every thread owns butterfly j = tid (n/4 threads).
template <bool INV, int NB>
__device__ void stockham4(cf *buf, int stride, int n, int Ns, const float *tw)
{
    const int j = threadIdx.x;
    const int q = n >> 2;
    const int k = j & (Ns - 1);
    const int tstep = n / (4 * Ns);
    cf w1 = ldtw(tw, k * tstep), w2 = ldtw(tw, 2 * k * tstep), w3 = ldtw(tw, 3 * k * tstep);
    if (INV) {
        w1 = cconj(w1);
        w2 = cconj(w2);
        w3 = cconj(w3);
    }
    cf v[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const cf *in = buf + b * stride;
#pragma unroll
        for (int r = 0; r < 4; r++)
            v[b][r] = in[j + r * q];
    }
    __syncthreads();
    const int idxD = (j / Ns) * Ns * 4 + k;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        cf v0 = v[b][0], v1 = cmul(v[b][1], w1), v2 = cmul(v[b][2], w2), v3 = cmul(v[b][3], w3);
        fft4<INV>(v0, v1, v2, v3);
        cf *o = buf + b * stride;
        o[idxD] = v0;
        o[idxD + Ns] = v1;
        o[idxD + 2 * Ns] = v2;
        o[idxD + 3 * Ns] = v3;
    }
    __syncthreads();
}

// Final radix-2 pass (Ns = n/2): butterflies j and j + n/4 per thread.
template <bool INV, int NB>
__device__ void stockham2_last(cf *buf, int stride, int n, const float *tw)
{
    const int q = n >> 2, half = n >> 1;
    cf v[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const cf *in = buf + b * stride;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int j = threadIdx.x + h * q;
            v[b][2 * h] = in[j];
            v[b][2 * h + 1] = in[j + half];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; b++) {
        cf *o = buf + b * stride;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int j = threadIdx.x + h * q;
            cf w = ldtw(tw, j);
            if (INV)
                w = cconj(w);
            const cf a = v[b][2 * h], c = cmul(v[b][2 * h + 1], w);
            o[j] = cadd(a, c);
            o[j + half] = csub(a, c);
        }
    }
    __syncthreads();
}

template <bool INV, int NB>
__device__ void fft_rest(cf *buf, int stride, int n, int Ns0, const float *tw)
{
    int Ns = Ns0;
    for (; Ns * 4 <= n; Ns *= 4)
        stockham4<INV, NB>(buf, stride, n, Ns, tw);
    if (Ns < n)
        stockham2_last<INV, NB>(buf, stride, n, tw);
}

template <int M>
__global__ void __launch_bounds__(512) k_gcc_phat(tdoa_kparams kp, tdoa_kout out,
                                                  const int16_t *__restrict__ frames, int64_t B,
                                                  float eps2)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int P = M * (M - 1) / 2;
    const int K = kp.K, N = kp.N;
    const int n = N;           // complex FFT length N' (L = 2N)
    const int tid = threadIdx.x;
    // carve
    size_t o = 0;
    cf *C = (cf *)(smem + o);                       // [M][n]
    o += (size_t)M * n * sizeof(cf);
    Smem sm;
    sm.X = (uint32_t *)(smem + o);                  // [M][N/2] staged words
    o += (size_t)M * (N / 2) * 4;
    float *scores = (float *)(smem + o);            // [P][K]
    o += (size_t)P * K * 4;
    o = (o + 15) & ~(size_t)15;
    float *redv = (float *)(smem + o);              // [nwaves][FMAX] (8-byte slots)
    o += (size_t)(blockDim.x >> 6) * TDOA_FMAX * 8;
    int *redi = (int *)(smem + o);
    o += (size_t)(blockDim.x >> 6) * TDOA_FMAX * 4;
    sm.sums = (int *)(smem + o);
    o += (size_t)M * 4;
    int *bestlag = (int *)(smem + o);

    const int64_t f0 = blockIdx.x;
    {
        tdoa_kparams k1 = kp;
        k1.PADW = 0;
        k1.RS = N / 2;
        k1.F = 1;
        stage_frames<false>(k1, sm, frames, f0, 1);
    }
    const float sc = 1.0f / 32768.0f;
    // pass 1 (Ns = 1) straight from the staged words: inputs j, j+q nonzero,
    // j+2q, j+3q are the zero padding.
    {
        const int j = tid, q = n >> 2;
#pragma unroll
        for (int m = 0; m < M; m++) {
            const uint32_t *xw = sm.X + m * (N / 2);
            const uint32_t a = xw[j], b = xw[j + q];
            const cf v0 = {(float)(int16_t)(a & 0xFFFFu) * sc, (float)(int16_t)(a >> 16) * sc};
            const cf v1 = {(float)(int16_t)(b & 0xFFFFu) * sc, (float)(int16_t)(b >> 16) * sc};
            cf *c = C + m * n + 4 * j;
            c[0] = cadd(v0, v1);
            c[1] = cadd(v0, mul_mi(v1));
            c[2] = csub(v0, v1);
            c[3] = cadd(v0, mul_i(v1));
        }
    }
    __syncthreads();
    fft_rest<false, M>(C, n, n, 4, kp.tw);

    // split -> X_m[k], X_m[n-k]; PHAT cross spectra; inverse pre-twiddle into
    // C[p] (bins are thread-private, so P <= M buffers are reused in place)
    for (int k = tid; k <= n / 2; k += blockDim.x) {
        const int kn = (n - k) & (n - 1);
        cf Xk[M], Xn[M];
        const cf w2k = ldtw(kp.tw2, k), w2n = ldtw(kp.tw2, n - k);
#pragma unroll
        for (int m = 0; m < M; m++) {
            const cf Zk = C[m * n + k], Zn = C[m * n + kn];
            if (k == 0) {
                Xk[m] = {Zk.x + Zk.y, 0.0f};      // X[0]
                Xn[m] = {Zk.x - Zk.y, 0.0f};      // X[n] (Nyquist of L)
            } else {
                // X[k] = (Z[k] + Z*[n-k])/2 - i/2 w^k (Z[k] - Z*[n-k]),  w = e^{-2 pi i/L}
                const cf e = cadd(Zk, cconj(Zn)), d = csub(Zk, cconj(Zn));
                const cf od = cmul(w2k, d);
                Xk[m] = {0.5f * (e.x + od.y), 0.5f * (e.y - od.x)};
                const cf e2 = cadd(Zn, cconj(Zk)), d2 = csub(Zn, cconj(Zk));
                const cf od2 = cmul(w2n, d2);
                Xn[m] = {0.5f * (e2.x + od2.y), 0.5f * (e2.y - od2.x)};
            }
        }
#pragma unroll
        for (int p = 0; p < P; p++) {
            // lexicographic pair p = (i, jj), compile-time after unrolling
            int i = 0, jj = 1;
            {
                int q = p;
                while (q >= M - 1 - i) {
                    q -= M - 1 - i;
                    i++;
                }
                jj = i + 1 + q;
            }
            cf Rk = cmul(cconj(Xk[i]), Xk[jj]);
            cf Rn = cmul(cconj(Xn[i]), Xn[jj]);
            const float ak = Rk.x * Rk.x + Rk.y * Rk.y, an = Rn.x * Rn.x + Rn.y * Rn.y;
            const float rk = rsqrtf(fmaxf(ak, eps2)), rn = rsqrtf(fmaxf(an, eps2));
            Rk = {Rk.x * rk, Rk.y * rk};
            Rn = {Rn.x * rn, Rn.y * rn};
            // Y[k] = (R[k] + R*[n-k]) + i (R[k] - R*[n-k]) conj(w^k)
            const cf ae = cadd(Rk, cconj(Rn));
            const cf ao = cmul(csub(Rk, cconj(Rn)), cconj(w2k));
            C[p * n + k] = cadd(ae, mul_i(ao));
            if (k != 0 && k != n / 2) {
                const cf ae2 = cadd(Rn, cconj(Rk));
                const cf ao2 = cmul(csub(Rn, cconj(Rk)), cconj(w2n));
                C[p * n + kn] = cadd(ae2, mul_i(ao2));
            }
        }
    }
    __syncthreads();
    fft_rest<true, P>(C, n, n, 1, kp.tw);

    // lags -S..S of r = y/L: r[2u] = Re y[u], r[2u+1] = Im y[u]
    const float invL = 1.0f / (float)(2 * n);
    for (int i = tid; i < P * K; i += blockDim.x) {
        const int p = i / K, s = i - p * K - kp.S;
        const int m = s < 0 ? s + 2 * n : s;
        const cf y = C[p * n + (m >> 1)];
        scores[i] = ((m & 1) ? y.y : y.x) * invL;
    }
    __syncthreads();
    argmax_prior_phase<float>(kp, scores, bestlag, out, f0, 1);
    __syncthreads();
    if (out.cell || out.xy || out.max_Lf)
        grid_phase_t<float>(kp, scores, redv, redi, out, f0, 1);
}

int hip_fail(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

}  // namespace

// Frames per workgroup and threads: F*items rounded to whole waves, chosen
// to waste the fewest lanes (cfg2: 144 items/frame -> F = 4, 576 threads).
static void direct_geometry(tdoa_kparams &kp, int &threads)
{
    const int items = kp.P * kp.T * kp.NSEG;
    int bestF = 1;
    double bestEff = -1.0;
    for (int F = 1; F <= 8; F++) {
        const int th = ((F * items + 63) / 64) * 64;
        if (th > 1024 && F > 1)
            break;
        kp.F = F;
        if (smem_bytes(kp, (th > 1024 ? 1024 : th) / 64) > 64 * 1024 && F > 1)
            break;
        const double eff = th > 1024 ? 1.0 : (double)(F * items) / th;
        if (eff > bestEff + 1e-9) {
            bestEff = eff;
            bestF = F;
        }
    }
    kp.F = bestF;
    threads = ((bestF * items + 63) / 64) * 64;
    if (threads > 1024)
        threads = 1024;
}

int tdoa_launch_direct(const tdoa_kparams &kp_in, const tdoa_kout &out, const int16_t *frames,
                       int64_t B, bool prepared, void *stream, int *lds_bytes_out)
{
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    tdoa_kparams kp = kp_in;
    int threads = 0;
    direct_geometry(kp, threads);
    const size_t lds = smem_bytes(kp, threads / 64);
    if (lds > 160 * 1024)
        return tdoa_set_error(-1, "DIRECT: shape needs more than 160 KiB LDS per workgroup");
    if (lds_bytes_out)
        *lds_bytes_out = (int)lds;
    const int64_t grid = (B + kp.F - 1) / kp.F;
    if (grid > INT_MAX)
        return tdoa_set_error(-1, "DIRECT: batch too large for one launch");
    hipStream_t st = (hipStream_t)stream;
    if (prepared)
        hipLaunchKernelGGL(k_direct<true>, dim3((unsigned)grid), dim3(threads), lds, st, kp, out,
                           frames, B);
    else
        hipLaunchKernelGGL(k_direct<false>, dim3((unsigned)grid), dim3(threads), lds, st, kp, out,
                           frames, B);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_direct launch");
    return 0;
}

int tdoa_launch_average(const tdoa_kparams &kp, int64_t S, int64_t *est, const int64_t *fresh,
                        const float *decay, int32_t *best, const tdoa_kout *solve, void *stream)
{
    if (S > INT_MAX)
        return tdoa_set_error(-1, "average: too many streams for one launch");
    tdoa_kout o{};
    if (solve)
        o = *solve;
    const size_t lds = (size_t)kp.P * kp.K * 8 + 4 * 8 + 4 * 4;
    hipLaunchKernelGGL(k_average, dim3((unsigned)S), dim3(256), lds, (hipStream_t)stream, kp,
                       est, fresh, decay, best, o, solve ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_average launch");
    return 0;
}

int tdoa_launch_gcc_phat(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames,
                         int64_t B, float phat_eps, void *stream)
{
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    if (kp.P > kp.M)
        return tdoa_set_error(-1, "GCC_PHAT: more pairs than mics (M > 3) not supported yet");
    if (kp.N > 2048)
        return tdoa_set_error(-1, "GCC_PHAT: frame_len > 2048 not supported yet");
    if (!kp.tw || !kp.tw2)
        return tdoa_set_error(-1, "GCC_PHAT: context has no twiddle tables");
    const int threads = kp.N / 4 < 64 ? 64 : kp.N / 4;
    if (threads != kp.N / 4)
        return tdoa_set_error(-1, "GCC_PHAT: frame_len must be >= 256");
    const int nw = threads / 64;
    size_t lds = (size_t)kp.M * kp.N * 8 + (size_t)kp.M * (kp.N / 2) * 4 + (size_t)kp.P * kp.K * 4;
    lds = (lds + 15) & ~(size_t)15;
    lds += (size_t)nw * TDOA_FMAX * 12 + (size_t)kp.M * 4 + (size_t)kp.P * 4 + 16;
    if (lds > 160 * 1024)
        return tdoa_set_error(-1, "GCC_PHAT: shape needs more than 160 KiB LDS");
    if (B > INT_MAX)
        return tdoa_set_error(-1, "GCC_PHAT: batch too large for one launch");
    if (kp.M == 2)
        hipLaunchKernelGGL(k_gcc_phat<2>, dim3((unsigned)B), dim3(threads), lds,
                           (hipStream_t)stream, kp, out, frames, B, phat_eps * phat_eps);
    else if (kp.M == 3)
        hipLaunchKernelGGL(k_gcc_phat<3>, dim3((unsigned)B), dim3(threads), lds,
                           (hipStream_t)stream, kp, out, frames, B, phat_eps * phat_eps);
    else
        return tdoa_set_error(-1, "GCC_PHAT: num_mics must be 2 or 3 for now");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_gcc_phat launch");
    return 0;
}

int tdoa_launch_ref_buffer(int op, int16_t *buf, const int16_t *ring, int head, int64_t *power,
                           const int16_t *window, int n, void *stream)
{
    int log2n = 0;
    while ((1 << log2n) < n)
        log2n++;
    hipLaunchKernelGGL(k_ref_buffer, dim3(1), dim3(256), 0, (hipStream_t)stream, op, buf, ring,
                       head, power, window, n, log2n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_ref_buffer launch");
    return 0;
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch(unsigned long long *host, int n)
{
    if (n > (1 << 20))
        n = 1 << 20;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
