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
    o += (size_t)nwaves * 8;
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
    o += (size_t)nwaves * 8;
    o += (size_t)kp.F * kp.M * 4;
    o += (size_t)kp.F * kp.P * 4;
    o += (size_t)nwaves * 4;
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
template <bool FLOATS>
__device__ void argmax_prior_phase(const tdoa_kparams &kp, const Smem &sm, const tdoa_kout &out,
                                   int64_t f0, int nf)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P;
    for (int fp = wave; fp < nf * P; fp += nwaves) {
        int64_t *sc = sm.scores + fp * K;
        const int k1 = lane, k2 = lane + 64;
        const int64_t v1 = k1 < K ? sc[k1] : INT64_MIN;
        const int64_t v2 = k2 < K ? sc[k2] : INT64_MIN;
        int64_t bv = v1;
        int bk = k1;
        if (v2 > bv) {
            bv = v2;
            bk = k2;
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const int64_t ov = __shfl_xor(bv, m, 64);
            const int ok = __shfl_xor(bk, m, 64);
            if (ov > bv || (ov == bv && ok < bk)) {
                bv = ov;
                bk = ok;
            }
        }
        const size_t gbase = (size_t)(f0 * P + fp) * K;
        if (out.scores) {
            if (k1 < K)
                out.scores[gbase + k1] = v1;
            if (k2 < K)
                out.scores[gbase + k2] = v2;
        }
        // correlations.c:27-32
        if (k1 < K) {
            const int d = k1 > bk ? k1 - bk : bk - k1;
            const float x = (float)v1 * kp.prior[d];
            const int64_t wv = (int64_t)x;
            sc[k1] = wv;
            if (out.weighted)
                out.weighted[gbase + k1] = wv;
        }
        if (k2 < K) {
            const int d = k2 > bk ? k2 - bk : bk - k2;
            const float x = (float)v2 * kp.prior[d];
            const int64_t wv = (int64_t)x;
            sc[k2] = wv;
            if (out.weighted)
                out.weighted[gbase + k2] = wv;
        }
        if (lane == 0) {
            sm.best[fp] = bk - kp.S;
            out.lags[f0 * P + fp] = bk - kp.S;
        }
    }
    __syncthreads();
    if (out.gate) {
        for (int f = tid; f < nf; f += blockDim.x) {
            int tot = 0;
            for (int p = 0; p < P; p++) {
                const int b = sm.best[f * P + p];
                tot += b * b;
            }
            out.gate[f0 + f] = tot > 4 ? 1 : 0;
        }
    }
}

// ------------------------------------------------------------- grid solve
__device__ void grid_phase(const tdoa_kparams &kp, const Smem &sm, const tdoa_kout &out,
                           int64_t f0, int nf)
{
    if (!out.cell && !out.xy && !out.max_L)
        return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P, TW = kp.TW, U = kp.U;
    for (int f = 0; f < nf; f++) {
        const int64_t *Wt = sm.scores + f * P * K;
        int64_t bv = INT64_MIN;
        int bu = INT_MAX;
        for (int u = tid; u < U; u += blockDim.x) {
            int64_t L = 0;
            for (int tw = 0; tw < TW; tw++) {
                const uint32_t word = kp.tuples[u * TW + tw];
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int p = 4 * tw + b;
                    if (p < P)
                        L += Wt[p * K + ((word >> (8 * b)) & 0xFFu)];
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
            sm.redv[wave] = bv;
            sm.redi[wave] = bu;
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < nwaves; w++) {
                if (sm.redv[w] > bv || (sm.redv[w] == bv && sm.redi[w] < bu)) {
                    bv = sm.redv[w];
                    bu = sm.redi[w];
                }
            }
            const int cell = kp.tuple_cell[bu];
            const int64_t fi = f0 + f;
            if (out.cell)
                out.cell[fi] = cell;
            if (out.max_L)
                out.max_L[fi] = bv;
            if (out.xy) {
                const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
                out.xy[2 * fi] = (float)(cx - kp.half_w) / kp.grid_scale;
                out.xy[2 * fi + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
            }
        }
        __syncthreads();
    }
}

template <bool PREPARED>
__global__ void __launch_bounds__(1024) k_direct(tdoa_kparams kp, tdoa_kout out,
                                                 const int16_t *__restrict__ frames, int64_t B)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Smem sm = carve(smem, kp, blockDim.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kp.F;
    const int nf = (int)((B - f0) < kp.F ? (B - f0) : kp.F);
    stage_frames<PREPARED>(kp, sm, frames, f0, nf);
    xcorr_phase(kp, sm, nf);
    argmax_prior_phase<false>(kp, sm, out, f0, nf);
    __syncthreads();
    grid_phase(kp, sm, out, f0, nf);
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

int tdoa_launch_gcc_phat(const tdoa_kparams &, const tdoa_kout &, const int16_t *, int64_t, float,
                         void *)
{
    return tdoa_set_error(-1, "GCC_PHAT engine not built yet");
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
