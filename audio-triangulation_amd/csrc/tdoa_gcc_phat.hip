// tdoa_gcc_phat.hip -- GCC-PHAT engine kernel.  Compiled
// with FMA contraction allowed: this engine is tolerance-checked against a
// float64 oracle, unlike DIRECT whose float steps must round like the
// reference's IEEE host build.
#include <hip/hip_runtime.h>

#include <cstring>

#ifndef TDOA_P1K_DEFAULT_W64
#define TDOA_P1K_DEFAULT_W64 0
#endif
// TDOA_AB=1: the A/B build (tdoa/libtdoa_ab.so) with k_p1k_w64 behind TDOA_P1K=w64
#ifndef TDOA_AB
#define TDOA_AB 0
#endif
#include <stdint.h>

#include <climits>
#include <cstdlib>

#include "tdoa_device.h"
#include "tdoa_fft32.h"
#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

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
    o += (size_t)(blockDim.x >> 6) * TDOA_FMAX * 12;  // (was the fused grid's reduction slots)
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
}


int hip_fail(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

}  // namespace

// ======================================================= GCC-PHAT, N = 1024
// k_gcc_phat_1024: the metric shape (M = 3, N = 1024, L = 2048).
//   * one 32-lane half-wave per complex FFT_1024, done as 32 x 32:
//     DFT-32 in registers (lane = column), twiddle W_1024^{lane*k},
//     one transpose through an XOR-swizzled 8 KiB LDS tile, DFT-32 again;
//   * forward: z[n] = x[2n] + i x[2n+1] is zero for n >= 512, so the first
//     radix-2 stage of the first DFT-32 is a copy + twiddle;
//   * inverse: only lags -S..S are needed (y[n] for n < 24 or n > 1000), so
//     the second DFT-32 evaluates just its outputs 0 and 31 per lane;
//   * 2 frames per 192-thread workgroup (6 half-waves = 6 FFTs), persistent
//     over frame pairs with the next pair's samples prefetched in registers.
// Since round 2 it is the fallback of the config-2 shape (tuple tables larger
// than k_p1k_lean's LDS image holds).  One workgroup per CU (launch bounds
// 192, 1): at two it spilled 7 VGPRs to 32 B of scratch; with the unified
// register file of a one-wave-per-SIMD launch it holds 258 registers and no
// scratch (tools/co_audit.py, tests/test_code_objects.py).

#ifdef TDOA_DIAG
// diagnostic build only: per-workgroup cycles per phase of k_gcc_phat_1024
__device__ unsigned long long g_diag_phat[1 << 16];
#define PH_MARK(i)                                            \
    do {                                                      \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph_acc[i] += t_ - ph_t;                               \
        ph_t = t_;                                            \
    } while (0)
#else
#define PH_MARK(i) \
    do {           \
    } while (0)
#endif

// element (row, col) of a 32 x 32 complex tile: 16-byte chunks XOR-swizzled by
// row so that both row reads (b128) and column writes (b64) are conflict-free
__device__ __forceinline__ int swz(int row, int col)
{
    return row * 32 + ((((col >> 1) ^ (row & 15)) << 1) | (col & 1));
}

__device__ __forceinline__ f2 ldf2(const float *p, int k) { return f2{p[2 * k], p[2 * k + 1]}; }

// Grid solve (vga_heatmap.h:99-108 on float scores) for the ns frames whose
// weighted scores sit in wsc[p][k][slot]: every lane scores its tuples for all
// GSLOTS slots at once (two b128 LDS reads per pair), strict '>' over
// increasing tuples per lane, then (max, first tuple) across the workgroup.
constexpr int GSLOTS = 8;

__device__ __forceinline__ void grid_tail(const tdoa_kparams &kp, const tdoa_kout &out,
                                          const float *wsc, const int64_t *gfr, float *gredv,
                                          int *gredi, int ns, uint32_t *tups)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, K = kp.K;
    // stage the tuple table (U words) in the idle FFT buffers: all loads in flight together
#pragma unroll 8
    for (int e = tid; e < kp.U; e += 192)
        tups[e] = kp.tuples[e];
    __syncthreads();
    float bv[GSLOTS];
    int bu[GSLOTS];
#pragma unroll
    for (int f = 0; f < GSLOTS; f++) {
        bv[f] = -INFINITY;
        bu[f] = INT_MAX;
    }
    for (int u = tid; u < kp.U; u += 192) {
        const uint32_t word = tups[u];
        float L[GSLOTS];
#pragma unroll
        for (int f = 0; f < GSLOTS; f++)
            L[f] = 0.0f;
#pragma unroll
        for (int p = 0; p < 3; p++) {
            const float4 *src = reinterpret_cast<const float4 *>(
                wsc + (p * K + (int)((word >> (8 * p)) & 0xFFu)) * GSLOTS);
            const float4 a = src[0], b = src[1];
            L[0] += a.x;
            L[1] += a.y;
            L[2] += a.z;
            L[3] += a.w;
            L[4] += b.x;
            L[5] += b.y;
            L[6] += b.z;
            L[7] += b.w;
        }
#pragma unroll
        for (int f = 0; f < GSLOTS; f++)
            if (L[f] > bv[f]) {
                bv[f] = L[f];
                bu[f] = u;
            }
    }
#pragma unroll
    for (int f = 0; f < GSLOTS; f++) {
        wave_argmax_to63(bv[f], bu[f]);
        if (lane == 63) {
            gredv[wave * GSLOTS + f] = bv[f];
            gredi[wave * GSLOTS + f] = bu[f];
        }
    }
    __syncthreads();
    if (tid < ns) {
        float v = gredv[tid];
        int ui = gredi[tid];
        for (int w = 1; w < 3; w++)
            better(v, ui, gredv[w * GSLOTS + tid], gredi[w * GSLOTS + tid]);
        if (ui < 0 || ui >= kp.U)  // every L compared false (NaN scores)
            ui = 0;
        const int cell = kp.tuple_cell[ui];
        const int64_t fi = gfr[tid];
        if (out.cell)
            out.cell[fi] = cell;
        if (out.max_Lf)
            out.max_Lf[fi] = v;
        if (out.xy) {
            const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
            out.xy[2 * fi] = (float)(cx - kp.half_w) / kp.grid_scale;
            out.xy[2 * fi + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
        }
    }
}

__global__ void __launch_bounds__(192, 1) k_gcc_phat_1024(tdoa_kparams kp, tdoa_kout out,
                                                          const int16_t *__restrict__ frames,
                                                          int64_t B, float eps2)
{
    constexpr int M = 3, P = 3, N = 1024;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = kp.K, S = kp.S;
    f2 *bufs = (f2 *)smem;                      // [6][1024] FFT tiles / spectra
    f2 *twm = bufs + 6 * 1024;                  // [32][32] W_1024^{l*k}, swizzled
    f2 *tw2s = twm + 1024;                      // [513] W_2048^k, k <= N/2
    f2 *wins = tw2s + 514;                      // [512] Q15 window / 128, sample pairs
    int *bestlag = (int *)(wins + 512);         // [2][P]
    // grid tail: weighted scores of the last GSLOTS frames, [p][k][slot], and
    // their frame indices / reduction slots
    float *wsc = (float *)(bestlag + 8);        // [P][K <= 127][GSLOTS]
    int64_t *gfr = (int64_t *)(wsc + P * 128 * GSLOTS);  // [GSLOTS]
    float *gredv = (float *)(gfr + GSLOTS);     // [3][GSLOTS]
    int *gredi = (int *)(gredv + 3 * GSLOTS);   // [3][GSLOTS]
    const bool do_grid = out.cell || out.xy || out.max_Lf;

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 31;
    const int h = wave * 2 + ((tid >> 5) & 1);  // half-wave: frame h/3, mic (then pair) h%3
    const int fr = h / 3, mp = h % 3;
    f2 *buf = bufs + h * 1024;

    for (int e = tid; e < 1024; e += 192) {
        const int l = e >> 5, k = e & 31;
        twm[swz(l, k)] = ldf2(kp.tw, (l * k) & (N - 1));
    }
    for (int e = tid; e <= N / 2; e += 192)
        tw2s[e] = ldf2(kp.tw2, e);
    for (int e = tid; e < 512; e += 192)
        wins[e] = f2{(float)kp.window[2 * e] * (1.0f / 128.0f),
                     (float)kp.window[2 * e + 1] * (1.0f / 128.0f)};
    __syncthreads();

    const int64_t npairs = (B + 1) >> 1;
    uint32_t pf[16];
    auto fetch = [&](int64_t pair) {
        const int64_t f = 2 * pair + fr;
        if (pair < npairs && f < B) {
            const uint32_t *row =
                reinterpret_cast<const uint32_t *>(frames + (f * M + mp) * (int64_t)N);
#pragma unroll
            for (int t = 0; t < 16; t++)
                pf[t] = __builtin_nontemporal_load(row + lane + 32 * t);
        } else {
#pragma unroll
            for (int t = 0; t < 16; t++)
                pf[t] = 0u;
        }
    };
    fetch(blockIdx.x);
    const float invL = 1.0f / 2048.0f;

#ifdef TDOA_DIAG
    unsigned long long ph_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long ph_t = __builtin_amdgcn_s_memtime();
    int ph_it = 0;
#endif
    int nslot = 0;  // frames waiting in wsc for the grid tail
    for (int64_t pair = blockIdx.x; pair < npairs; pair += gridDim.x) {
#ifdef TDOA_DIAG
        ph_it++;
#endif
        const int64_t f0 = 2 * pair;
        const int nf = (B - f0) < 2 ? (int)(B - f0) : 2;
        uint32_t w[16];
#pragma unroll
        for (int t = 0; t < 16; t++)
            w[t] = pf[t];
        fetch(pair + gridDim.x);

        // ---- integer front end: floor-mean DC, <<8, Q15 window (rolling_buffer.c:64-66,
        //      buffer.c:13-16, buffer.c:4-11) on words lane + 32 t of this mic row.
        //      Only the low byte of x - off survives `<<= 8`, so with s = sext8(x - off)
        //      the windowed sample is ((s << 8) * W) >> 15 = floor(s * W / 128), an
        //      integer below 2^23: exact in fp32 (wf holds W / 128).  Samples stay in
        //      int16 units (PHAT is scale-invariant; eps2 is scaled to match).
        int s = 0;
#pragma unroll
        for (int t = 0; t < 16; t++)
            s += (int)(int16_t)(w[t] & 0xFFFFu) + (int)(int16_t)(w[t] >> 16);
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1)
            s += __shfl_xor(s, o, 64);
        const uint32_t off = (uint32_t)(s >> 10) & 0xFFu;
        const uint32_t off2 = off | (off << 16);
        f2 v[32];
#pragma unroll
        for (int t = 0; t < 16; t++) {
            // bit 8 set in each half: no borrow crosses into the high sample.  (Plain
            // int8 casts: __builtin_amdgcn_sbfe on a masked word was converted as unsigned.)
            const uint32_t d = (w[t] | 0x01000100u) - off2;
            const float s0 = (float)(int8_t)(d & 0xFFu);
            const float s1 = (float)(int8_t)((d >> 16) & 0xFFu);
            const f2 wf = wins[lane + 32 * t];
            v[t] = f2{floorf(s0 * wf.x), floorf(s1 * wf.y)};
        }
        // ---- forward FFT_1024 of z: lane = n2, v[n1] = z[n2 + 32 n1]
        fft32<false, true>(v);
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const float4 q = *reinterpret_cast<const float4 *>(&twm[swz(lane, 2 * c)]);
            buf[swz(2 * c, lane)] = cmulf(v[brev5(2 * c)], f2{q.x, q.y});
            buf[swz(2 * c + 1, lane)] = cmulf(v[brev5(2 * c + 1)], f2{q.z, q.w});
        }
        wave_lds_sync();
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const float4 q = *reinterpret_cast<const float4 *>(&buf[swz(lane, 2 * c)]);
            v[2 * c] = f2{q.x, q.y};
            v[2 * c + 1] = f2{q.z, q.w};
        }
        fft32<false, false>(v);
        wave_lds_sync();
        // spectrum Z[lane + 32 k] at (row k, col lane)
#pragma unroll
        for (int k = 0; k < 32; k++)
            buf[swz(k, lane)] = v[brev5(k)];
        __syncthreads();

        PH_MARK(0);
        // ---- split to X_m, PHAT cross spectra, inverse pre-twiddle (in place per bin pair).
        // Items it = tid + 192 r (2 frames x 513 bin pairs (k, N-k)), 3 per batch with all
        // loads issued before any store.  The generic split is exact at k = 0 too
        // (X[0] = Re + Im, X[N] = Re - Im with W_2048^N = -1), and the duplicate
        // stores at k = 0 / N/2 write equal values.
#pragma unroll
        for (int r0 = 0; r0 < 6; r0 += 3) {
            f2 Zk[3][M], Zn[3][M], w2[3];
            int ik[3], ikn[3], fo[3];
            bool live[3];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int it = tid + 192 * (r0 + q);
                const int f = it >= 513 ? 1 : 0;
                const int k = it - 513 * f;
                live[q] = it < 2 * 513 && f < nf;
                const int kk = live[q] ? k : 0;
                const int kn = (N - kk) & (N - 1);
                fo[q] = (live[q] ? f : 0) * 3 * 1024;
                ik[q] = swz(kk >> 5, kk & 31);
                ikn[q] = swz(kn >> 5, kn & 31);
                w2[q] = tw2s[kk];
#pragma unroll
                for (int m = 0; m < M; m++) {
                    Zk[q][m] = bufs[fo[q] + m * 1024 + ik[q]];
                    Zn[q][m] = bufs[fo[q] + m * 1024 + ikn[q]];
                }
            }
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const f2 w2k = w2[q], w2n = -conjf2(w2[q]);  // W_2048^{N-k} = -conj(W_2048^k)
                f2 Xk[M], Xn[M];
#pragma unroll
                for (int m = 0; m < M; m++) {
                    const f2 a = Zk[q][m], b = Zn[q][m];
                    const f2 e = a + conjf2(b), d = cmulf(w2k, a - conjf2(b));
                    Xk[m] = 0.5f * f2{e.x + d.y, e.y - d.x};
                    const f2 e2 = b + conjf2(a), d2 = cmulf(w2n, b - conjf2(a));
                    Xn[m] = 0.5f * f2{e2.x + d2.y, e2.y - d2.x};
                }
                if (live[q]) {
#pragma unroll
                    for (int p = 0; p < P; p++) {
                        const int i = p < 2 ? 0 : 1, j = p == 0 ? 1 : 2;
                        f2 Rk = cmulf(conjf2(Xk[i]), Xk[j]);
                        f2 Rn = cmulf(conjf2(Xn[i]), Xn[j]);
                        Rk *= __builtin_amdgcn_rsqf(fmaxf(Rk.x * Rk.x + Rk.y * Rk.y, eps2));
                        Rn *= __builtin_amdgcn_rsqf(fmaxf(Rn.x * Rn.x + Rn.y * Rn.y, eps2));
                        bufs[fo[q] + p * 1024 + ik[q]] =
                            (Rk + conjf2(Rn)) + times_i(cmulf(Rk - conjf2(Rn), conjf2(w2k)));
                        bufs[fo[q] + p * 1024 + ikn[q]] =
                            (Rn + conjf2(Rk)) + times_i(cmulf(Rn - conjf2(Rk), conjf2(w2n)));
                    }
                }
            }
        }
        __syncthreads();

        PH_MARK(1);
        // ---- inverse FFT_1024 of Y_p: lane = k2, v[k1] = Y[32 k1 + k2]
#pragma unroll
        for (int k1 = 0; k1 < 32; k1++)
            v[k1] = buf[swz(k1, lane)];
        fft32<true, false>(v);
        wave_lds_sync();
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const float4 q = *reinterpret_cast<const float4 *>(&twm[swz(lane, 2 * c)]);
            buf[swz(2 * c, lane)] = cmulf(v[brev5(2 * c)], f2{q.x, -q.y});
            buf[swz(2 * c + 1, lane)] = cmulf(v[brev5(2 * c + 1)], f2{q.z, -q.w});
        }
        wave_lds_sync();
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const float4 q = *reinterpret_cast<const float4 *>(&buf[swz(lane, 2 * c)]);
            v[2 * c] = f2{q.x, q.y};
            v[2 * c + 1] = f2{q.z, q.w};
        }
        // outputs n_hi = 0 and 31 of the second DFT-32 (W_32^{-31 k} = W_32^{k})
        f2 y0 = v[0], y31 = v[0];
#pragma unroll
        for (int k = 1; k < 32; k++) {
            y0 += v[k];
            y31 += k < 16 ? tw32<false>(v[k], k) : -tw32<false>(v[k], k - 16);
        }
        // y[lane] -> lags 2 lane + {0,1};  y[lane + 992] -> lags 2 lane - 64 + {0,1}
        // argmax + lag prior fused here (correlations.c:20-33 semantics, float scores):
        // candidates in ascending lag order, strict '>' keeps the first maximum.
        {
            const int a = 2 * lane, b = 2 * lane - 64;
            const float cv[4] = {y31.x * invL, y31.y * invL, y0.x * invL, y0.y * invL};
            const int ck[4] = {b + S, b + 1 + S, a + S, a + 1 + S};
            const bool ok[4] = {b >= -S, b + 1 >= -S, a <= S, a + 1 <= S};
            float bv = -INFINITY;
            int bk = INT_MAX;
#pragma unroll
            for (int c = 0; c < 4; c++)
                if (ok[c] && (cv[c] > bv || bk == INT_MAX)) {
                    bv = cv[c];
                    bk = ck[c];
                }
            half_argmax_to31(bv, bk);
            bk = __shfl(bk, 31, 32);  // uniform per half-wave even for NaN scores
            bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);
            if (fr < nf) {
                const size_t gb = (size_t)((f0 + fr) * P + mp) * K;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    if (ok[c]) {
                        const int d = ck[c] > bk ? ck[c] - bk : bk - ck[c];
                        const float wv = cv[c] * kp.prior[d];
                        if (out.scores_f)
                            out.scores_f[gb + ck[c]] = cv[c];
                        if (out.weighted_f)
                            out.weighted_f[gb + ck[c]] = wv;
                        if (do_grid)
                            wsc[(mp * K + ck[c]) * GSLOTS + nslot + fr] = wv;
                    }
                }
                if (lane == 0) {
                    bestlag[fr * P + mp] = bk - S;
                    out.lags[(f0 + fr) * P + mp] = bk - S;
                    if (mp == 0)
                        gfr[nslot + fr] = f0 + fr;
                }
            }
        }
        __syncthreads();
        PH_MARK(2);
        if (out.gate && tid < nf) {
            int tot = 0;
#pragma unroll
            for (int p = 0; p < P; p++)
                tot += bestlag[tid * P + p] * bestlag[tid * P + p];
            out.gate[f0 + tid] = tot > 4 ? 1 : 0;
        }
        PH_MARK(3);
        __syncthreads();  // bestlag / buffers are rewritten by the next pair
        nslot += nf;
        if (do_grid && (nslot == GSLOTS || pair + gridDim.x >= npairs)) {
            grid_tail(kp, out, wsc, gfr, gredv, gredi, nslot, (uint32_t *)bufs);
            nslot = 0;
            __syncthreads();  // wsc / reduction slots are rewritten next
        }
        PH_MARK(4);
    }
#ifdef TDOA_DIAG
    if (threadIdx.x == 0 && blockIdx.x < (1 << 13)) {
        for (int i = 0; i < 5; i++)
            g_diag_phat[blockIdx.x * 8 + i] = ph_acc[i];
        g_diag_phat[blockIdx.x * 8 + 7] = ph_it;
    }
#endif
}

bool tdoa_gcc_phat_needs_split(int M, int N) { return M > 3 || N > 2048; }

// the N = 1024, 3-mic kernel runs the grid solve itself (grid_tail)
bool tdoa_phat1024_fits(const tdoa_kparams &kp);
int tdoa_launch_phat1024(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames,
                         int64_t B, float phat_eps, void *stream);

#if TDOA_AB
// one frame per 64-lane wave (tdoa_p1k_w64.hip, A/B build only)
bool tdoa_p1k_w64_fits(const tdoa_kparams &kp);
int tdoa_launch_p1k_w64(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
                        float phat_eps, void *stream);
#endif
// config-2 kernel choice: TDOA_P1K=lean | w64 (A/B runs, A/B build), else the default
static bool use_w64(const tdoa_kparams &kp)
{
#if !TDOA_AB
    (void)kp;
    return false;
#else
    static const int pick = [] {
        const char *e = getenv("TDOA_P1K");
        return e && !strcmp(e, "w64") ? 1 : (e && !strcmp(e, "lean") ? 0 : -1);
    }();
    const bool want = pick < 0 ? TDOA_P1K_DEFAULT_W64 : pick == 1;
    return want && tdoa_p1k_w64_fits(kp);
#endif
}

bool tdoa_phat_r16_fits(int M, int N, int S);
bool frame16_shape(const tdoa_kparams &kp);
const char *frame16_kernel_name(const tdoa_kparams &kp);

bool tdoa_gcc_phat_fused_grid(const tdoa_kparams &kp);

// The one dispatch decision of tdoa_launch_gcc_phat, shared with
// tdoa_gcc_phat_kernel_name so the reported kernel is the launched one.
enum class PhatRoute { W64, P1K_LEAN, R16, SPLIT, FUSED_1024, GENERIC };
static PhatRoute phat_route(const tdoa_kparams &kp)
{
    if (use_w64(kp))
        return PhatRoute::W64;
    if (tdoa_phat1024_fits(kp))
        return PhatRoute::P1K_LEAN;
    // frame_len 2048 / 4096 with M > 3 or N > 2048: register-pass kernels
    // (tdoa_phat_r16.hip); other long shapes the LDS Stockham pair
    if (tdoa_gcc_phat_needs_split(kp.M, kp.N))
        return tdoa_phat_r16_fits(kp.M, kp.N, kp.S) ? PhatRoute::R16 : PhatRoute::SPLIT;
    if (tdoa_gcc_phat_fused_grid(kp))
        return PhatRoute::FUSED_1024;
    return PhatRoute::GENERIC;
}

const char *tdoa_gcc_phat_kernel_name(const tdoa_kparams &kp)
{
    switch (phat_route(kp)) {
    case PhatRoute::W64:
        return "k_p1k_w64";
    case PhatRoute::P1K_LEAN:
        return "k_p1k_lean";
    case PhatRoute::R16:
        return frame16_shape(kp) ? frame16_kernel_name(kp) : "k_spec16";
    case PhatRoute::SPLIT:
        return "k_phat_spectra";
    case PhatRoute::FUSED_1024:
        return "k_gcc_phat_1024";
    case PhatRoute::GENERIC:
        break;
    }
    return "k_gcc_phat";
}
int tdoa_launch_phat_r16(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
                         float phat_eps, void *scratch, size_t scratch_bytes, void *stream);

bool tdoa_phat_r16_peak3(const tdoa_kparams &kp);

bool tdoa_frame16_fused_grid(const tdoa_kparams &kp);
// the launch solves the grid itself (no weighted-score scratch, no grid launch)
bool tdoa_gcc_phat_grid_in_kernel(const tdoa_kparams &kp)
{
    const PhatRoute r = phat_route(kp);
    if (r == PhatRoute::R16)
        return tdoa_frame16_fused_grid(kp);
    return !tdoa_gcc_phat_needs_split(kp.M, kp.N) && tdoa_gcc_phat_fused_grid(kp);
}

// the launch writes the least-squares peak scores (kout.peak3) itself
bool tdoa_gcc_phat_peak3(const tdoa_kparams &kp) { return tdoa_phat_r16_peak3(kp); }

// the N = 1024, M = 3 kernels (k_p1k_lean, k_gcc_phat_1024) solve the grid
bool tdoa_gcc_phat_fused_grid(const tdoa_kparams &kp)
{
    if (tdoa_phat1024_fits(kp))
        return true;
    // the tuple table is staged in the 48 KiB of FFT buffers
    return kp.M == 3 && kp.N == 1024 && kp.S <= 63 && kp.TW == 1 && kp.U <= 6 * 1024 * 2;
}

int tdoa_launch_gcc_phat(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames,
                         int64_t B, float phat_eps, void *spec_scratch, size_t spec_bytes,
                         void *stream)
{
    // |X_i^* X_j|^2 floor; kept a normal float (v_rsq_f32 flushes denormals)
    float eps2 = phat_eps * phat_eps;
    if (!(eps2 >= 1e-30f))
        eps2 = 1e-30f;
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    if (!kp.tw || !kp.tw2)
        return tdoa_set_error(-1, "GCC_PHAT: context has no twiddle tables");
    const PhatRoute route = phat_route(kp);
#if TDOA_AB
    if (route == PhatRoute::W64)
        return tdoa_launch_p1k_w64(kp, out, frames, B, phat_eps, stream);
#endif
    if (route == PhatRoute::P1K_LEAN)
        return tdoa_launch_phat1024(kp, out, frames, B, phat_eps, stream);
    if (route == PhatRoute::R16)
        return tdoa_launch_phat_r16(kp, out, frames, B, phat_eps, spec_scratch, spec_bytes, stream);
    if (route == PhatRoute::SPLIT)
        return tdoa_launch_gcc_phat_split(kp, out, frames, B,
                                          eps2 * 1152921504606846976.0f /* 2^60: int16 units */,
                                          spec_scratch, spec_bytes, stream);
    hipStream_t st = (hipStream_t)stream;
    if (route == PhatRoute::FUSED_1024) {
        // persistent 2-frame workgroups, as many as are resident at once
        // + grid tail: [3][128][8] scores, 8 frame indices, [3][8] reductions
        const size_t lds1024 = 7 * 1024 * 8 + 514 * 8 + 512 * 8 + 8 * 4 + 3 * 128 * GSLOTS * 4 +
                               GSLOTS * 8 + 3 * GSLOTS * 8;
        const int resident = tdoa_resident_blocks((const void *)k_gcc_phat_1024, 192, lds1024);
        const int64_t npairs = (B + 1) / 2;
        const int64_t iters = (npairs + resident - 1) / resident;
        const int64_t grid = (npairs + iters - 1) / iters;
        hipLaunchKernelGGL(k_gcc_phat_1024, dim3((unsigned)grid), dim3(192), lds1024, st, kp, out,
                           frames, B, eps2 * 1152921504606846976.0f /* 2^60: int16 units */);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "k_gcc_phat_1024 launch");
    }
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
        hipLaunchKernelGGL(k_gcc_phat<2>, dim3((unsigned)B), dim3(threads), lds, st, kp, out, frames, B, eps2);
    else if (kp.M == 3)
        hipLaunchKernelGGL(k_gcc_phat<3>, dim3((unsigned)B), dim3(threads), lds, st, kp, out, frames, B, eps2);
    else
        return tdoa_set_error(-1, "GCC_PHAT: num_mics must be 2 or 3 for now");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_gcc_phat launch");
    return 0;
}



#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch_phat(unsigned long long *host, int n)
{
    if (n > (1 << 16))
        n = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_phat), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
