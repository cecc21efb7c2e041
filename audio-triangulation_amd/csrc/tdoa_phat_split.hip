// tdoa_phat_split.hip -- GCC-PHAT for the shapes whose spectra do not fit one
// workgroup's LDS next to each other (M > 3 or N > 2048: BASELINE configs 3
// and 4).  Same definition as the fused kernels (oracle/gcc_phat_oracle.py),
// split in two passes over chunks of frames:
//
//   k_phat_spectra  one workgroup per (frame, mic) row: the integer front end
//                   (rolling_buffer.c:64-66, buffer.c:13-16, buffer.c:4-11),
//                   complex FFT_N of z[n] = x[2n] + i x[2n+1] in LDS and the
//                   split to X[0..N] of the real FFT_2N, stored N complex per
//                   row (slot 0 packs the two real bins X[0], X[N]) to a
//                   scratch sized to stay in L2 / MALL between the passes;
//   k_phat_pairs    one workgroup per (frame, pair): PHAT cross spectrum and
//                   inverse pre-twiddle straight from the scratch, inverse
//                   FFT_N in LDS, lags -S..S, first argmax, lag prior
//                   (correlations.c:20-33 semantics on float scores);
//   k_phat_gate     sum of squared best lags > 4 (sample_compute.h:124-134).
//
// Samples stay in int16 units; the launcher scales eps^2 by 2^60 to match.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

constexpr int TPB = 256;  // threads per workgroup
constexpr int BPT = 4;    // radix-4 butterflies per thread: N/4 <= 1024

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 cmul(f2 a, f2 b)
{
    return f2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ f2 conj2(f2 a) { return f2{a.x, -a.y}; }
__device__ __forceinline__ f2 mul_i(f2 a) { return f2{-a.y, a.x}; }
__device__ __forceinline__ f2 mul_mi(f2 a) { return f2{a.y, -a.x}; }
__device__ __forceinline__ f2 ldtw(const float *tw, int k) { return f2{tw[2 * k], tw[2 * k + 1]}; }

// In-place complex FFT of length n (256 <= n <= 4096, power of two) held in
// LDS: Stockham radix-4 passes (one radix-2 pass last when log2 n is odd),
// each pass staged through registers so one buffer suffices.  tw = W_n^k.
template <bool INV>
__device__ void fft_inplace(f2 *buf, int n, const float *__restrict__ tw)
{
    const int tid = threadIdx.x, q = n >> 2;
    int Ns = 1;
    for (; Ns * 4 <= n; Ns *= 4) {
        const int tstep = n / (4 * Ns);
        f2 v[BPT][4];
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = tid + TPB * b;
            if (j < q) {
#pragma unroll
                for (int r = 0; r < 4; r++)
                    v[b][r] = buf[j + r * q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = tid + TPB * b;
            if (j < q) {
                const int k = j & (Ns - 1);
                f2 w1 = ldtw(tw, k * tstep), w2 = ldtw(tw, 2 * k * tstep),
                   w3 = ldtw(tw, 3 * k * tstep);
                if (INV) {
                    w1 = conj2(w1);
                    w2 = conj2(w2);
                    w3 = conj2(w3);
                }
                const f2 x0 = v[b][0], x1 = cmul(v[b][1], w1), x2 = cmul(v[b][2], w2),
                         x3 = cmul(v[b][3], w3);
                const f2 a = x0 + x2, c = x0 - x2, s = x1 + x3;
                const f2 d = INV ? mul_i(x1 - x3) : mul_mi(x1 - x3);
                const int o = (j / Ns) * Ns * 4 + k;
                buf[o] = a + s;
                buf[o + Ns] = c + d;
                buf[o + 2 * Ns] = a - s;
                buf[o + 3 * Ns] = c - d;
            }
        }
        __syncthreads();
    }
    if (Ns < n) {  // radix-2, Ns = n/2: butterflies j < n/2 = 2q
        const int half = n >> 1;
        f2 v[BPT][2];
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = tid + TPB * b;
            if (j < half) {
                v[b][0] = buf[j];
                v[b][1] = buf[j + half];
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < BPT; b++) {
            const int j = tid + TPB * b;
            if (j < half) {
                f2 w = ldtw(tw, j);
                if (INV)
                    w = conj2(w);
                const f2 c = cmul(v[b][1], w);
                buf[j] = v[b][0] + c;
                buf[j + half] = v[b][0] - c;
            }
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t prep_word(uint32_t v, uint32_t off16, uint32_t wv)
{
    // (int16)(x - off), then <<= 8 keeps the low byte, then (x * W) >> 15
    uint32_t r = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t x = (v >> (16 * h)) & 0xFFFFu;
        const int32_t w = (int32_t)(int16_t)((wv >> (16 * h)) & 0xFFFFu);
        const int32_t z = (int32_t)(int16_t)(uint16_t)((((x - off16) & 0xFFFFu) << 8) & 0xFFFFu);
        r |= ((uint32_t)((z * w) >> 15) & 0xFFFFu) << (16 * h);
    }
    return r;
}

// ---------------------------------------------------------------- pass 1
__global__ void __launch_bounds__(TPB) k_phat_spectra(tdoa_kparams kp,
                                                      const int16_t *__restrict__ frames,
                                                      int64_t row0, f2 *__restrict__ spec)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *buf = (f2 *)smem;  // [N]
    __shared__ int red[TPB / 64];
    const int N = kp.N, NW = N / 2, tid = threadIdx.x;
    const int64_t row = row0 + blockIdx.x;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(frames + row * (int64_t)N);
    const uint32_t *win = reinterpret_cast<const uint32_t *>(kp.window);

    int s = 0;
    for (int w = tid; w < NW; w += TPB) {
        const uint32_t v = x[w];
        s += (int)(int16_t)(v & 0xFFFFu) + (int)(int16_t)(v >> 16);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0)
        red[tid >> 6] = s;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int w = 0; w < TPB / 64; w++)
        tot += red[w];
    const uint32_t off16 = (uint32_t)(tot >> kp.log2N) & 0xFFFFu;  // floor mean, (int16)
    for (int w = tid; w < N; w += TPB) {
        f2 z = f2{0.0f, 0.0f};
        if (w < NW) {
            const uint32_t p = prep_word(x[w], off16, win[w]);
            z = f2{(float)(int16_t)(p & 0xFFFFu), (float)(int16_t)(p >> 16)};
        }
        buf[w] = z;
    }
    __syncthreads();
    fft_inplace<false>(buf, N, kp.tw);

    // X[k] = (Z[k] + Z*[N-k])/2 - i/2 W_2N^k (Z[k] - Z*[N-k])
    f2 *o = spec + (size_t)blockIdx.x * N;
    for (int k = tid; k <= N / 2; k += TPB) {
        const int kn = (N - k) & (N - 1);
        const f2 a = buf[k], b = buf[kn];
        if (k == 0) {
            o[0] = f2{a.x + a.y, a.x - a.y};  // X[0], X[N]: both real
            continue;
        }
        const f2 w2k = ldtw(kp.tw2, k), w2n = ldtw(kp.tw2, N - k);
        const f2 e = a + conj2(b), d = cmul(w2k, a - conj2(b));
        o[k] = 0.5f * f2{e.x + d.y, e.y - d.x};
        if (k != N / 2) {
            const f2 e2 = b + conj2(a), d2 = cmul(w2n, b - conj2(a));
            o[kn] = 0.5f * f2{e2.x + d2.y, e2.y - d2.x};
        }
    }
}

// ---------------------------------------------------------------- pass 2
__device__ __forceinline__ void load_bins(const f2 *X, int k, int kn, f2 &xk, f2 &xn)
{
    if (k == 0) {
        const f2 s = X[0];
        xk = f2{s.x, 0.0f};
        xn = f2{s.y, 0.0f};
    } else {
        xk = X[k];
        xn = X[kn];
    }
}

__global__ void __launch_bounds__(TPB) k_phat_pairs(tdoa_kparams kp, tdoa_kout out,
                                                    const f2 *__restrict__ spec, int64_t f_begin,
                                                    int64_t nblocks, float eps2)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *buf = (f2 *)smem;                    // [N]
    float *sc = (float *)(buf + kp.N);       // [K]
    const int N = kp.N, P = kp.P, M = kp.M, K = kp.K, S = kp.S, tid = threadIdx.x;
    // XCD-aware order: consecutive dispatch slots go to different XCDs, so give
    // each XCD a contiguous run of (frame, pair) items -- the P pairs of a frame
    // then read its spectra through one L2
    int64_t b = blockIdx.x;
    if ((nblocks & 7) == 0)
        b = (b & 7) * (nblocks >> 3) + (b >> 3);
    const int64_t fl = b / P;
    const int p = (int)(b - fl * P);
    const f2 *Xi = spec + (size_t)(fl * M + kp.pair_i[p]) * N;
    const f2 *Xj = spec + (size_t)(fl * M + kp.pair_j[p]) * N;

    // R = conj(X_i) X_j / max(|.|, eps);  Y[k] = (R[k] + R*[N-k]) + i (R[k] - R*[N-k]) conj(W_2N^k)
    for (int k = tid; k <= N / 2; k += TPB) {
        const int kn = (N - k) & (N - 1);
        f2 ik, in, jk, jn;
        load_bins(Xi, k, kn, ik, in);
        load_bins(Xj, k, kn, jk, jn);
        f2 Rk = cmul(conj2(ik), jk), Rn = cmul(conj2(in), jn);
        Rk *= __builtin_amdgcn_rsqf(fmaxf(Rk.x * Rk.x + Rk.y * Rk.y, eps2));
        Rn *= __builtin_amdgcn_rsqf(fmaxf(Rn.x * Rn.x + Rn.y * Rn.y, eps2));
        const f2 w2k = ldtw(kp.tw2, k), w2n = ldtw(kp.tw2, N - k);
        buf[k] = (Rk + conj2(Rn)) + mul_i(cmul(Rk - conj2(Rn), conj2(w2k)));
        if (k != 0 && k != N / 2)
            buf[kn] = (Rn + conj2(Rk)) + mul_i(cmul(Rn - conj2(Rk), conj2(w2n)));
    }
    __syncthreads();
    fft_inplace<true>(buf, N, kp.tw);

    // r[s] = y / 2N at s mod 2N:  r[2u] = Re y[u], r[2u+1] = Im y[u]
    const float invL = 1.0f / (float)(2 * N);
    for (int i = tid; i < K; i += TPB) {
        const int s = i - S;
        const int m = s < 0 ? s + 2 * N : s;
        const f2 y = buf[m >> 1];
        sc[i] = ((m & 1) ? y.y : y.x) * invL;
    }
    __syncthreads();
    if (tid < 64) {  // K <= 127: two candidates per lane, ascending lag order
        const int lane = tid, k1 = lane, k2 = lane + 64;
        const float v1 = k1 < K ? sc[k1] : -INFINITY, v2 = k2 < K ? sc[k2] : -INFINITY;
        float bv = v1;
        int bk = k1 < K ? k1 : INT_MAX;
        if (k2 < K && (v2 > bv || bk == INT_MAX)) {
            bv = v2;
            bk = k2;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int ok = __shfl_xor(bk, o, 64);
            if (ov > bv || (ov == bv && ok < bk) || (bk == INT_MAX && ok != INT_MAX)) {
                bv = ov;
                bk = ok;
            }
        }
        bk = __shfl(bk, 0, 64);
        bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);  // NaN scores: keep the index in range
        const int64_t fg = f_begin + fl;
        const size_t gb = (size_t)(fg * P + p) * K;
        if (k1 < K) {
            const int d = k1 > bk ? k1 - bk : bk - k1;
            if (out.scores_f)
                out.scores_f[gb + k1] = v1;
            if (out.weighted_f)
                out.weighted_f[gb + k1] = v1 * kp.prior[d];
        }
        if (k2 < K) {
            const int d = k2 > bk ? k2 - bk : bk - k2;
            if (out.scores_f)
                out.scores_f[gb + k2] = v2;
            if (out.weighted_f)
                out.weighted_f[gb + k2] = v2 * kp.prior[d];
        }
        if (lane == 0)
            out.lags[fg * P + p] = bk - S;
    }
}

__global__ void k_phat_gate(const int32_t *__restrict__ lags, uint8_t *__restrict__ gate, int64_t B,
                            int P)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B)
        return;
    int tot = 0;
    for (int p = 0; p < P; p++) {
        const int b = lags[f * P + p];
        tot += b * b;
    }
    gate[f] = tot > 4 ? 1 : 0;
}

int fail_hip(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

}  // namespace

int64_t tdoa_phat_split_row_bytes(int N) { return (int64_t)N * 8; }

int tdoa_launch_gcc_phat_split(const tdoa_kparams &kp, const tdoa_kout &out,
                               const int16_t *frames, int64_t B, float eps2_int16,
                               void *scratch, size_t scratch_bytes, void *stream)
{
    const int N = kp.N, M = kp.M, P = kp.P;
    if (N < 256 || N > 4096 || (N & (N - 1)))
        return tdoa_set_error(-1, "GCC_PHAT: frame_len must be a power of two in [256, 4096]");
    if (kp.K > 127)
        return tdoa_set_error(-1, "GCC_PHAT: max_shift > 63 not supported");
    if (!scratch)
        return tdoa_set_error(-1, "GCC_PHAT: context has no spectrum scratch");
    const size_t per_frame = (size_t)M * N * sizeof(f2);
    const int64_t chunk = (int64_t)(scratch_bytes / per_frame);
    if (chunk < 1)
        return tdoa_set_error(-1, "GCC_PHAT: spectrum scratch smaller than one frame");
    hipStream_t st = (hipStream_t)stream;
    const size_t lds1 = (size_t)N * sizeof(f2);
    const size_t lds2 = (size_t)N * sizeof(f2) + 128 * sizeof(float);
    for (int64_t c0 = 0; c0 < B; c0 += chunk) {
        const int64_t nf = (B - c0) < chunk ? (B - c0) : chunk;
        if (nf * P > INT_MAX)
            return tdoa_set_error(-1, "GCC_PHAT: chunk too large for one launch");
        hipLaunchKernelGGL(k_phat_spectra, dim3((unsigned)(nf * M)), dim3(TPB), lds1, st, kp, frames,
                           c0 * M, (f2 *)scratch);
        hipLaunchKernelGGL(k_phat_pairs, dim3((unsigned)(nf * P)), dim3(TPB), lds2, st, kp, out,
                           (const f2 *)scratch, c0, nf * P, eps2_int16);
    }
    if (out.gate) {
        const int64_t g = (B + 255) / 256;
        hipLaunchKernelGGL(k_phat_gate, dim3((unsigned)g), dim3(256), 0, st, out.lags, out.gate, B, P);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip(e, "GCC_PHAT split launch");
}
