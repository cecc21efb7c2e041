// tdoa_phat_r16.hip -- GCC-PHAT for the long-frame shapes (frame_len 2048 or
// 4096, any M <= 8: BASELINE configs 3 and 4), two passes per chunk of frames
// through a unit-spectrum scratch sized to stay in the Infinity Cache:
//
//   k_spec16<C>  one workgroup of T = C/16 threads per (frame, mic) row:
//                integer front end (rolling_buffer.c:64-66 floor-mean DC,
//                buffer.c:13-16 low byte, buffer.c:4-11 Q15 window) on the
//                packed samples z[n] = x[2n] + i x[2n+1], a C-point complex
//                FFT as three register passes (radix C/256, 16, 16; Stockham
//                order through one padded LDS buffer), the real-FFT split to
//                X[0..C] of the 2C-point real transform, and the per-mic PHAT
//                factor U = X / max(|X|, sqrt(eps)), stored as C + 1 bins.
//   k_pair16<C>  one workgroup per (frame, pair): R = conj(U_i) U_j is already
//                the unit cross spectrum; the inverse pre-twiddle packs it
//                into C bins whose inverse C-point FFT holds the correlation
//                at even / odd lags in its real / imaginary parts.  Only lags
//                -S..S (S <= 63) are needed, so the inverse is pruned: pass 1
//                in full, pass 2 computes 4 of its 16 outputs, pass 3 one
//                output for 64 of its C/R1 columns.  Then the first argmax and
//                the lag prior (correlations.c:20-33 semantics on float scores).
//
// Thread j of a row holds bins j + T q (q < 16) after the forward transform
// and the same bins of Y before the inverse, so neither end needs a transpose;
// the partner bin C - b of the split and of the pre-twiddle is read from LDS /
// the scratch.  LDS index i is padded to i + i/16 (conflict-free b64 access for
// every pass's stride).  Same definition as oracle/gcc_phat_oracle.py; the PHAT
// factorisation equals its R / max(|R|, eps) whenever |X_i|, |X_j| >= sqrt(eps).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

// the long-frame kernels measured faster with the asm constant-twiddle
// products (k_frame16<2048, 8>: 123.4 vs 127.4 ms per 1e6 frames)
#define TDOA_ASM_MUL_S 1  // pinned asm twiddle products (tdoa_cplx.h)
#include "tdoa_cplx.h"
#include "tdoa_internal.h"
#include "tdoa_keys.h"

int tdoa_set_error(int code, const char *msg);

namespace {

typedef short v2s_r16 __attribute__((ext_vector_type(2)));

// scratch row stride in complex bins: U[0..C] plus padding to 256 B
template <int C>
constexpr int r16_row() { return C + 32; }

__device__ __forceinline__ int pidx(int i) { return i + (i >> 4); }
// LDS reads of the fused long-frame kernels: volatile (never merged into
// ds_read2_b64, which costs twice the LDS cycles of two ds_read_b64) unless
// F16_VLDS=0
#ifndef F16_VLDS
#define F16_VLDS 1
#endif
#ifndef F16_TWPOW
#define F16_TWPOW 1  // the forward's pass-3 twiddles as powers of W_C^j (see frame16_forward)
#endif
// the Q15 window words of config 3's shape (C = 4096) sit in LDS (8 KiB):
// read from L2 at every frame's start, their latency followed the DC barrier
// the prefetched frame words waited for before the output stores (k_frame16)
#ifndef F16_PIN
#define F16_PIN 1
#endif
// the split's twiddles in registers for the launch (see k_frame16)
#ifndef F16_TW_REG
#define F16_TW_REG 1
#endif
// C = 4096 too keeps its window words in registers (F16_WIN_LDS4096=1: the
// LDS copy instead; config 3 3.70 vs 3.62 ms per step, same box)
#ifndef F16_WIN_LDS4096
#define F16_WIN_LDS4096 0
#endif
template <int C>
constexpr bool f16_win_lds()
{
    return C == 4096 && F16_WIN_LDS4096;
}
// the other shapes (C = 2048: LDS is full with the deferred epilogue) keep the
// thread's 8 window words in registers for the launch instead of reading them
// from L2 at every frame's start (F16_WIN_REG=0: from L2)
#ifndef F16_WIN_REG
#define F16_WIN_REG 1
#endif
template <int C>
constexpr int f16_win_mode()
{
    return f16_win_lds<C>() ? 1 : (F16_WIN_REG ? 2 : 0);
}
#if F16_VLDS
#define F16_LD(p) lds_rd(p)
#else
#define F16_LD(p) (*(p))
#endif
// padded offset of o, a multiple of 16: pidx(i + o) == pidx(i) + po(o) -- the
// k_frame16 accesses are a per-thread base plus compile-time offsets (folded
// into the ds instruction) instead of a shift and add per access
__host__ __device__ constexpr int po(int o) { return o + (o >> 4); }
__device__ __forceinline__ f2 lds2(const f2 *buf, int i) { return buf[pidx(i)]; }
__device__ __forceinline__ void sts2(f2 *buf, int i, f2 v) { buf[pidx(i)] = v; }

// k_frame16's transform buffers (F16_XS, default): element i at xs(i) =
// i ^ ((i >> 4) & 15), a permutation inside each aligned 16-element block, no
// padding.  The padded layout (pidx: i + i/16) keeps the 16-lane stride-16
// writes conflict-free, but every 32-lane ds_read_b64 of 32 consecutive
// elements spans 33 slots there, so its first and last lanes share a bank
// (2-way, the read's 2 LDS cycles become 3+).  The swizzle is conflict-free
// for both: a consecutive read stays a permutation of its two aligned 16-blocks,
// and the stride-16 writes 16 j + r land on slots r ^ (j & 15).  Every access
// below is a per-thread base and a compile-time part (an offset, or one XOR)
// -- see ColIdx and the pass writes.  The padding's C / 16 elements per buffer
// are freed (8 KiB at config 4).
// the DM 1 epilogue four pairs per wave (frame16_out16); F16_OUT16=0: a wave
// per pair, two interleaved (frame16_pair_out<2>)
#ifndef F16_OUT16
#define F16_OUT16 1
#endif
// DM 1 with the four-pairs epilogue: the epilogue of frame f runs in frame
// f + 1's forward, after its pass-3 stores (F16_EPI_LAG=0: after frame f's
// last round, the workgroup waiting)
#ifndef F16_EPI_LAG
#define F16_EPI_LAG 1
#endif
// lagged epilogue: the first F16_EPI_SPLIT output waves run after the forward's
// pass-2 stores, the rest after its pass-3 stores (-1: half).  Default 0, all
// after pass 3: half and half measured slower (config 4 90.4 vs 88.5 ms per
// step, config 3 3.57 vs 3.42 -- the pass-2 interval feeds pass 3's VALU-bound DFT)
#ifndef F16_OUT16_LOOPS
// frame16_out16: a loop per output kind under its pointer test (0: one loop
// with the tests inside; 1: config 3 1.925e7 -> 1.967e7, config 4 equal; 2:
// as 1, and with the compact scratch the only weighted output each lag's prior
// read next to its store: config 3 1.966e7 -> 1.980e7, config 4 equal)
#define F16_OUT16_LOOPS 2
#endif
#ifndef F16_EPI_SPLIT
#define F16_EPI_SPLIT 0
#endif
// a barrier between the split (unit spectra) and the first round's Y stores
#ifndef F16_SPLIT_BAR
#define F16_SPLIT_BAR 0
#endif
// a barrier between the forward's pass-3 reads and its stores
#ifndef F16_P3_BAR
#define F16_P3_BAR 0
#endif
// timing only (A/B builds): no per-pair outputs at all (lags, compact scores, grid
// inputs wrong) -- what the output stage costs
#ifndef F16_NO_OUT
#define F16_NO_OUT 0
#endif
#ifndef F16_XS
#define F16_XS 1
#endif
#ifndef F16_PRIO
#define F16_PRIO 0
#endif
// the round's Y[C/2] values: lane-parallel in wave 0 (1) or thread 0 per pair (0):
// config 4 83.7-84.0 vs 85.8-85.9 ms, config 3 3.270-3.277 vs 3.294-3.303 ms per
// step (same box)
#ifndef F16_YHALF
#define F16_YHALF 1
#endif
// the gate's sum of squared lags at P > 16: wave 0's lanes + a DPP sum (1) or thread 0 (0)
#ifndef F16_GATEW
#define F16_GATEW 1
#endif
// the four-pairs epilogue's pairs spread over a multiple of four waves
// (f16_epi_pair).  A/B: config 4 82.8-83.0 vs 82.7-82.9 ms (neutral), config 3
// 3.309 vs 3.279-3.285 ms (slower), same box -- default 0, the packed map
#ifndef F16_EPI_SPREAD
#define F16_EPI_SPREAD 0
#endif
// the lagged epilogue's lambdas forced inline (F16_LAMBDA_AI=0: the inliner
// decides -- an A/B build for the ISA audit only, see DESIGN.md "k_frame16:
// the two unexplained failures")
// TDOA_AB=1: the A/B build (Makefile "ab", tdoa/libtdoa_ab.so for tools and the
// variant tests): k_frame16w and the fused grid (FG) are compiled in; the
// product library holds only the dispatched kernels
#ifndef TDOA_AB
#define TDOA_AB 0
#endif
// the four-pairs epilogue's compact ranges as the wave's four scalar loads
// and a per-lane pick (F16_RNG_SCALAR=1: A/B build for the ISA audit only)
#ifndef F16_RNG_SCALAR
#define F16_RNG_SCALAR 0
#endif
#ifndef F16_LAMBDA_AI
#define F16_LAMBDA_AI 1
#endif
#if F16_LAMBDA_AI
#define F16_AI __attribute__((always_inline))
#else
#define F16_AI
#endif
__host__ __device__ constexpr int xs(int i) { return i ^ ((i >> 4) & 15); }
template <bool XS>
__host__ __device__ constexpr int lidx(int i) { return XS ? xs(i) : pidx(i); }
// buffer length in elements (one group's transform)
template <int C, bool XS>
constexpr int f16_buf() { return XS ? C : C + C / 16; }
// element j + T r (T = C / 16, j < T, r a compile-time constant after
// unrolling) of a group buffer: xs(j + T r) = T r + (xs(j) ^ ((T r >> 4) & 15)),
// which is xs(j) + T r at T = 256 and (xs(j) ^ 8 (r & 1)) + T r at T = 128
template <int C, bool XS>
struct ColIdx {
    int b0, b1;
    __device__ __forceinline__ explicit ColIdx(int j)
    {
        static_assert(C == 2048 || C == 4096, "k_frame16 shapes");
        b0 = XS ? xs(j) : pidx(j);
        b1 = XS && C == 2048 ? (b0 ^ 8) : b0;
    }
    __device__ __forceinline__ int at(int r) const
    {
        constexpr int T = C / 16;
        return XS ? ((r & 1) ? b1 : b0) + T * r : b0 + po(T * r);
    }
};

template <int R>
__device__ constexpr int brev(int k)
{
    return R == 16 ? (((k & 1) << 3) | ((k & 2) << 1) | ((k & 4) >> 1) | ((k & 8) >> 3))
                   : (((k & 1) << 2) | (k & 2) | ((k & 4) >> 2));
}

// F16_PRIO (A/B builds): progress-balanced issue priority in k_frame16.  The
// four waves of a SIMD issue oldest-first, so inside every barrier interval they
// finish one after another (waves 0-3 / 4-7 / 8-11 / 12-15 of config 4's
// forward pass 1: 1090 / 1610 / 2125 / 2690 cycles) and the last one runs
// alone, without latency cover, while the others wait at the barrier.  Every
// wave takes priority 3 after a barrier and lowers it at checkpoints inside the
// interval's work (1: the middle of each DFT, of the split and of the Y build;
// 2: every DFT stage), so a wave that is ahead yields issue to the ones behind
template <int L>
__device__ __forceinline__ void f16_prio()
{
#if F16_PRIO
    __builtin_amdgcn_s_setprio(L);
#endif
}

// in-place radix-2 DIF DFT-R (R = 8, 16) on the packed primitives: natural-order
// input, X[k] ends in v[brev<R>(k)].  HZ: inputs R/2..R-1 are zero.  The
// butterfly twiddle of span s is W_{2s}^j = W_32^{16 j / s}.  PM: k_frame16's
// priority checkpoints (F16_PRIO)
template <int R, bool INV, bool HZ, int PM = 0>
__device__ __forceinline__ void dftp(f2 (&v)[R])
{
    constexpr int LOG2R = R == 16 ? 4 : 3;
#pragma unroll
    for (int st = 0; st < LOG2R; st++) {  // linear stage index: fully unrolled
        if constexpr (PM == 1) {
            if (st == LOG2R / 2)
                f16_prio<1>();
        } else if constexpr (PM == 2) {
            if (st == 1)
                f16_prio<2>();
            else if (st == 2)
                f16_prio<1>();
            else if (st == 3)
                f16_prio<0>();
        }
        const int span = R >> (st + 1);
#pragma unroll
        for (int start = 0; start < R; start += 2 * span) {
#pragma unroll
            for (int j = 0; j < span; j++) {
                const int k = j * (16 / span);
                if (HZ && span == R / 2) {
                    v[j + span] = tw_only<INV>(v[j], k);
                } else {
                    const f2 a = v[start + j], b = v[start + j + span];
                    v[start + j] = a + b;
                    v[start + j + span] = dif_tw<INV>(a, b, k);
                }
            }
        }
    }
}

// coalesced twiddles (kp.r16_tw): [0][r][k] W_C^{R1 r k} = W_256^{r k},
// [1][r][l] W_C^{r l}, [2][r][h] W_C^{16 r h}; W_C^{r x} (x < 256) = [1][r][x&15] [2][r][x>>4]
__device__ __forceinline__ f2 tw256(const f2 *tt, int r, int k) { return tt[16 * r + k]; }
__device__ __forceinline__ f2 tw16h(const f2 *tt, int r, int h) { return tt[512 + 16 * r + h]; }
__device__ __forceinline__ f2 twC(const f2 *tt, int r, int x)
{
    return c_mul(tt[256 + 16 * r + (x & 15)], tt[512 + 16 * r + (x >> 4)]);
}

__device__ __forceinline__ int block_sum(int s, int *red)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0)
        red[threadIdx.x >> 6] = s;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++)
        t += red[w];
    return t;
}

// ------------------------------------------------------------------ pass 1
template <int C>
__global__ void __launch_bounds__(C / 16, 4) k_spec16(tdoa_kparams kp, const int16_t *__restrict__ frames,
                                                      int64_t row0, f2 *__restrict__ spec, float e2)
{
    constexpr int T = C / 16, R1 = C / 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *buf = (f2 *)smem;  // [C + C/16]
    __shared__ int red[T / 64];
    const int j = threadIdx.x;
    const int64_t row = row0 + blockIdx.x;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(frames + row * (int64_t)C);
    const uint32_t *win = reinterpret_cast<const uint32_t *>(kp.window);
    const f2 *tw2 = reinterpret_cast<const f2 *>(kp.tw2);
    const f2 *tt = reinterpret_cast<const f2 *>(kp.r16_tw);

    // words j + T s (s < 8) = samples 2(j + T s), +1 = z[j + T s]
    uint32_t w[8], wn[8];
#pragma unroll
    for (int s = 0; s < 8; s++)
        w[s] = __builtin_nontemporal_load(x + j + T * s);
#pragma unroll
    for (int s = 0; s < 8; s++)
        wn[s] = win[j + T * s];
    int sum = 0;
#pragma unroll
    for (int s = 0; s < 8; s++)
        sum = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s_r16, w[s]), v2s_r16{1, 1}, sum, false);
    sum = block_sum(sum, red);
    // floor-mean DC (int64 arithmetic shift == floor); x <<= 8 keeps the low
    // byte of x - off; ((s << 8) * W) >> 15 == floor(s * W / 128), exact in fp32
    const uint32_t off = (uint32_t)(sum >> kp.log2N) & 0xFFu;
    const uint32_t off2 = off | (off << 16);
    f2 v[16];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const uint32_t d = (w[s] | 0x01000100u) - off2;  // no borrow across the halves
        const float s0 = (float)(int8_t)(d & 0xFFu), s1 = (float)(int8_t)((d >> 16) & 0xFFu);
        const float w0 = (float)(int16_t)(wn[s] & 0xFFFFu) * (1.0f / 128.0f);
        const float w1 = (float)(int16_t)(wn[s] >> 16) * (1.0f / 128.0f);
        v[s] = f2{floorf(s0 * w0), floorf(s1 * w1)};
    }

    // Stockham pass 1 (radix R1, Ns = 1): virtual thread j' reads z[j' + 256 r]
    if constexpr (R1 == 16) {
#pragma unroll
        for (int s = 8; s < 16; s++)
            v[s] = f2{0.0f, 0.0f};
        dftp<16, false, true>(v);
#pragma unroll
        for (int r = 0; r < 16; r++)
            sts2(buf, 16 * j + r, v[brev<16>(r)]);
    } else {  // R1 = 8, T = 128: j' = j (z = v[2r]) and j + 128 (z = v[2r + 1])
#pragma unroll
        for (int h = 0; h < 2; h++) {
            f2 u[8];
#pragma unroll
            for (int r = 0; r < 4; r++)
                u[r] = v[2 * r + h];
#pragma unroll
            for (int r = 4; r < 8; r++)
                u[r] = f2{0.0f, 0.0f};
            dftp<8, false, true>(u);
            const int jv = j + 128 * h;
#pragma unroll
            for (int r = 0; r < 8; r++)
                sts2(buf, 8 * jv + r, u[brev<8>(r)]);
        }
    }
    __syncthreads();

    // pass 2 (radix 16, Ns = R1): twiddle W_{16 R1}^{r k} = W_C^{16 r k}, k = j mod R1
    {
        const int k = j % R1;
        f2 t[16];
#pragma unroll
        for (int r = 1; r < 16; r++)
            t[r] = tw16h(tt, r, k);  // W_C^{16 r k}
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = lds2(buf, j + T * r);
#pragma unroll
        for (int r = 1; r < 16; r++)
            v[r] = c_mul(v[r], t[r]);
        dftp<16, false, false>(v);
        __syncthreads();
        const int o = (j / R1) * 16 * R1 + k;
#pragma unroll
        for (int r = 0; r < 16; r++)
            sts2(buf, o + R1 * r, v[brev<16>(r)]);
    }
    __syncthreads();

    // pass 3 (radix 16, Ns = T): twiddle W_C^{r j}; outputs Z[j + T r] stay here
    f2 Z[16];
    {
        f2 t[16];
#pragma unroll
        for (int r = 1; r < 16; r++)
            t[r] = twC(tt, r, j);
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = lds2(buf, j + T * r);
#pragma unroll
        for (int r = 1; r < 16; r++)
            v[r] = c_mul(v[r], t[r]);
        dftp<16, false, false>(v);
#pragma unroll
        for (int r = 0; r < 16; r++)
            Z[r] = v[brev<16>(r)];
    }
    __syncthreads();

    // real-FFT split (x2): X[b] = (Z[b] + Z*[C-b]) - i W_2C^b (Z[b] - Z*[C-b]), b = j + T q
#pragma unroll
    for (int q = 0; q < 16; q++)
        sts2(buf, j + T * q, Z[q]);
    __syncthreads();
    f2 *o = spec + (size_t)blockIdx.x * r16_row<C>();
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int b = j + T * q;
        const f2 zp = lds2(buf, (C - b) & (C - 1));
        const f2 e = c_addconj(Z[q], zp);
        const f2 od = c_mul(c_subconj(Z[q], zp), tw2[b]);
        o[b] = c_unit(c_add_mi(e, od), e2);
    }
    if (j == 0)  // X[C] = 2 (Re Z[0] - Im Z[0]), real
        o[C] = c_unit(f2{2.0f * (Z[0].x - Z[0].y), 0.0f}, e2);
}

// ------------------------------------------------------------------ pass 2
template <int C>
__global__ void __launch_bounds__(C / 16, 6) k_pair16(tdoa_kparams kp, tdoa_kout out,
                                                      const f2 *__restrict__ spec, int64_t f_begin,
                                                      int64_t nblocks)
{
    constexpr int T = C / 16, R1 = C / 256, RS = r16_row<C>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *buf = (f2 *)smem;  // [C/2 + C/32]: half of the padded C-point buffer
    const int j = threadIdx.x, P = kp.P, M = kp.M, K = kp.K, S = kp.S;
    const f2 *tw2 = reinterpret_cast<const f2 *>(kp.tw2);
    const f2 *tt = reinterpret_cast<const f2 *>(kp.r16_tw);
    // XCD-aware order: each XCD gets a contiguous run of (frame, pair) items,
    // so the P pairs of a frame read its M unit spectra through one L2
    int64_t bi = blockIdx.x;
    if ((nblocks & 7) == 0)
        bi = (bi & 7) * (nblocks >> 3) + (bi >> 3);
    const int64_t fl = bi / P;
    const int p = (int)(bi - fl * P);
    const f2 *Ui = spec + (size_t)(fl * M + kp.pair_i[p]) * RS;
    const f2 *Uj = spec + (size_t)(fl * M + kp.pair_j[p]) * RS;

    // Y[b] = s + i q with s = R[b] + R*[C-b], q = (R[b] - R*[C-b]) conj(W_2C^b),
    // R = conj(U_i) U_j; and, from the same four bins, Y[C-b] = conj(s - i q)
    // (W_2C^{C-b} = -conj(W_2C^b)).  Thread j computes b = j + T r for r < 8 and
    // the partners C - b, which are the bins r >= 8 of thread T - j (thread 0:
    // its own, plus the self-paired C/2): one read of every U bin per pair.
    f2 v[16];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int b = j + T * r, pb = C - b;  // b = 0 pairs with bin C
        const f2 Rk = c_conjmul(Ui[b], Uj[b]), Rn = c_conjmul(Ui[pb], Uj[pb]);
        const f2 s = c_addconj(Rk, Rn);
        const f2 qq = c_mulconj(c_subconj(Rk, Rn), tw2[b]);
        v[r] = c_add_i(s, qq);
        if (b != 0)
            sts2(buf, pb - C / 2, c_conj_add_mi(s, qq));  // pb in (C/2, C)
    }
    if (j == 0) {  // Y[C/2] from R[C/2] alone
        const f2 Rh = c_conjmul(Ui[C / 2], Uj[C / 2]);
        sts2(buf, 0, c_add_i(c_addconj(Rh, Rh), c_mulconj(c_subconj(Rh, Rh), tw2[C / 2])));
    }
    __syncthreads();
#pragma unroll
    for (int r = 8; r < 16; r++)
        v[r] = lds2(buf, j + T * r - C / 2);
    __syncthreads();  // the exchange slots are overwritten by pass 1

    // inverse pass 1 (radix 16, Ns = 1) straight from the registers; its
    // outputs 16 j + r'' go through the half-size buffer in two rounds
    // (threads j < T/2 write positions [0, C/2), then the rest), and pass 2
    // (radix 16, Ns = 16) accumulates its DIF halves v[r], v[r + 8] per round
    dftp<16, true, false>(v);
    const int k = j & 15;
    f2 a[8], d[8];
    if (j < T / 2) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            sts2(buf, 16 * j + r, v[brev<16>(r)]);
    }
    __syncthreads();
    f2 h0[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        h0[r] = lds2(buf, j + T * r);
        if (r)
            h0[r] = c_mulconj(h0[r], tw256(tt, r, k));
    }
    __syncthreads();
    if (j >= T / 2) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            sts2(buf, 16 * j + r - C / 2, v[brev<16>(r)]);
    }
    __syncthreads();
    // pass 2 outputs r'' in {0, 1, 14, 15} only: the last pass reads columns
    // j' mod 256 in [0, 32) u [224, 256)
    {
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const f2 hi = c_mulconj(lds2(buf, j + T * (r + 8) - C / 2), tw256(tt, r + 8, k));
            a[r] = h0[r] + hi;
            d[r] = dif_tw<true>(h0[r], hi, 2 * r);
        }
        // X0 = sum a, X1 = sum d, X14 = sum_{r<4} (a_r - a_{r+4}) W_8^r, X15 likewise on d
        f2 x0 = a[0], x1 = d[0], x14 = a[0] - a[4], x15 = d[0] - d[4];
#pragma unroll
        for (int r = 1; r < 8; r++) {
            x0 = x0 + a[r];
            x1 = x1 + d[r];
        }
#pragma unroll
        for (int r = 1; r < 4; r++) {
            x14 = x14 + dif_tw<false>(a[r], a[r + 4], 4 * r);
            x15 = x15 + dif_tw<false>(d[r], d[r + 4], 4 * r);
        }
        __syncthreads();
        // compact: block q = j / 16 of 64 slots holding offsets k, 16 + k,
        // 224 + k, 240 + k of the 256-column block (lane l of pass 3 reads 64 r + l)
        const int o = (j >> 4) * 64 + k;
        sts2(buf, o, x0);
        sts2(buf, o + 16, x1);
        sts2(buf, o + 32, x14);
        sts2(buf, o + 48, x15);
    }
    __syncthreads();
    if (j >= 64)
        return;

    // inverse pass 3 (radix R1, Ns = 256), one output per column:
    //   lane l < 32:  column j' = l, output 0 -> y[l]
    //   lane l >= 32: column j' = 192 + l, output R1 - 1 -> y[C - m], m = 64 - l
    const int l = j;
    const int jc = l < 32 ? l : 192 + l;
    const int m = 64 - l;
    f2 y = lds2(buf, l);
#pragma unroll
    for (int r = 1; r < R1; r++) {
        const f2 u = lds2(buf, 64 * r + l);
        y = y + (l < 32 ? c_mulconj(u, twC(tt, r, jc)) : c_mul(u, twC(tt, r, m)));
    }
    // y[n] = r[2n] + i r[2n+1]: lags 2n, 2n + 1 with n = l or -m
    const float invL = 1.0f / (float)(2 * C);
    const int n = l < 32 ? l : -m;
    const int ka = 2 * n + S, kb = 2 * n + 1 + S;
    const bool oka = ka >= 0 && ka < K, okb = kb >= 0 && kb < K;
    const float sa = y.x * invL, sb = y.y * invL;
    // first maximum (the lowest lag wins ties), by keys to every lane
    int bkey = INT_MIN, bk = INT_MAX;
    if (oka) {
        bkey = fkey(sa);
        bk = ka;
    }
    if (okb && fkey(sb) > bkey) {
        bkey = fkey(sb);
        bk = kb;
    }
    wave_argmax_key(bkey, bk);
    bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);  // NaN scores: keep the index in range
    const int64_t fg = f_begin + fl;
    const size_t gb = (size_t)(fg * P + p) * K;
    if (oka) {
        const int dd = ka > bk ? ka - bk : bk - ka;
        if (out.scores_f)
            out.scores_f[gb + ka] = sa;
        if (out.weighted_f)
            out.weighted_f[gb + ka] = sa * kp.prior[dd];
    }
    if (okb) {
        const int dd = kb > bk ? kb - bk : bk - kb;
        if (out.scores_f)
            out.scores_f[gb + kb] = sb;
        if (out.weighted_f)
            out.weighted_f[gb + kb] = sb * kp.prior[dd];
    }
    if (l == 0)
        out.lags[fg * P + p] = bk - S;
}

// ------------------------------------------------------------ fused, per frame
// k_frame16<C, M>: one workgroup of 1024 threads per frame; the unit spectra
// never leave the chip (the two-pass pair above writes them to a scratch and
// reads them back, ~4x the frame's own bytes).  G = 16384 / C groups of
// T = C / 16 threads (C = 4096: 4 groups, C = 2048: 8), M <= G mics.  The
// pairs are the host's lexicographic (i, j) order resolved at compile time (a
// runtime pair index selected each spectrum through M-way v_cndmask chains,
// which cost more than the transforms), and the twiddle tables are staged in
// LDS (each pass reads them right after a barrier):
//  1. forward: group g runs k_spec16's front end and three register passes on
//     mic g in LDS slot g (padded C-point buffer); every thread then reads, for
//     every mic, its bin-pair slots (b, C - b), b = tid + 1024 s (s < C / 2048),
//     and keeps the split + PHAT-normalised U_m[b], U_m[C - b] in registers
//     (thread 0 also U_m[C / 2], through LDS);
//  2. pairs, G at a time: every thread writes the packed inverse input of its
//     slots (k_pair16's pre-twiddle) for each pair of the round into that
//     pair's buffer; group g then runs k_pair16's pruned inverse (pass 1 full,
//     pass 2 outputs {0, 1, 14, 15}, pass 3 one output for 64 columns), the
//     first argmax and the lag prior;
//  3. gate from the frame's lags.
// a thread index the compiler cannot prove loop-invariant: keeps twiddle
// loads inside the pair-round loop instead of hoisted (and spilled) above it
__device__ __forceinline__ int opaque_idx(int t)
{
    asm volatile("" : "+v"(t));
    return t;
}

// the four-pairs epilogue's lane -> pair map (frame16_out16: a 16-lane row per
// pair): packed, wave w row q = pair 4 w + q (waves 0 .. 6 at config 4: SIMDs
// 0-2 get eight pairs, SIMD 3 four); F16_EPI_SPREAD=1 (A/B): EW = ceil(P / 4)
// rounded up to a multiple of four waves, wave w < EW row q takes pair w + EW q,
// equal shares per SIMD (measured no faster).
// P: the lane has no pair
template <int P>
__device__ __forceinline__ constexpr int f16_epi_waves()
{
    return F16_EPI_SPREAD ? ((((P + 3) / 4 + 3) & ~3) < 16 ? (((P + 3) / 4 + 3) & ~3) : 16) : (P + 3) / 4;
}
template <int P>
__device__ __forceinline__ int f16_epi_pair(int t)
{
    constexpr int EW = f16_epi_waves<P>();
    const int w = t >> 6, q = (t >> 4) & 3;
    const int p = F16_EPI_SPREAD ? w + EW * q : 4 * w + q;
    return w < EW && p < P ? p : P;
}

// pairs in the host's lexicographic order (tdoa_capi.cpp): pair p = (i, j)
template <int M>
__host__ __device__ constexpr int pair_first(int p)
{
    int i = 0;
    while (p >= M - 1 - i) {
        p -= M - 1 - i;
        i++;
    }
    return i;
}
template <int M>
__host__ __device__ constexpr int pair_second(int p)
{
    int i = 0;
    while (p >= M - 1 - i) {
        p -= M - 1 - i;
        i++;
    }
    return i + 1 + p;
}
static_assert(pair_first<4>(5) == 2 && pair_second<4>(5) == 3 && pair_second<8>(6) == 7, "pair order");

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

#ifdef TDOA_DIAG
// diagnostic build only: s_memtime per phase boundary (32 per wave: stamps
// 0..28, [29] end of the stamped frame, [30] / [31] realtime start / end), per
// wave of the first 128 workgroups.  The stamped frame is the workgroup's
// frame number F16_DIAG_FRAME (default 2: steady state, not the cold start)
#ifndef F16_DIAG_FRAME
#define F16_DIAG_FRAME 2
#endif
__device__ unsigned long long g_diag_f16[1 << 16];
// ... and each wave's arrival at the stamped frame's barriers (g_diag_f16b,
// NSTAMP per wave): arrival -> the next stamp is the wave's barrier wait
__device__ unsigned long long g_diag_f16b[1 << 16];
#define F16_MARK()                                       \
    do {                                                 \
        if (nst < NSTAMP - 3)                            \
            stamp[nst++] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define F16_PRE()                                        \
    do {                                                 \
        if (nar < NSTAMP)                                \
            arrive[nar++] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define F16_MARK() \
    do {           \
    } while (0)
#define F16_PRE() \
    do {          \
    } while (0)
#endif

// forward transform of mic g by its group of T threads (k_spec16's front end
// and three register passes in the group's LDS slot buf): the DC sum of the
// group's words w, the Q15 window, radix R1 / 16 / 16 Stockham passes; Z[j + T q]
// ends in buf at pidx(j + T q), after a closing barrier
// WM: where the thread's window words come from -- 0 global (L2), 1 LDS (win
// is the LDS copy), 2 registers (wr, loaded once per launch)
struct NoHook16 {
    __device__ void operator()(int) const {}
};
struct NoPre16 {  // pre_h(): right before each of the forward's barriers (diagnostic arrival stamps)
    __device__ void operator()() const {}
};
// hook(2) / hook(3): called once every thread's pass-2 / pass-3 stores are
// issued, before the pass's closing barrier (LDS-store-bound intervals whose
// VALU is idle):
// k_frame16's lagged epilogue runs the previous frame's outputs there
template <int C, int WM, typename Mark, bool XS = false, typename Hook = NoHook16, typename Pre = NoPre16>
__device__ __forceinline__ void frame16_forward(const uint32_t (&w)[8], const uint32_t *win, const uint32_t (&wr)[8],
                                                f2 *buf, int *red, const f2 *tt, int tid, int g, int j, int pj,
                                                int log2N, Mark mark, Hook hook = Hook(), Pre pre_h = Pre())
{
    constexpr int T = C / 16, R1 = C / 256;
    const ColIdx<C, XS> cj(j);  // XS: pj is unused (the column reads / writes go through cj)
    uint32_t wn[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        if constexpr (WM == 2)
            wn[s] = wr[s];
        else if constexpr (WM == 1)
            wn[s] = lds_rd_u32(win + j + T * s);
        else
            wn[s] = win[j + T * s];
    }
    int sum = 0;
#pragma unroll
    for (int s = 0; s < 8; s++)
        sum = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s_r16, w[s]), v2s_r16{1, 1}, sum, false);
    sum = group_sum_dpp(sum, 64);  // DPP moves to lane 63 (no LDS round trips)
    if ((tid & 63) == 63)
        red[tid >> 6] = sum;
    pre_h();
    __syncthreads();
    f16_prio<3>();
    mark();
    sum = 0;
#pragma unroll
    for (int wv = 0; wv < T / 64; wv++)
        sum += red[g * (T / 64) + wv];
    const uint32_t off = (uint32_t)(sum >> log2N) & 0xFFu;
    const uint32_t off2 = off | (off << 16);
    f2 v[16];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const uint32_t d = (w[s] | 0x01000100u) - off2;
        const float s0 = (float)(int8_t)(d & 0xFFu), s1 = (float)(int8_t)((d >> 16) & 0xFFu);
        const float w0 = (float)(int16_t)(wn[s] & 0xFFFFu) * (1.0f / 128.0f);
        const float w1 = (float)(int16_t)(wn[s] >> 16) * (1.0f / 128.0f);
        v[s] = f2{floorf(s0 * w0), floorf(s1 * w1)};
    }
    if constexpr (R1 == 16) {
#pragma unroll
        for (int s = 8; s < 16; s++)
            v[s] = f2{0.0f, 0.0f};
        dftp<16, false, true, F16_PRIO>(v);
        // element 16 j + r: pidx = 17 j + r; xs = (16 j | (j & 15)) ^ r
        const int b1 = 16 * j | (j & 15);
#pragma unroll
        for (int r = 0; r < 16; r++)
            buf[XS ? (b1 ^ r) : 17 * j + r] = v[brev<16>(r)];
    } else {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            f2 u[8];
#pragma unroll
            for (int r = 0; r < 4; r++)
                u[r] = v[2 * r + h];
#pragma unroll
            for (int r = 4; r < 8; r++)
                u[r] = f2{0.0f, 0.0f};
            dftp<8, false, true, F16_PRIO>(u);
            // element 8 (j + 128 h) + r (r < 8): pidx = 8 j + (j >> 1) + 1088 h + r;
            // xs = 1024 h + ((16 (j >> 1) | (8 (j & 1) ^ ((j >> 1) & 15))) ^ r)
            const int b2 = 16 * (j >> 1) | ((8 * (j & 1)) ^ ((j >> 1) & 15));
#pragma unroll
            for (int r = 0; r < 8; r++)
                buf[XS ? 1024 * h + (b2 ^ r) : 8 * j + (j >> 1) + 1088 * h + r] = u[brev<8>(r)];
        }
    }
    pre_h();
    __syncthreads();
    f16_prio<3>();
    mark();
    {
        const int k = j % R1;
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = F16_LD(buf + (XS ? cj.at(r) : pj + po(T * r)));
#pragma unroll
        for (int r = 1; r < 16; r++)
            v[r] = c_mul(v[r], F16_LD(tt + 512 + 16 * r + k));  // tw16h
        dftp<16, false, false, F16_PRIO>(v);
        pre_h();
        __syncthreads();
        f16_prio<3>();
    mark();
        // element (j / R1) 16 R1 + k + R1 r.  pad: o mod 16 = k < R1, so
        // pidx(o + R1 r) = pidx(o) + R1 r + R1 r / 16.  xs: the lane part
        // (256 (j / 16) | k at R1 = 16; 128 (j / 8) | 8 ((j / 8) & 1) | k at R1 = 8)
        // XOR a compile-time part (17 r; 16 (r / 2) | 8 (r & 1) | r / 2)
        const int o = pidx((j / R1) * 16 * R1 + k);
        const int lv = R1 == 16 ? (256 * (j / 16) | k) : (128 * (j / 8) | 8 * ((j / 8) & 1) | k);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int cr = R1 == 16 ? 17 * r : (16 * (r / 2) | 8 * (r & 1) | (r / 2));
            buf[XS ? (lv ^ cr) : o + R1 * r + (R1 * r >> 4)] = v[brev<16>(r)];
        }
    }
    f16_prio<3>();  // F16_PRIO: the lagged epilogue is the interval's critical path
    hook(2);
    pre_h();
    __syncthreads();
    f16_prio<3>();
    mark();
    {
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = F16_LD(buf + (XS ? cj.at(r) : pj + po(T * r)));
#if F16_TWPOW
        {
            // W_C^{r j}, r = 1..15, as powers of W_C^j (the tables give W_C^j
            // in one product; then squares and one-step products, depth <= 5):
            // two LDS reads instead of thirty per thread
            f2 t[16];
            t[1] = c_mul(F16_LD(tt + 256 + 16 + (j & 15)), F16_LD(tt + 512 + 16 + (j >> 4)));
#pragma unroll
            for (int r = 2; r < 16; r++)
                t[r] = (r & 1) ? c_mul(t[r - 1], t[1]) : c_mul(t[r / 2], t[r / 2]);
#pragma unroll
            for (int r = 1; r < 16; r++)
                v[r] = c_mul(v[r], t[r]);
        }
#else
#pragma unroll
        for (int r = 1; r < 16; r++)
            v[r] = c_mul(v[r], c_mul(F16_LD(tt + 256 + 16 * r + (j & 15)), F16_LD(tt + 512 + 16 * r + (j >> 4))));  // twC
#endif
        dftp<16, false, false, F16_PRIO>(v);
        // the pass's stores go to exactly the 16 positions this thread read (its
        // column): no barrier between the reads and the stores (F16_P3_BAR=1: one)
#if F16_P3_BAR
        pre_h();
        __syncthreads();
        f16_prio<3>();
#endif
    mark();
#pragma unroll
        for (int q = 0; q < 16; q++)  // Z[j + T q] back into the slot
            buf[XS ? cj.at(q) : pj + po(T * q)] = v[brev<16>(q)];
    }
    f16_prio<3>();
    hook(3);
    pre_h();
    __syncthreads();
    f16_prio<3>();
    mark();
}

// LDS bytes of k_frame16
template <int C, bool XS = (F16_XS != 0)>
constexpr size_t frame16_lds_base()
{
    constexpr int G = 16384 / C, BUF = f16_buf<C, XS>();
    return (size_t)G * BUF * sizeof(f2) + G * sizeof(f2) + 16 * 4 + TDOA_MAX_PAIRS * 4 +
           3 * 16 * 16 * sizeof(f2) + 128 * sizeof(float) + (size_t)(C / 256) * 64 * sizeof(f2) +
           (f16_win_lds<C>() ? (size_t)C * 2 : 0);
}

// The output block read through an opaque kernarg pointer: loads used once
// per frame (the least-squares lags) stay where they are used instead of being
// hoisted out of the frame loop and held in scalar registers across the
// transforms.  kp and out are the kernel's first two arguments (kernarg
// offsets 0 and sizeof(kp) rounded to 8).  The pointer keeps the constant
// address space: its loads are scalar (s_load, lgkmcnt only).  A generic
// pointer made them flat loads, whose vmcnt wait also waited for the next
// frame's prefetched words.
typedef __attribute__((address_space(4))) const char kchar;
__device__ __forceinline__ kchar *kernarg_base()
{
    kchar *k = (kchar *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return k;
}
// The offset below holds only while both structs are 8-byte aligned and
// (kp, out) stay k_frame16's first two parameters.
static_assert(alignof(tdoa_kparams) <= 8 && alignof(tdoa_kout) == 8,
              "kernarg_out(): tdoa_kout must sit at sizeof(tdoa_kparams) rounded to 8");
__device__ __forceinline__ const __attribute__((address_space(4))) tdoa_kout *kernarg_out()
{
    return reinterpret_cast<const __attribute__((address_space(4))) tdoa_kout *>(
        kernarg_base() + ((sizeof(tdoa_kparams) + 7) & ~(size_t)7));
}

// The outputs of NP pairs from one wave (NP = 2: two independent argmax
// chains interleaved): lane l holds pair h's raw scores sa[h], sb[h] at lags
// ka, kb (valid where oka / okb; on[h] false: no pair h).  The first maximum
// (the lowest lag wins ties) by keys to every lane, then the lag prior
// (correlations.c:20-33 semantics on float scores), scores / weighted scores,
// the compact weighted scratch of k_grid_bb, the least-squares peak scores and
// the lag.  wlo, ww, woff: each pair's compact-scratch range (kp.wc_lo /
// wc_w / wc_off), passed in: a kp byte indexed by a runtime pair is a VMEM
// load whose vmcnt wait would also wait for the next frame's prefetched words.
template <int NP>
__device__ __forceinline__ void frame16_pair_out(const tdoa_kparams &kp, const tdoa_kout &out,
                                                 const float *priorl, int *lagl, int64_t fr, int P,
                                                 const int (&p)[NP], const bool (&on)[NP], int ka, int kb,
                                                 bool oka, bool okb, const float (&sa)[NP], const float (&sb)[NP],
                                                 bool lane0, const int (&wlo)[NP], const int (&ww)[NP],
                                                 const int (&woff)[NP], float *wl = nullptr)
{
    const int K = kp.K, S = kp.S;
    int bkey[NP], bk[NP];
#pragma unroll
    for (int h = 0; h < NP; h++) {
        bkey[h] = INT_MIN;
        bk[h] = INT_MAX;
        if (oka) {
            bkey[h] = fkey(sa[h]);
            bk[h] = ka;
        }
        if (okb && fkey(sb[h]) > bkey[h]) {
            bkey[h] = fkey(sb[h]);
            bk[h] = kb;
        }
    }
    int mk[NP];
#pragma unroll
    for (int h = 0; h < NP; h++)
        mk[h] = wave_reduce<true>(bkey[h]);
#pragma unroll
    for (int h = 0; h < NP; h++)
        bk[h] = wave_reduce<false>(bkey[h] == mk[h] ? bk[h] : INT_MAX);
    float *wc = kernarg_out()->weighted_c;
    float *pk3 = kernarg_out()->peak3;
#pragma unroll
    for (int h = 0; h < NP; h++) {
        if (!on[h])
            break;
        const int b = bk[h] < 0 ? 0 : (bk[h] >= K ? K - 1 : bk[h]);  // NaN scores: keep the index in range
        const size_t gb = (size_t)(fr * P + p[h]) * K;
        float *wcp = wc ? wc + (size_t)fr * kp.wc_CK + woff[h] - wlo[h] : nullptr;
        float *wlp = wl ? wl + woff[h] - wlo[h] : nullptr;  // FG: the frame's compact scores in LDS
        if (oka) {
            const int dd = ka > b ? ka - b : b - ka;
            const float wa = sa[h] * priorl[dd];
            if (out.scores_f)
                out.scores_f[gb + ka] = sa[h];
            if (out.weighted_f)
                out.weighted_f[gb + ka] = wa;
            if (wcp && ka >= wlo[h] && ka < wlo[h] + ww[h])
                wcp[ka] = wa;
            if (wlp && ka >= wlo[h] && ka < wlo[h] + ww[h])
                wlp[ka] = wa;
        }
        if (okb) {
            const int dd = kb > b ? kb - b : b - kb;
            const float wb = sb[h] * priorl[dd];
            if (out.scores_f)
                out.scores_f[gb + kb] = sb[h];
            if (out.weighted_f)
                out.weighted_f[gb + kb] = wb;
            if (wcp && kb >= wlo[h] && kb < wlo[h] + ww[h])
                wcp[kb] = wb;
            if (wlp && kb >= wlo[h] && kb < wlo[h] + ww[h])
                wlp[kb] = wb;
        }
        if (pk3) {
            // the least-squares refinement's raw scores around the peak: the
            // lanes holding lags b - 1 .. b + 1 store them
            float *dst = pk3 + (size_t)(fr * P + p[h]) * 3 + 1 - b;
            if (oka && ka >= b - 1 && ka <= b + 1)
                dst[ka] = sa[h];
            if (okb && kb >= b - 1 && kb <= b + 1)
                dst[kb] = sb[h];
        }
        if (lane0) {
            out.lags[fr * P + p[h]] = b - S;
            lagl[p[h]] = b - S;
        }
    }
}

// The DM 1 epilogue's outputs, four pairs per wave: 16-lane row q of the wave
// takes pair p, lane r of the row its lags r + 16 i (i < KL; K <= 16 KL).  The
// first maximum is a row reduction (four DPP steps, no cross-row moves) and
// every row instruction serves four pairs, where frame16_pair_out spends a
// whole wave (and a wave reduction) on one -- its VALU work, 8 % of a config-4
// frame, was the epilogue's cost.  Same values, same tie rule (ascending lags
// per lane with a strict '>', then the smallest lag among equal keys), same
// stores.  wlo, ww, woff: this lane's pair's compact-scratch range.
template <int KL, bool SPLIT = (F16_OUT16_LOOPS != 0)>
__device__ __forceinline__ void frame16_out16(const tdoa_kparams &kp, const tdoa_kout &out, const float *scl,
                                              const float *priorl, int *lagl, int64_t fr, int P, int p, int r,
                                              int wlo, int ww, int woff)
{
    const int K = kp.K, S = kp.S;
    float sv[KL];
    int bkey = INT_MIN, bk = INT_MAX;
#pragma unroll
    for (int i = 0; i < KL; i++) {
        const int k = r + 16 * i;
        sv[i] = k < K ? scl[p * K + k] : 0.0f;
        const int key = fkey(sv[i]);
        if (k < K && key > bkey) {
            bkey = key;
            bk = k;
        }
    }
    const int mk = row_reduce<true>(bkey);
    bk = row_reduce<false>(bkey == mk ? bk : INT_MAX);
    const int b = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);  // NaN scores: keep the index in range
    const size_t gb = (size_t)(fr * P + p) * K;
    float *wc = kernarg_out()->weighted_c;
    float *pk3 = kernarg_out()->peak3;
    float *wcp = wc ? wc + (size_t)fr * kp.wc_CK + woff - wlo : nullptr;
#if F16_OUT16_LOOPS
    if constexpr (SPLIT) {
    // one loop per output kind under its (uniform) pointer test: inside one
    // loop, every lag re-derived each test's lane mask (VALU) and branched
    if (out.scores_f)
#pragma unroll
        for (int i = 0; i < KL; i++)
            if (r + 16 * i < K)
                out.scores_f[gb + r + 16 * i] = sv[i];
#if F16_OUT16_LOOPS == 2
    if (out.weighted_f) {
#else
    if (out.weighted_f || wcp) {
#endif
        float wv[KL];
#pragma unroll
        for (int i = 0; i < KL; i++) {
            const int k = r + 16 * i;
            wv[i] = k < K ? sv[i] * priorl[k > b ? k - b : b - k] : 0.0f;
        }
        if (out.weighted_f)
#pragma unroll
            for (int i = 0; i < KL; i++)
                if (r + 16 * i < K)
                    out.weighted_f[gb + r + 16 * i] = wv[i];
        if (wcp)
#pragma unroll
            for (int i = 0; i < KL; i++) {
                const int k = r + 16 * i;
                if (k < K && k >= wlo && k < wlo + ww)
                    wcp[k] = wv[i];
            }
    }
#if F16_OUT16_LOOPS == 2
    else if (wcp) {
        // the compact scratch alone (the bench path): each lag's prior read next
        // to its store, as in the one-loop form
#pragma unroll
        for (int i = 0; i < KL; i++) {
            const int k = r + 16 * i;
            if (k < K && k >= wlo && k < wlo + ww)
                wcp[k] = sv[i] * priorl[k > b ? k - b : b - k];
        }
    }
#endif
    if (pk3)
#pragma unroll
        for (int i = 0; i < KL; i++) {
            const int k = r + 16 * i;
            if (k < K && k >= b - 1 && k <= b + 1)
                pk3[(size_t)(fr * P + p) * 3 + 1 - b + k] = sv[i];
        }
    } else
#endif
    {
#pragma unroll
    for (int i = 0; i < KL; i++) {
        const int k = r + 16 * i;
        if (k < K) {
            const int dd = k > b ? k - b : b - k;
            const float wv = sv[i] * priorl[dd];
            if (out.scores_f)
                out.scores_f[gb + k] = sv[i];
            if (out.weighted_f)
                out.weighted_f[gb + k] = wv;
            if (wcp && k >= wlo && k < wlo + ww)
                wcp[k] = wv;
            if (pk3 && k >= b - 1 && k <= b + 1)
                pk3[(size_t)(fr * P + p) * 3 + 1 - b + k] = sv[i];
        }
    }
    }
    if (r == 0) {
#ifndef F16_RNG_DUMP  // (the dump build owns out.lags, see the frame loop's end)
        out.lags[fr * P + p] = b - S;
#endif
        lagl[p] = b - S;
    }
}

// ---- the grid solve fused into k_frame16 (FG; vga_heatmap.h:99-108, the
// exact branch and bound of tdoa_grid_bb.h spread over waves).  The last pair
// round leaves groups idle (config 4: pairs 24-27 on 4 of 8 groups; config 3:
// pairs 4-5 on 2 of 4); their NGW = 8 waves solve the PREVIOUS frame's grid
// between the round's barriers, from that frame's weighted scores kept in LDS
// in the compact layout (kp.wc_*), while the busy groups run the round's
// passes.  Segments (one per barrier interval of the round):
//   A  sparse-table levels S_lv[i] = max w[i .. i + 2^lv - 1], lv = 1..3, of the
//      compact array (lane: 8 elements from 15 reads), into the idle groups'
//      transform buffers; the entries' query rows (kp.fg_q) requested
//   B  every entry's bound: sum over pairs, in L's own pair order from 0, of
//      the range maximum max(S_lv[e], S_lv[e + d]) -- >= the float L of every
//      tuple of the entry (float addition is monotone in each operand)
//   C  wave gw takes the largest bound among the entries t = gw mod NGW (first
//      on ties, NaN never) and evaluates it: its <= 64 tuples, one per lane,
//      L = 0 + w_0[l_0] + w_1[l_1] + ... (the exhaustive scan's association),
//      (max L, smallest first-cell index) by a 64-bit key
//   D  the wave's key and candidate to LDS
//   E  best8 = the best of the NGW keys; each wave then evaluates, in entry
//      order, every entry of its partition other than its candidate whose
//      bound is not below the best so far (NaN bounds included) -- an entry
//      below it cannot hold the maximum -- and stores its key
// and after the round's closing barrier one lane takes the best of the NGW
// final keys: cell, max_Lf, (x, y) of k_grid_bb, bit for bit (ties: the
// smallest first-cell tuple; no L above -inf: tuple 0 and -inf).  The last
// frame of a workgroup is solved the same way after the frame loop.
constexpr int FG_NGW = 8;  // grid waves
struct FgLds {
    float *w;        // [2][CKp] compact weighted scores (DM 0: by frame parity; DM 1: [0] only)
    float *bnd;      // [256] entry bounds
    uint64_t *key;   // [NGW] seg C keys, then [NGW] seg E keys
    int *cand;       // [NGW] seg C candidates
};
__device__ __forceinline__ uint64_t fg_key(float L, int ui)
{
    if (!(L > -INFINITY))  // the exhaustive scan records only L above its start value
        return 0;
    return ((uint64_t)((uint32_t)fkey(L) ^ 0x80000000u) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)ui);
}
__device__ __forceinline__ float fg_key_value(uint64_t k)
{
    return k ? fkey_value((int)((uint32_t)(k >> 32) ^ 0x80000000u)) : -INFINITY;
}
__device__ __forceinline__ uint64_t fg_wave_max(uint64_t k) { return lane63_u64(wave_umax_dpp(k)); }

// kp's fields through an opaque kernarg pointer (kernarg_base): loaded where the
// segment uses them (scalar loads) instead of hoisted to the kernel's start and
// held in scalar registers across the frame loop (they spilled)
__device__ __forceinline__ const __attribute__((address_space(4))) tdoa_kparams *kernarg_kp()
{
    return reinterpret_cast<const __attribute__((address_space(4))) tdoa_kparams *>(kernarg_base());
}
template <int P>
struct FgGrid {
    FgLds L;
    float *lvl;  // [3][LV] levels (the idle groups' buffers), LV = CK rounded to 8
    int CK, CKp;
    __device__ __forceinline__ int LV() const { return (CK + 7) & ~7; }  // a lane writes 8 elements per level
    // seg A: levels of the compact array w; prefetch of the bound rows
    __device__ __forceinline__ void levels(const float *w, int gw, int lane, uint4 (&qr)[4]) const
    {
        const auto *kp = kernarg_kp();
        const int t = gw * 64 + lane;
        const uint4 *row = reinterpret_cast<const uint4 *>(kp->fg_q + (size_t)(t < kp->bb_NT ? t : 0) * 32);
#pragma unroll
        for (int i = 0; i < 4; i++)
            qr[i] = row[i];
        for (int i0 = 8 * t; i0 < CK; i0 += 8 * 64 * FG_NGW) {
            float x[15];
#pragma unroll
            for (int d = 0; d < 15; d++)
                x[d] = w[i0 + d < CK ? i0 + d : CK - 1];
#pragma unroll
            for (int d = 0; d < 14; d++)
                x[d] = fmaxf(x[d], x[d + 1]);
            float4 *d1 = reinterpret_cast<float4 *>(lvl + i0);
            d1[0] = make_float4(x[0], x[1], x[2], x[3]);
            d1[1] = make_float4(x[4], x[5], x[6], x[7]);
#pragma unroll
            for (int d = 0; d < 12; d++)
                x[d] = fmaxf(x[d], x[d + 2]);
            float4 *d2 = reinterpret_cast<float4 *>(lvl + LV() + i0);
            d2[0] = make_float4(x[0], x[1], x[2], x[3]);
            d2[1] = make_float4(x[4], x[5], x[6], x[7]);
#pragma unroll
            for (int d = 0; d < 8; d++)
                x[d] = fmaxf(x[d], x[d + 4]);
            float4 *d3 = reinterpret_cast<float4 *>(lvl + 2 * LV() + i0);
            d3[0] = make_float4(x[0], x[1], x[2], x[3]);
            d3[1] = make_float4(x[4], x[5], x[6], x[7]);
        }
    }
    // seg B: the bounds of entries gw * 64 + lane
    __device__ __forceinline__ void bounds(const float *w, int gw, int lane, const uint4 (&qr)[4]) const
    {
        const int t = gw * 64 + lane;
        if (t >= kernarg_kp()->bb_NT)
            return;
        uint32_t qw[16];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            qw[4 * i] = qr[i].x;
            qw[4 * i + 1] = qr[i].y;
            qw[4 * i + 2] = qr[i].z;
            qw[4 * i + 3] = qr[i].w;
        }
        float mp[P];
#pragma unroll
        for (int p = 0; p < P; p++) {
            const uint32_t q = (qw[p >> 1] >> (16 * (p & 1))) & 0xFFFFu;
            const int e = (int)(q & 2047u), lv = (int)((q >> 11) & 3u), dd = (int)(q >> 13);
            const float *base = lv ? lvl + (lv - 1) * LV() : w;
            mp[p] = fmaxf(base[e], base[e + dd]);
        }
        float b = 0.0f;
#pragma unroll
        for (int p = 0; p < P; p++)  // in L's own pair order, from 0
            b += mp[p];
        L.bnd[t] = b;
    }
    // one entry's tuples, one per lane: the wave's best key.  The tuples come as
    // compact element indices (kp.fg_tup: no per-pair offsets in scalar registers)
    __device__ __forceinline__ uint64_t evaluate(const float *w, int c, int lane) const
    {
        constexpr int NQ = (P + 7) / 8;  // 16-B loads of 8 indices
        const auto *kp = kernarg_kp();
        const int start = kp->bb_tile[2 * c], cnt = kp->bb_tile[2 * c + 1];
        uint64_t k = 0;
        if (lane < cnt) {
            const int u = start + lane;
            const uint4 *row = reinterpret_cast<const uint4 *>(kp->fg_tup + (size_t)u * 32);
            uint4 q[NQ];
#pragma unroll
            for (int i = 0; i < NQ; i++)
                q[i] = row[i];
            const int ui = kp->bb_uidx[u];
            float Lv = 0.0f;
#pragma unroll
            for (int p = 0; p < P; p++) {
                const uint4 &qq = q[p >> 3];
                const uint32_t wd = ((p >> 1) & 3) == 0 ? qq.x : (((p >> 1) & 3) == 1 ? qq.y : (((p >> 1) & 3) == 2 ? qq.z : qq.w));
                Lv += w[(wd >> (16 * (p & 1))) & 0xFFFFu];
            }
            k = fg_key(Lv, ui);
        }
        return fg_wave_max(k);
    }
    // seg C: the partition's best-bound entry, evaluated
    __device__ __forceinline__ uint64_t candidate(const float *w, int gw, int lane, int &cand) const
    {
        const int t = gw + FG_NGW * lane;
        uint64_t bk = 0;
        if (t < kernarg_kp()->bb_NT) {
            const float b = L.bnd[t];
            if (b == b)  // NaN bounds never seed (k_grid_bb)
                bk = ((uint64_t)((uint32_t)fkey(b) ^ 0x80000000u) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)t);
        }
        bk = fg_wave_max(bk);
        cand = bk ? (int)(0xFFFFFFFFu - (uint32_t)bk) : -1;
        return cand >= 0 ? evaluate(w, cand, lane) : 0;
    }
    // seg E: best8, then the partition's other entries not below the best
    __device__ __forceinline__ uint64_t rest(const float *w, int gw, int lane) const
    {
        uint64_t best = 0;
#pragma unroll
        for (int i = 0; i < FG_NGW; i++)
            best = L.key[i] > best ? L.key[i] : best;
        const int mine = L.cand[gw];
        const int t = gw + FG_NGW * lane;
        const float bl = fg_key_value(best);
        const bool need = t < kernarg_kp()->bb_NT && t != mine && !(L.bnd[t] < bl);
        uint64_t m = __ballot(need);
        while (m) {
            const int j = __builtin_ctzll(m);
            m &= m - 1;
            const int c = gw + FG_NGW * j;
            if (L.bnd[c] < fg_key_value(best))  // the best may have risen since
                continue;
            const uint64_t k = evaluate(w, c, lane);
            best = k > best ? k : best;
        }
        return best;
    }
    // after the closing barrier: the frame's outputs (one lane)
    __device__ __forceinline__ void finish(int64_t f) const
    {
        const auto *kp = kernarg_kp();
        const auto *out = kernarg_out();
        uint64_t best = 0;
#pragma unroll
        for (int i = 0; i < FG_NGW; i++)
            best = L.key[FG_NGW + i] > best ? L.key[FG_NGW + i] : best;
        int ui = best ? (int)(0xFFFFFFFFu - (uint32_t)best) : 0;
        ui = (ui < 0 || ui >= kp->U) ? 0 : ui;  // no L above -inf: tuple 0 (k_grid_bb)
        const int cell = kp->tuple_cell[ui];
        if (int32_t *oc = out->cell)
            oc[f] = cell;
        if (float *om = out->max_Lf)
            om[f] = fg_key_value(best);
        if (float *oxy = out->xy) {
            const int W = kp->grid_W, cx = cell % W, cy = cell / W;
            oxy[2 * f] = (float)(cx - kp->half_w) / kp->grid_scale;
            oxy[2 * f + 1] = (float)(kp->half_h - cy) / kp->grid_scale;
        }
    }
};

// (kp, out) must stay the first two parameters: kernarg_out() reads `out`
// at its kernarg offset
// DM (deferred outputs): 0 -- every round's pass 3 runs its pair's argmax and
// outputs (one wave per group, the workgroup waiting at the round's closing
// barrier); 1 -- pass 3 leaves the raw scores in LDS (scl, [P][K] floats) and
// one epilogue after the last round runs every pair's argmax and outputs, a
// wave per pair in parallel.  (Running the earlier rounds' epilogue on the
// last round's idle groups instead measured slower at config 3: 3.865 vs
// 3.826 ms per step.)
template <int C, int M, int DM, bool XS = (F16_XS != 0), bool FG = false>
__global__ void __launch_bounds__(1024, 1) k_frame16(tdoa_kparams kp, tdoa_kout out,
                                                     const int16_t *__restrict__ frames, int64_t B,
                                                     float e2)
{
    constexpr int T = C / 16, R1 = C / 256, G = 16384 / C, NS = C / 2048, BUF = f16_buf<C, XS>();
    static_assert(M >= 2 && M <= G, "one forward round: every mic has its own group");
    constexpr int P = M * (M - 1) / 2, ROUNDS = (P + G - 1) / G;
    constexpr int WPG = T / 64;  // waves per group (4 or 2)
    static_assert(WPG == 2 || WPG == 4, "group of 2 or 4 waves");
    static_assert(DM == 0 || DM == 1, "deferred-output mode");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f2 *bufs = (f2 *)smem;                    // [G][BUF]
    f2 *xhalf = bufs + G * BUF;               // [G] U_m[C / 2]
    int *red = (int *)(xhalf + G);            // [16] per-wave DC partial sums
    int *lagl = red + 16;                     // [TDOA_MAX_PAIRS]
    f2 *ttl = (f2 *)(lagl + TDOA_MAX_PAIRS);  // [3][16][16] the r16 twiddle tables
    float *priorl = (float *)(ttl + 3 * 16 * 16);  // [128] the lag prior (K <= 127)
    f2 *tw3 = (f2 *)(priorl + 128);  // [R1][64] pass-3 twiddles per lane (row 0 unused)
    uint32_t *winl = (uint32_t *)(tw3 + R1 * 64);  // f16_win_lds: [C / 2] window words
    float *scl = (float *)(winl + (f16_win_lds<C>() ? C / 2 : 0));  // DM 1: [P][K] raw scores of the frame
    // FG: the fused grid's LDS (FgLds) after scl, 16-B aligned; its levels in
    // the last round's idle groups' buffers
    constexpr int GI0 = P - (ROUNDS - 1) * G;  // first idle group of the last round
    static_assert(!FG || (G - GI0) * (T / 64) >= FG_NGW, "the last round must leave FG_NGW idle waves");
    const int CKp = (kp.wc_CK + 3) & ~3;
    FgLds fgl{};
    if constexpr (FG) {
        const int fo = (int)(((char *)(scl + (DM == 1 ? P * kp.K : 0)) - smem + 15) & ~15);
        fgl.w = (float *)(smem + fo);
        fgl.bnd = fgl.w + (DM == 0 ? 2 : 1) * CKp;  // DM 1: one buffer (written after the last round)
        fgl.key = (uint64_t *)(fgl.bnd + 256);
        fgl.cand = (int *)(fgl.key + 2 * FG_NGW);
    }
    const FgGrid<P> fgg{fgl, (float *)(bufs + GI0 * BUF), kp.wc_CK, CKp};
    int64_t prev = -1;  // FG: the previous frame of this workgroup (its grid is still to solve)
    int fpar = 0;       // FG, DM 0: this iteration's half of the double-buffered scores (by iteration, not
                        // frame parity: a workgroup's frames are gridDim.x apart)
    const int g = (int)threadIdx.x / T;
    const int K = kp.K, S = kp.S;
    f2 *buf = bufs + g * BUF;
    const uint32_t *win = reinterpret_cast<const uint32_t *>(kp.window);
    const f2 *tw2 = reinterpret_cast<const f2 *>(kp.tw2);
    // the twiddle tables in LDS (6 KiB): every pass reads them right after a
    // barrier, where a global (L2) round trip would stall the whole workgroup
    if (threadIdx.x < 3 * 16 * 16)  // 8-B units: kp.r16_tw is 8-B aligned
        ttl[threadIdx.x] = reinterpret_cast<const f2 *>(kp.r16_tw)[threadIdx.x];
    // the prior too: a pass-3 global read waits (vmcnt) for the next frame's
    // words, requested just before the pair rounds
    if (threadIdx.x < (unsigned)kp.K)
        priorl[threadIdx.x] = kp.prior[threadIdx.x];
    // (pass 3 multiplied two table entries per term before: 4.51 vs 4.26 ms per config-3 step)
    if (threadIdx.x < R1 * 64) {  // lane l: conj(W_C^{r l}) (l < 32), W_C^{r (64 - l)}
        const int r = threadIdx.x >> 6, l = threadIdx.x & 63;
        const f2 t = twC(reinterpret_cast<const f2 *>(kp.r16_tw), r, l < 32 ? l : 64 - l);
        tw3[threadIdx.x] = f2{t.x, l < 32 ? -t.y : t.y};
    }
#if F16_TW_REG
    // W_2C^b of this thread's split bins and W_2C^{C/2}: loaded once for the
    // launch (read per frame from L2, their latency opened every split)
    f2 twb[NS];
#pragma unroll
    for (int s2 = 0; s2 < NS; s2++)
        twb[s2] = tw2[(int)threadIdx.x + 1024 * s2];
    f2 twh = tw2[C / 2];
#endif
    uint32_t wr[8] = {};  // f16_win_mode 2: this thread's window words
    if constexpr (f16_win_mode<C>() == 2) {
        const int j0 = (int)threadIdx.x - g * T;
#pragma unroll
        for (int s2 = 0; s2 < 8; s2++)
            wr[s2] = win[j0 + T * s2];
    }
    if constexpr (f16_win_lds<C>()) {
        for (int i = threadIdx.x; i < C / 2; i += 1024)
            winl[i] = win[i];
        __syncthreads();  // the forward reads the window before its first barrier
    }
    const f2 *tt = ttl;  // visible after the first barrier (the DC sum's)
    const int mg = g < M ? g : 0;  // groups without a mic transform mic 0 (unused)
    const int P3W = (g / (4 / WPG)) % WPG;  // the group's pass-3 wave: SIMD (g WPG + P3W) mod 4
    // the compact-scratch ranges (kp.wc_lo / wc_w / wc_off) of every pair this
    // wave outputs, read once here: a kp byte indexed by a runtime pair is a
    // VMEM load whose vmcnt wait would also wait for the next frame's words.
    // rl_*[r]: round r's pair of the group (pass 3); ep_*: the epilogue's pairs
    int rl_lo[ROUNDS], rl_w[ROUNDS], rl_off[ROUNDS];
#pragma unroll
    for (int r = 0; r < ROUNDS; r++) {
        const int q = r * G + g < P ? r * G + g : 0;
        rl_lo[r] = __builtin_amdgcn_readfirstlane(kp.wc_lo[q]);
        rl_w[r] = __builtin_amdgcn_readfirstlane(kp.wc_w[q]);
        rl_off[r] = __builtin_amdgcn_readfirstlane(kp.wc_off[q]);
    }
    // DM 1 (frame16_out16): this lane's pair 4 w + (lane >> 4) and its compact range
    constexpr bool OUT16 = DM == 1 && !FG && F16_OUT16 != 0;
    // (one register: lo | w << 8 | off << 16; the lagged epilogue runs where the
    // forward's registers peak)
    uint32_t e16_rng = 0;
    if constexpr (OUT16) {
        const int e16_p = f16_epi_pair<P>((int)threadIdx.x);  // this lane's row's pair
        const int pq = e16_p < P ? e16_p : 0;
        // per-lane loads, waited for below.  Workaround for a codegen bug: picking
        // each row's range from the wave's four scalar loads (F16_RNG_SCALAR=1)
        // makes hipcc address wc_off[p] (u16, p = 4 w + 2) as SBASE = kernarg + p,
        // SOFFSET = p, and gfx950's scalar loads drop the base's low two address
        // bits: every wave's row 2 read the offset of its row 0 (round 5: cfg4
        // cells 72 % equal; root cause round 6, tools/probe/smem_sbase_align.hip,
        // tools/diag_rng.py; tests/test_code_objects.py flags the pattern)
#if F16_RNG_SCALAR
        // A/B for the ISA audit: the wave's four ranges as scalar loads, the
        // row's picked by a per-lane select
        (void)pq;
        const int w0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        uint32_t rq[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int p = 4 * w0 + q < P ? 4 * w0 + q : 0;
            rq[q] = (uint32_t)kp.wc_lo[p] | (uint32_t)kp.wc_w[p] << 8 | (uint32_t)kp.wc_off[p] << 16;
        }
        const int row = ((int)threadIdx.x >> 4) & 3;
#if F16_RNG_SCALAR == 2
        // branch-free: the four ranges forced into SGPRs, a v_cndmask chain
#pragma unroll
        for (int q = 0; q < 4; q++)
            rq[q] = __builtin_amdgcn_readfirstlane(rq[q]);
        e16_rng = rq[0];
        e16_rng = row == 1 ? rq[1] : e16_rng;
        e16_rng = row == 2 ? rq[2] : e16_rng;
        e16_rng = row == 3 ? rq[3] : e16_rng;
#else
        e16_rng = row == 0 ? rq[0] : (row == 1 ? rq[1] : (row == 2 ? rq[2] : rq[3]));
#endif
#else
        const auto *kk = kernarg_kp();
        e16_rng = (uint32_t)kk->wc_lo[pq] | (uint32_t)kk->wc_w[pq] << 8 | (uint32_t)kk->wc_off[pq] << 16;
#endif
        asm volatile("" : "+v"(e16_rng));
    }
    // DM 1 (four-pairs epilogue), lagged (F16_EPI_LAG): frame f's outputs run in
    // frame f + 1's forward, after its pass-3 stores; its gate after that forward
    constexpr bool ELAG = OUT16 && F16_EPI_LAG != 0;
    // the waves (four pairs each) whose outputs run after the forward's pass-2
    // stores; the rest after its pass-3 stores (F16_EPI_SPLIT: -1 half, else count)
    constexpr int EPW = f16_epi_waves<P>(), EPS = F16_EPI_SPLIT < 0 ? EPW / 2 : (F16_EPI_SPLIT < EPW ? F16_EPI_SPLIT : EPW);
    auto epi16 = [&](int64_t f, int ps) F16_AI {
        const int t = opaque_idx((int)threadIdx.x);
        const int wv = __builtin_amdgcn_readfirstlane(t >> 6), pe = f16_epi_pair<P>(t);
        const bool mine = ps == 0 || (ps == 2 ? wv < EPS : wv >= EPS);
        if (!F16_NO_OUT && mine && wv < f16_epi_waves<P>() && pe < P) {
            const int r = t & 15, lo = (int)(e16_rng & 0xFFu), wd = (int)((e16_rng >> 8) & 0xFFu),
                      of = (int)(e16_rng >> 16);
            constexpr bool SPL = F16_OUT16_LOOPS != 0;
            if (kp.K <= 96)
                frame16_out16<6, SPL>(kp, out, scl, priorl, lagl, f, P, pe, r, lo, wd, of);
            else
                frame16_out16<8, SPL>(kp, out, scl, priorl, lagl, f, P, pe, r, lo, wd, of);
        }
    };
    auto gate_of = [&](int64_t f) F16_AI {
        // P > 16: wave 0's lanes one lag each, a DPP sum -- thread 0 alone read
        // and summed config 4's 28 lags one after another (83.2 vs 84.0 ms per
        // step, same box; at config 3's 6 lags the DPP sum cost more: 3.300 vs
        // 3.273 ms)
        if (F16_GATEW && P > 16 && threadIdx.x < 64 && out.gate) {
            const int ln = (int)threadIdx.x;
            int tot = 0;
            for (int q = ln; q < P; q += 64)
                tot += lagl[q] * lagl[q];
            tot = group_sum_dpp(tot, 64);
            if (ln == 63)
                out.gate[f] = tot > 4 ? 1 : 0;  // sample_compute.h:124-134
        } else if ((!F16_GATEW || P <= 16) && threadIdx.x == 0 && out.gate) {
            int tot = 0;
            for (int q = 0; q < P; q++)
                tot += lagl[q] * lagl[q];
            out.gate[f] = tot > 4 ? 1 : 0;
        }
    };
    // DM 1: the epilogue's pairs w, w + 16
    int ep_lo[2] = {0, 0}, ep_w[2] = {0, 0}, ep_off[2] = {0, 0};
    if constexpr (DM == 1 && !OUT16) {
        const int w0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int q = w0 + 16 * h < P ? w0 + 16 * h : 0;
            ep_lo[h] = __builtin_amdgcn_readfirstlane(kp.wc_lo[q]);
            ep_w[h] = __builtin_amdgcn_readfirstlane(kp.wc_w[q]);
            ep_off[h] = __builtin_amdgcn_readfirstlane(kp.wc_off[q]);
        }
    }
#ifdef TDOA_DIAG
    constexpr int NSTAMP = 48;  // k_frame16: up to 45 phase marks (config 4: 33)
    unsigned long long stamp[NSTAMP] = {};
    unsigned long long arrive[NSTAMP] = {};
    int nst = 0, nar = 0;
    const int64_t diag_fr = blockIdx.x + (B >= (int64_t)(F16_DIAG_FRAME + 1) * gridDim.x ? F16_DIAG_FRAME : 0) *
                                             (int64_t)gridDim.x;
#else
    constexpr int64_t diag_fr = -1;
#endif
    // persistent over frames (one workgroup per CU): the next frame's words are
    // requested when the pair rounds start, so their HBM latency hides behind
    // them instead of opening every frame
    uint32_t w[8];
    auto fetch = [&](int64_t f) {
        const uint32_t *x = reinterpret_cast<const uint32_t *>(frames + (f * M + mg) * (int64_t)C) +
                            ((int)threadIdx.x - g * T);
#pragma unroll
        for (int s = 0; s < 8; s++)
            w[s] = __builtin_nontemporal_load(x + T * s);
    };
    fetch(blockIdx.x);
    // the next frame's words are waited for here, before this wave's output
    // stores: gfx9's vmcnt counts stores and retires in order, and with stores
    // in branches the loop head's wait for the words was vmcnt(0) -- it also
    // waited for the frame's last stores to be acknowledged (F16_PIN=0: off)
    auto pin_words = [&] {
#if F16_PIN
#pragma unroll
        for (int s = 0; s < 8; s++)
            asm volatile("" : "+v"(w[s]));
#endif
    };
#if F16_PIN
    // and every value loaded before the loop is waited for before it: a load
    // still pending on the loop's entry edge put a vmcnt(0) at the loop head,
    // which on the back edge waited for the stores
    pin_words();
#pragma unroll
    for (int s = 0; s < 8; s++)
        asm volatile("" : "+v"(wr[s]));
#if F16_TW_REG
#pragma unroll
    for (int s = 0; s < NS; s++)
        asm volatile("" : "+v"(twb[s].x), "+v"(twb[s].y));
    asm volatile("" : "+v"(twh.x), "+v"(twh.y));
#endif
#endif
    for (int64_t fr = blockIdx.x; fr < B; fr += gridDim.x) {
    // thread indices the compiler cannot prove loop-invariant: the passes'
    // twiddle reads stay in the body instead of being hoisted (and spilled)
    const int tid = opaque_idx((int)threadIdx.x), j = tid - g * T, pj = pidx(j);
    // FG: this frame's compact scores go to fgw, the previous frame's are at pgw
    float *fgw = FG ? fgl.w + (DM == 0 ? fpar * CKp : 0) : nullptr;
    const float *pgw = FG ? fgl.w + (DM == 0 ? (fpar ^ 1) * CKp : 0) : nullptr;
    const bool fgr = FG && prev >= 0 && kp.fg_ok == 1;  // (fg_ok 2: TDOA_F16_FG=skip, A/B of the bare structure)
    if (fr == diag_fr) {
#ifdef TDOA_DIAG
        stamp[NSTAMP - 2] = __builtin_amdgcn_s_memrealtime();
#endif
        F16_MARK();
    }

    // ---- 1. forward transform of mic g (k_spec16's passes in slot g)
    auto fwd_mark = [&] {
        if (fr == diag_fr)
            F16_MARK();  // the forward's barriers (diagnostic build)
    };
    auto fwd_pre = [&] {
        if (fr == diag_fr)
            F16_PRE();  // ... and the waves' arrivals at them
    };
    if constexpr (ELAG) {
        auto lag_hook = [&](int ps) F16_AI {
            if (prev >= 0)
                epi16(prev, ps);  // the previous frame's outputs (scl holds its scores until round 0's pass 3)
        };
        frame16_forward<C, f16_win_mode<C>(), decltype(fwd_mark), XS, decltype(lag_hook), decltype(fwd_pre)>(
            w, f16_win_lds<C>() ? winl : win, wr, buf, red, tt, tid, g, j, pj, kp.log2N, fwd_mark, lag_hook, fwd_pre);
        if (prev >= 0)
            gate_of(prev);  // its lags are in lagl since the forward's closing barrier
    } else {
        frame16_forward<C, f16_win_mode<C>(), decltype(fwd_mark), XS, NoHook16, decltype(fwd_pre)>(
            w, f16_win_lds<C>() ? winl : win, wr, buf, red, tt, tid, g, j, pj, kp.log2N, fwd_mark, NoHook16(), fwd_pre);
    }
    if (fr == diag_fr)
        F16_MARK();  // forward transforms done
    // split + unit normalisation of every mic at this thread's bin pairs:
    // X[b] = (Z[b] + Z*[C-b]) - i W_2C^b (Z[b] - Z*[C-b]), X[C-b] = conj(e + i W od)
    // (b = 0: its partner output is X[C])
    // W_2C^b of this thread's bins (the split and every pair's pre-twiddle), W_2C^{C/2}
    // (requested before the forward's last pass instead, they measured slower:
    // 4.89 vs 4.71 ms per config-3 step)
#if !F16_TW_REG
    f2 twb[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
        twb[s] = tw2[tid + 1024 * s];
    const f2 twh = tw2[C / 2];
#endif
    f2 Ub[M][NS], Un[M][NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int b = tid + 1024 * s;
        const int pb = lidx<XS>(b), pp = lidx<XS>((C - b) & (C - 1));
        const f2 wb = twb[s];
#pragma unroll
        for (int m = 0; m < M; m++) {
            const f2 *zb = bufs + m * BUF;
            const f2 z = F16_LD(zb + pb), zp = F16_LD(zb + pp);
            const f2 e = c_addconj(z, zp);
            const f2 od = c_mul(c_subconj(z, zp), wb);
            Ub[m][s] = c_unit(c_add_mi(e, od), e2);
            Un[m][s] = c_unit(c_conj_add_i(e, od), e2);
        }
    }
    if constexpr (F16_PRIO != 0)
        f16_prio<2>();  // split done (F16_PRIO checkpoint)
    if (tid < M) {  // X[C/2] = conj(Z[C/2]) (x2): self-paired bin
        const f2 zh = bufs[tid * BUF + lidx<XS>(C / 2)];
        xhalf[tid] = c_unit(f2{2.0f * zh.x, -2.0f * zh.y}, e2);
    }
    // No barrier before the first round's Y stores (F16_SPLIT_BAR=0): a thread
    // stores Y only at the positions it has just read (bins b and C - b of every
    // slot), and position C / 2 -- read for X[C/2] by threads 0 .. M - 1, stored
    // by thread 0 -- stays inside wave 0, whose LDS operations are in order
#if F16_SPLIT_BAR
    if (fr == diag_fr)
        F16_PRE();
    __syncthreads();  // slots consumed: they become the pairs' buffers
    f16_prio<3>();
#endif
    if (fr == diag_fr)
        F16_MARK();  // unit spectra in registers
    {
        const int64_t fn = fr + gridDim.x;
        fetch(fn < B ? fn : fr);  // the next frame's words (or a harmless re-read)
    }

    // ---- 2. pairs, G per round (rounds and pair slots unrolled: every
    // register index below is a compile-time constant)
    const float invL = 1.0f / (float)(2 * C);
    static_for<0, ROUNDS>([&](auto rc) {
        constexpr int p0 = decltype(rc)::value * G;
        const int tl = opaque_idx(tid), jl = tl - g * T, pjl = pidx(jl);
        const ColIdx<C, XS> cjl(jl);
        // this thread's Y slots b = tl + 1024 s and C - b (b = 0: C / 2, whose
        // value thread 0 writes after, in program order)
        int yb0[NS], yb1[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int b = tl + 1024 * s;
            yb0[s] = lidx<XS>(b);
            yb1[s] = b == 0 ? lidx<XS>(C / 2) : lidx<XS>(C - b);
        }
        // packed inverse input Y of pair p0 + gg into buffer gg (all threads)
        static_for<0, G>([&](auto gc) {
            constexpr int pc = p0 + decltype(gc)::value;
            if constexpr (F16_PRIO != 0 && decltype(gc)::value == G / 2)
                f16_prio<1>();
            if constexpr (pc < P) {
                constexpr int pi = pair_first<M>(pc), pj = pair_second<M>(pc);
                f2 *yb = bufs + decltype(gc)::value * BUF;
#pragma unroll
                for (int s = 0; s < NS; s++) {
                    const f2 Rk = c_conjmul(Ub[pi][s], Ub[pj][s]);  // R[b]
                    const f2 Rq = c_conjmul(Un[pi][s], Un[pj][s]);  // R[C-b]
                    const f2 ss = c_addconj(Rk, Rq);
                    const f2 qq = c_mulconj(c_subconj(Rk, Rq), twb[s]);
                    yb[yb0[s]] = c_add_i(ss, qq);
                    yb[yb1[s]] = c_conj_add_mi(ss, qq);
                }
                if (!F16_YHALF && tl == 0) {  // Y[C/2] from R[C/2] alone
                    const f2 Rh = c_conjmul(xhalf[pi], xhalf[pj]);
                    yb[lidx<XS>(C / 2)] = c_add_i(c_addconj(Rh, Rh), c_mulconj(c_subconj(Rh, Rh), twh));
                }
            }
        });
#if F16_YHALF
        // Y[C/2] of the round's pairs, lane gg of wave 0 for pair p0 + gg: one
        // branch instead of one per pair on thread 0 (wave 0 ran ~1.1 k cycles
        // longer than its SIMD's other waves in every Y interval).  Wave 0 as
        // before: its LDS operations are in order -- X[C/2] (xhalf) was written by
        // its threads 0 .. M - 1 after they read Z[C/2] at the positions
        // written here, and thread 0's stores above put the partner value there first
        if (tl < G && p0 + tl < P) {
            const int pc = p0 + tl;
            int pi = 0, q = pc;
            while (q >= M - 1 - pi) {  // pair_first / pair_second at run time
                q -= M - 1 - pi;
                pi++;
            }
            const f2 Rh = c_conjmul(xhalf[pi], xhalf[pi + 1 + q]);
            bufs[tl * BUF + lidx<XS>(C / 2)] = c_add_i(c_addconj(Rh, Rh), c_mulconj(c_subconj(Rh, Rh), twh));
        }
#endif
        if (fr == diag_fr)
            F16_PRE();
        __syncthreads();
        f16_prio<3>();
        if (fr == diag_fr)
            F16_MARK();  // the round's Y buffers written
        const int p = p0 + g;
        const bool pair_on = p < P;
        // inverse pass 1 (radix 16, Ns = 1)
        // a partial last round (P mod G pairs): the idle groups skip the
        // transforms, leaving their SIMDs' issue slots to the busy groups
        const bool on = p0 + G <= P || pair_on;
        f2 v[16];
        if (on) {
#pragma unroll
            for (int r = 0; r < 16; r++)
                v[r] = F16_LD(buf + (XS ? cjl.at(r) : pjl + po(T * r)));
            dftp<16, true, false, F16_PRIO>(v);
        }
        // FG, last round: the idle groups' waves solve the previous frame's grid
        constexpr bool FGL = FG && decltype(rc)::value == ROUNDS - 1;
        const int gw = (tl - GI0 * T) >> 6, gln = tl & 63;
        uint4 fqr[4];
        if constexpr (FGL) {
            if (!on && fgr)
                fgg.levels(pgw, gw, gln, fqr);  // seg A
        }
        if (fr == diag_fr)
            F16_PRE();
        __syncthreads();
        f16_prio<3>();
        if (fr == diag_fr)
            F16_MARK();
        if (on) {
            const int b1 = 16 * jl | (jl & 15);  // xs(16 jl + r) = b1 ^ r
#pragma unroll
            for (int r = 0; r < 16; r++)
                buf[XS ? (b1 ^ r) : 17 * jl + r] = v[brev<16>(r)];
        }
        if constexpr (FGL) {
            if (!on && fgr)
                fgg.bounds(pgw, gw, gln, fqr);  // seg B
        }
        if (fr == diag_fr)
            F16_PRE();
        __syncthreads();
        f16_prio<3>();
        if (fr == diag_fr)
            F16_MARK();
        // pass 2: outputs r'' in {0, 1, 14, 15} only
        const int k = jl & 15;
        f2 x0 = f2{0, 0}, x1 = f2{0, 0}, x14 = f2{0, 0}, x15 = f2{0, 0};
#define F16_TW256(r) F16_LD(tt + 16 * (r) + k)
        if (on)
#pragma unroll
        for (int r = 0; r < 4; r++) {  // inputs r, r + 4, r + 8, r + 12 at a time
            if (r == 2)
                f16_prio<1>();
            f2 l0 = F16_LD(buf + (XS ? cjl.at(r) : pjl + po(T * r)));
            f2 l1 = F16_LD(buf + (XS ? cjl.at(r + 4) : pjl + po(T * (r + 4))));
            const f2 h0 = c_mulconj(F16_LD(buf + (XS ? cjl.at(r + 8) : pjl + po(T * (r + 8)))), F16_TW256(r + 8));
            const f2 h1 = c_mulconj(F16_LD(buf + (XS ? cjl.at(r + 12) : pjl + po(T * (r + 12)))), F16_TW256(r + 12));
            if (r)
                l0 = c_mulconj(l0, F16_TW256(r));  // tw256
            l1 = c_mulconj(l1, F16_TW256(r + 4));
            const f2 a0 = l0 + h0, a1 = l1 + h1;
            const f2 d0 = dif_tw<true>(l0, h0, 2 * r), d1 = dif_tw<true>(l1, h1, 2 * (r + 4));
            x0 = x0 + (a0 + a1);
            x1 = x1 + (d0 + d1);
            x14 = x14 + (r ? dif_tw<false>(a0, a1, 4 * r) : a0 - a1);
            x15 = x15 + (r ? dif_tw<false>(d0, d1, 4 * r) : d0 - d1);
        }
#undef F16_TW256
        uint64_t fgk = 0;
        int fgc = -1;
        if constexpr (FGL) {
            if (!on && fgr)
                fgk = fgg.candidate(pgw, gw, gln, fgc);  // seg C
        }
        // XS: the four outputs go to this thread's own column rows 0-3 (element
        // jl + T c for output c), positions no other thread reads in this pass:
        // no barrier between the pass's reads and its stores.  Padded layout:
        // element 64 a + 16 c + k (a = jl >> 4), after a barrier
        if constexpr (!XS) {
            if (fr == diag_fr)
                F16_PRE();
            __syncthreads();
            f16_prio<3>();
        }
        if (fr == diag_fr)
            F16_MARK();
        if (on) {
            if constexpr (XS) {
                buf[cjl.at(0)] = x0;
                buf[cjl.at(1)] = x1;
                buf[cjl.at(2)] = x14;
                buf[cjl.at(3)] = x15;
            } else {
                const int o = pidx((jl >> 4) * 64 + k);
                buf[o] = x0;
                buf[o + 17] = x1;
                buf[o + 34] = x14;
                buf[o + 51] = x15;
            }
        }
        if constexpr (FGL) {
            if (!on && fgr && gln == 0) {  // seg D
                fgl.key[gw] = fgk;
                fgl.cand[gw] = fgc;
            }
        }
        if (fr == diag_fr)
            F16_PRE();
        __syncthreads();
        f16_prio<3>();
        if (fr == diag_fr)
            F16_MARK();
        // pass 3 by one wave of the group, one output per column.  Waves of a
        // workgroup go to SIMD (wave index mod 4): the group's wave P3W lands
        // the G pass-3 waves evenly on the four SIMDs (the group's first wave
        // put them all on SIMD 0, or 0 and 2, one after another)
        if constexpr (DM == 0 && decltype(rc)::value == 0)
            pin_words();  // every wave, before the first round's output stores
        if ((jl >> 6) == P3W && pair_on) {
            const int l = jl & 63;
            const int mm = 64 - l;
            // column 192 + l (l >= 32): W_C^{-r (192 + l)} term == W_C^{r (64 - l)} after
            // the output index C - m; tw3 holds each lane's factors (conjugated for l < 32)
            // term r of lane l = 16 c + k: output c of pass-2 thread 16 r + k.  XS:
            // element 16 r + k + T c, xs = (T c + 16 r) | (k ^ ((r + (T / 16) c) & 15));
            // padded: element l + 64 r, pidx = pidx(l) + 68 r
            const int pl = lidx<XS>(l);
            const int c3 = l >> 4, k3 = l & 15;
            auto p3pos = [&](int r) {
                return XS ? ((T * c3 + 16 * r) | (k3 ^ ((r + (T / 16) * c3) & 15))) : pl + 68 * r;
            };
            // the R1 terms summed as a tree (a running sum was a dependent
            // chain of R1 - 1 complex products and adds on the round's critical path)
            f2 t[R1];
            t[0] = F16_LD(buf + p3pos(0));
#pragma unroll
            for (int r = 1; r < R1; r++)
                t[r] = c_mul(F16_LD(buf + p3pos(r)), F16_LD(tw3 + 64 * r + l));
#pragma unroll
            for (int h = R1 / 2; h >= 1; h >>= 1)
#pragma unroll
                for (int r = 0; r < h; r++)
                    t[r] = t[r] + t[r + h];
            const f2 y = t[0];
            const int n = l < 32 ? l : -mm;
            const int ka = 2 * n + S, kb = 2 * n + 1 + S;
            const bool oka = ka >= 0 && ka < K, okb = kb >= 0 && kb < K;
            const float sa = y.x * invL, sb = y.y * invL;
            constexpr int RI = decltype(rc)::value;
            if constexpr (DM == 1) {
                if (oka)
                    scl[p * K + ka] = sa;
                if (okb)
                    scl[p * K + kb] = sb;
            } else {
                const int pp[1] = {p}, lo[1] = {rl_lo[RI]}, wd[1] = {rl_w[RI]}, of[1] = {rl_off[RI]};
                const bool on1[1] = {true};
                const float a1[1] = {sa}, b1[1] = {sb};
                if (!F16_NO_OUT)
                frame16_pair_out<1>(kp, out, priorl, lagl, fr, P, pp, on1, ka, kb, oka, okb, a1, b1, l == 0, lo, wd,
                                    of, fgw);
            }
        }
        if constexpr (FGL) {
            if (!on && fgr) {  // seg E
                const uint64_t kk = fgg.rest(pgw, gw, gln);
                if (gln == 0)
                    fgl.key[FG_NGW + gw] = kk;
            }
        }
        if (fr == diag_fr)
            F16_PRE();
        __syncthreads();  // the buffers are rewritten by the next round
        f16_prio<3>();
        if (fr == diag_fr)
            F16_MARK();
    });
    if constexpr (FG) {
        if (fgr && tid == 0)
            fgg.finish(prev);  // the previous frame's cell, max L, (x, y)
    }
    if constexpr (DM == 1) {
        // every pair's argmax and outputs, wave w: pairs w, w + 16 (lane l:
        // lags l and l + 64, K <= 127)
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), ln = tid & 63;
        static_assert(P <= 32, "two epilogue pairs per wave at most");
        if constexpr (OUT16) {
            // waves 0 .. ceil(P / 4) - 1, four pairs each (rows past P idle);
            // ELAG: in the next frame's forward (or after the loop) instead
            if constexpr (!ELAG) {
                pin_words();
                epi16(fr, 0);
            }
        } else {
        const bool oka = ln < K, okb = ln + 64 < K;
        const int pp[2] = {wv, wv + 16 < P ? wv + 16 : wv};
        const bool on2[2] = {wv < P, wv + 16 < P};
        float sa[2], sb[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            sa[h] = oka ? scl[pp[h] * K + ln] : 0.0f;
            sb[h] = okb ? scl[pp[h] * K + ln + 64] : 0.0f;
        }
        pin_words();
        if (on2[0])
            frame16_pair_out<2>(kp, out, priorl, lagl, fr, P, pp, on2, ln, ln + 64, oka, okb, sa, sb, ln == 0, ep_lo,
                                ep_w, ep_off, fgw);
        }
        if constexpr (!ELAG) {
            if (fr == diag_fr)
                F16_PRE();
            __syncthreads();  // lagl complete for the gate; scl free for the next frame
            f16_prio<3>();
            if (fr == diag_fr)
                F16_MARK();
        }
    }
    pin_words();
    if constexpr (!ELAG)
        gate_of(fr);
    prev = fr;
    fpar ^= 1;
#ifdef TDOA_DIAG
    if (fr == diag_fr) {
        stamp[NSTAMP - 1] = __builtin_amdgcn_s_memrealtime();
        stamp[NSTAMP - 3] = __builtin_amdgcn_s_memtime();
    }
#endif
    }  // frames
    if constexpr (ELAG) {
        // the last frame's outputs (its last round closed with a barrier: scl complete)
        if (prev >= 0) {
            epi16(prev, 0);
            __syncthreads();
            gate_of(prev);
        }
#ifdef F16_RNG_DUMP
        // diagnostic builds only: every thread's packed compact range over the
        // first 1024 lag slots (tools/diag_rng.py)
        __syncthreads();
        if (blockIdx.x == 0)
            out.lags[threadIdx.x] = (int32_t)e16_rng;
#endif
    }
    if constexpr (FG) {
        // the last frame's grid, by waves 0 .. FG_NGW - 1 (every buffer is free)
        if (prev >= 0 && kp.fg_ok == 1) {
            const int tid = (int)threadIdx.x, gw = tid >> 6, gln = tid & 63;
            const bool act = gw < FG_NGW;
            const float *pgw = fgl.w + (DM == 0 ? (fpar ^ 1) * CKp : 0);  // (fpar toggled after the last frame)
            uint4 fqr[4];
            __syncthreads();  // the last frame's scores are in LDS
            if (act)
                fgg.levels(pgw, gw, gln, fqr);
            __syncthreads();
            if (act)
                fgg.bounds(pgw, gw, gln, fqr);
            __syncthreads();
            int fgc = -1;
            uint64_t fgk = 0;
            if (act)
                fgk = fgg.candidate(pgw, gw, gln, fgc);
            if (act && gln == 0) {
                fgl.key[gw] = fgk;
                fgl.cand[gw] = fgc;
            }
            __syncthreads();
            if (act) {
                const uint64_t kk = fgg.rest(pgw, gw, gln);
                if (gln == 0)
                    fgl.key[FG_NGW + gw] = kk;
            }
            __syncthreads();
            if (tid == 0)
                fgg.finish(prev);
        }
    }
#ifdef TDOA_DIAG
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 64)
        for (int i = 0; i < NSTAMP; i++) {
            g_diag_f16[(blockIdx.x * 16 + (threadIdx.x >> 6)) * NSTAMP + i] = stamp[i];
            g_diag_f16b[(blockIdx.x * 16 + (threadIdx.x >> 6)) * NSTAMP + i] = arrive[i];
        }
#endif
}
#undef F16_MARK

// the fused grid (FG) applies: the last pair round leaves FG_NGW idle waves,
// the tables exist, TDOA_F16_FG is not "0", and the LDS fits (with the
// deferred scores where the launch defers)
template <int C, int M>
constexpr bool fg_shape()
{
    constexpr int G = 16384 / C, P = M * (M - 1) / 2, ROUNDS = (P + G - 1) / G, GI0 = P - (ROUNDS - 1) * G;
    return (G - GI0) * (C / 16 / 64) >= FG_NGW;
}
// TDOA_F16_FG: 1 on, skip (A/B of the bare FG structure); unset or 0: off.
// Measured slower at both shapes it applies to (same box, ms per step):
// config 3 4.04 vs 3.50, config 4 100.9 vs 93.0 (k_frame16 + k_grid_bb) -- the
// last round's idle waves hold one frame's dependent search chain (bounds, then
// entry evaluations on L2 tuple rows) and it outlasts the round; k_grid_bb
// hides the same chains behind other frames' (DESIGN.md "Fused grid")
static int fg_mode()
{
    static const int m = [] {
        const char *e = getenv("TDOA_F16_FG");
        if (!e)
            return -1;
        return !strcmp(e, "1") ? 1 : (!strcmp(e, "skip") ? 2 : 0);
    }();
    return m;
}
static size_t fg_lds_bytes(const tdoa_kparams &kp, bool defer)
{
    // DM 0 double-buffers the compact scores by iteration; DM 1 writes them in
    // the epilogue, after the last round that reads the previous frame's
    const size_t CKp = (size_t)((kp.wc_CK + 3) & ~3);
    return 16 + (defer ? 1 : 2) * CKp * 4 + 256 * 4 + 2 * FG_NGW * 8 + FG_NGW * 4;
}
template <int C, int M>
static bool frame16_defer(const tdoa_kparams &kp)
{
    // deferred pair outputs (DM 1) at two or more pair rounds when the frame's
    // [P][K] scores fit next to the buffers: with the lagged four-pairs epilogue
    // config 3 3.48 vs 3.50 ms per step, config 4 90.1 vs 95.0 (round 5; with
    // the round-4 epilogue config 3 had measured 3.87 vs 3.83, in-round faster)
    constexpr int P = M * (M - 1) / 2, G = 16384 / C, ROUNDS = (P + G - 1) / G;
    // TDOA_F16_DEFER=0 / 1 forces a mode
    static const int force = [] {
        const char *e = getenv("TDOA_F16_DEFER");
        return e ? atoi(e) : -1;
    }();
    const size_t lds_defer = frame16_lds_base<C>() + (size_t)P * kp.K * sizeof(float);
    constexpr int MIN_ROUNDS = (F16_OUT16 && F16_EPI_LAG) ? 2 : 3;
    return (force >= 0 ? force == 1 : ROUNDS >= MIN_ROUNDS) && lds_defer <= 160 * 1024;
}
template <int C, int M>
static bool frame16_fg(const tdoa_kparams &kp)
{
#if !TDOA_AB
    return false;  // the fused grid is an A/B path (tools libraries only)
#endif
    if (!fg_shape<C, M>() || !kp.fg_ok || !kp.fg_q || !kp.fg_tup || fg_mode() == 0 || kp.P != M * (M - 1) / 2)
        return false;
    const bool defer = frame16_defer<C, M>(kp);
    if (fg_mode() < 0)
        return false;
    const size_t base = frame16_lds_base<C>() + (defer ? (size_t)kp.P * kp.K * sizeof(float) : 0);
    return base + fg_lds_bytes(kp, defer) <= 160 * 1024;
}

template <int C, int M>
int launch_frame16(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
                   float e2, hipStream_t st)
{
    if (B <= 0)
        return 0;
    constexpr int P = M * (M - 1) / 2;
    const bool defer = frame16_defer<C, M>(kp);
    // the grid solved in the kernel when the caller asks for it (FG)
    const bool fg = frame16_fg<C, M>(kp) && (out.cell || out.xy || out.max_Lf);
    const void *fn;
#if TDOA_AB
    if constexpr (fg_shape<C, M>())
        fn = defer ? (fg ? (const void *)k_frame16<C, M, 1, F16_XS != 0, true> : (const void *)k_frame16<C, M, 1>)
                   : (fg ? (const void *)k_frame16<C, M, 0, F16_XS != 0, true> : (const void *)k_frame16<C, M, 0>);
    else
        fn = defer ? (const void *)k_frame16<C, M, 1> : (const void *)k_frame16<C, M, 0>;
#else
    fn = defer ? (const void *)k_frame16<C, M, 1> : (const void *)k_frame16<C, M, 0>;
#endif
    const size_t lds =
        (defer ? frame16_lds_base<C>() + (size_t)P * kp.K * sizeof(float) : frame16_lds_base<C>()) +
        (fg ? fg_lds_bytes(kp, defer) : 0);
    tdoa_kparams kpl = kp;
    if (fg && fg_mode() == 2)
        kpl.fg_ok = 2;  // A/B only: the FG kernel without its grid work (no grid outputs)
    const int res = tdoa_resident_blocks(fn, 1024, lds);
    if (res < 1)
        return tdoa_set_error(-2, "k_frame16: no resident workgroup (LDS / registers)");
    const int64_t grid = B < (int64_t)res ? B : (int64_t)res;
#if TDOA_AB
    if constexpr (fg_shape<C, M>()) {
        if (fg) {
            if (defer)
                hipLaunchKernelGGL((k_frame16<C, M, 1, F16_XS != 0, true>), dim3((unsigned)grid), dim3(1024), lds, st,
                                   kpl, out, frames, B, e2);
            else
                hipLaunchKernelGGL((k_frame16<C, M, 0, F16_XS != 0, true>), dim3((unsigned)grid), dim3(1024), lds, st,
                                   kpl, out, frames, B, e2);
        }
    }
#endif
    if (!fg) {
        if (defer)
            hipLaunchKernelGGL((k_frame16<C, M, 1>), dim3((unsigned)grid), dim3(1024), lds, st, kp, out, frames, B, e2);
        else
            hipLaunchKernelGGL((k_frame16<C, M, 0>), dim3((unsigned)grid), dim3(1024), lds, st, kp, out, frames, B, e2);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof msg, "k_frame16 launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, msg);
    }
    return 0;
}


#if TDOA_AB  // the A/B kernel k_frame16w: built into tools libraries only (Makefile "ab")
// ------------------------------------------------ fused, one wave per pair
// k_frame16w<2048, 8> (BASELINE config 4).  k_frame16's forward transforms,
// then the split writes the unit spectra U_m[0..C] back into the mics' LDS
// slots, and every wave runs whole pairs from there on its own: no workgroup
// barrier between the spectra and the frame's end (k_frame16 spends five per
// round of 8 pairs, and writes every pair's inverse input and first pass
// through LDS).  For pair (i, j), lane l of the wave:
//   * Y[b], b = l + 64 q (q < 32): k_pair16's pre-twiddle from U_i, U_j at b
//     and C - b, R = conj(U_i) U_j, with conj(W_2C^b) = conj(W_2C^l) conj(W_64^q)
//     (a lane constant, then a compile-time one);
//   * A_l[k] = sum_q Y[l + 64 q] W_32^{-q k}: a register DFT-32 (fft32d);
//   * y[n] = sum_l W_C^{-l n} A_l[n mod 32], needed for n in [-32, 32) only:
//     y[k] = sum_l B_l[k] and y[k - 32] = sum_l W_64^l B_l[k], B_l[k] =
//     W_C^{-l k} A_l[k] (LDS table) -- a reduce-scatter over the wave:
//     v_permlane32_swap (lanes 0-31 keep the y[k] sums, 32-63 the y[k - 32]
//     ones), v_permlane16_swap (k bit 4), then DPP row_ror:8, row_half_mirror,
//     quad_perm [1,0,3,2] and [2,3,0,1] (k bits 3, 2, 0, 1), after which lane l
//     holds y[n] with n = l (l < 32) or l - 64: k_frame16's pass-3 lag layout;
//   * the first argmax, the lag prior and the outputs as in k_frame16.
// The 28 pairs go to waves w and w + 16: seven per SIMD.
template <int C>
struct f16w_lds {
    static constexpr int G = 16384 / C;
    static constexpr int SLOT = C + C / 16 + 2;  // Z at pidx(0..C-1), then U at 0..C
    static constexpr size_t TBL = (size_t)G * SLOT * sizeof(f2);    // [31][64] W_C^{-l k}, k = 1..31
    static constexpr size_t TT = TBL + 31 * 64 * sizeof(f2);         // [3][16][16] kp.r16_tw
    static constexpr size_t PRIOR = TT + 3 * 16 * 16 * sizeof(f2);   // [128] the lag prior
    static constexpr size_t RED = PRIOR + 128 * sizeof(float);       // [16] DC partial sums
    static constexpr size_t LAG = RED + 16 * sizeof(int);            // [TDOA_MAX_PAIRS] lags
    static constexpr size_t BYTES = LAG + TDOA_MAX_PAIRS * sizeof(int);
};
static_assert(f16w_lds<2048>::BYTES <= 160 * 1024, "k_frame16w LDS");

// cos(2 pi q / 64), q = 0..16
__device__ constexpr double COS64D[17] = {
    1.0, 0.99518472667219693, 0.98078528040323043, 0.95694033573220882, 0.92387953251128674,
    0.88192126434835505, 0.83146961230254524, 0.77301045336273699, 0.70710678118654757,
    0.63439328416364549, 0.55557023301960229, 0.47139673682599781, 0.38268343236508984,
    0.29028467725446233, 0.19509032201612833, 0.09801714032956077, 0.0};
// conj(W_64^q) = e^{+2 pi i q / 64}, q < 32 (q = 0, 16: no product)
__device__ constexpr f2 w64conj(int q)
{
    return q <= 16 ? f2{(float)COS64D[q], (float)COS64D[16 - q]}
                   : f2{(float)-COS64D[32 - q], (float)COS64D[q - 16]};
}

// one step of the reduce-scatter over DPP partners: lanes with lane bit BIT
// clear keep the sum of the registers' lo values, the others of hi
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ f2 rs_dpp(f2 lo, f2 hi, bool up)
{
    const float kx = up ? hi.x : lo.x, ky = up ? hi.y : lo.y;
    const float sx = up ? lo.x : hi.x, sy = up ? lo.y : hi.y;
    return f2{kx + dpp_f<CTRL>(sx), ky + dpp_f<CTRL>(sy)};
}
constexpr int DPP_QP_1032 = 0xB1;  // quad_perm [1,0,3,2]: lane bit 0 partner
constexpr int DPP_QP_2301 = 0x4E;  // quad_perm [2,3,0,1]: lane bit 1 partner
constexpr int DPP_ROW_HMIRROR = 0x141;  // i <-> 7 - i in each half row
constexpr int DPP_ROW_ROR8 = 0x128;     // i <-> i ^ 8 in each row

#ifndef F16W_PREFETCH_EARLY
#define F16W_PREFETCH_EARLY 1  // the next frame's words requested before the pairs
#endif
#ifndef F16W_DIF
#define F16W_DIF 0  // 1: the in-place DIF DFT-32 (fft32p) instead of the FMA DIT one
#endif
#ifndef F16W_QB
#define F16W_QB 8  // bins (q) between scheduling barriers
#endif
#ifndef F16W_KB
#define F16W_KB 2  // DFT outputs (k) between scheduling barriers
#endif
// the pruned inverse of pair (Ui, Uj) by one wave: lane l returns y[n],
// n = l (l < 32) or l - 64, unscaled (x 2C)
template <int C>
__device__ __forceinline__ f2 frame16w_inverse(const f2 *Ui, const f2 *Uj, const f2 *tbl, f2 w2l, f2 oml, int lane)
{
    static_assert(C == 2048, "32 bins per lane");
    constexpr int PQ = 64;  // index step of one q (U in the plain layout)
    const int ob = lane;                  // b = l + 64 q
    const int pbase = PQ - lane;          // C - b = pbase + PQ (31 - q)
    f2 y[32];
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const f2 Rk = c_conjmul(F16_LD(Ui + ob + PQ * q), F16_LD(Uj + ob + PQ * q));  // R[b]
        const f2 Rq = c_conjmul(F16_LD(Ui + pbase + PQ * (31 - q)), F16_LD(Uj + pbase + PQ * (31 - q)));  // R[C-b]
        const f2 ss = c_addconj(Rk, Rq);
        const f2 dd = c_mulconj(c_subconj(Rk, Rq), w2l);
        if (q == 0)
            y[q] = c_add_i(ss, dd);
        else if (q == 16)  // conj(W_64^16) = i: ss + i (i dd)
            y[q] = ss - dd;
        else
            y[q] = c_add_i(ss, c_mul_s(dd, w64conj(q)));
        if ((q & (F16W_QB - 1)) == F16W_QB - 1)  // bounded read-ahead (the reads all hoisted spill)
            __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
#if F16W_DIF
    fft32p<true, false>(y);  // A_l[k] in y[brev5(k)]
#define F16W_A(k) y[brev5(k)]
#else
    fft32d<true, false>(y);
#define F16W_A(k) y[k]
#endif
    __builtin_amdgcn_sched_barrier(0);
    // B = W_C^{-l k} A, C = W_64^l B; permlane32: lanes 0-31 (B_l, B_{l+32}),
    // lanes 32-63 (C_l, C_{l+32})
    f2 z[32];
#pragma unroll
    for (int k = 0; k < 32; k++) {
        f2 b = k == 0 ? F16W_A(0) : c_mul(F16W_A(k), F16_LD(tbl + (k - 1) * 64 + lane));
        f2 c = c_mul(b, oml);
        pswap32(b, c);
        z[k] = b + c;
        asm volatile("" ::"v"(z[k]));  // the sum here: not sunk to stage 2 (both halves live until then)
        if ((k & (F16W_KB - 1)) == F16W_KB - 1)
            __builtin_amdgcn_sched_barrier(0);
    }
#undef F16W_A
    // permlane16: even rows keep k, odd rows k + 16
#pragma unroll
    for (int k = 0; k < 16; k++) {
        f2 a = z[k], b = z[k + 16];
        pswap16(a, b);
        y[k] = a + b;
    }
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
#pragma unroll
    for (int k = 0; k < 8; k++)
        y[k] = rs_dpp<DPP_ROW_ROR8>(y[k], y[k + 8], b3);
#pragma unroll
    for (int k = 0; k < 4; k++)
        y[k] = rs_dpp<DPP_ROW_HMIRROR>(y[k], y[k + 4], b2);
    y[0] = rs_dpp<DPP_QP_1032>(y[0], y[1], b0);
    y[1] = rs_dpp<DPP_QP_1032>(y[2], y[3], b0);
    return rs_dpp<DPP_QP_2301>(y[0], y[1], b1);
}

#ifdef TDOA_DIAG
#define F16W_MARK()                                      \
    do {                                                 \
        if (nst < NSTAMP - 3)                            \
            stamp[nst++] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define F16W_MARK() \
    do {            \
    } while (0)
#endif

// (kp, out) must stay the first two parameters: kernarg_out() reads `out`
// at its kernarg offset
template <int C, int M>
__global__ void __launch_bounds__(1024, 1) k_frame16w(tdoa_kparams kp, tdoa_kout out,
                                                      const int16_t *__restrict__ frames, int64_t B, float e2)
{
    using L = f16w_lds<C>;
    constexpr int T = C / 16, G = L::G, SLOT = L::SLOT;
    static_assert(M == G, "one forward group per mic");
    constexpr int P = M * (M - 1) / 2;
    static_assert(P <= 32 && P > 16, "two pair slots per wave");
    __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
    f2 *bufs = (f2 *)smem;
    f2 *tbl = (f2 *)(smem + L::TBL);
    f2 *ttl = (f2 *)(smem + L::TT);
    float *priorl = (float *)(smem + L::PRIOR);
    int *red = (int *)(smem + L::RED);
    int *lagl = (int *)(smem + L::LAG);
    const int g = (int)threadIdx.x / T;
    const int K = kp.K, S = kp.S;
    f2 *buf = bufs + g * SLOT;
    const uint32_t *win = reinterpret_cast<const uint32_t *>(kp.window);
    const f2 *tw = reinterpret_cast<const f2 *>(kp.tw);
    const f2 *tw2 = reinterpret_cast<const f2 *>(kp.tw2);
    if (threadIdx.x < 3 * 16 * 16)
        ttl[threadIdx.x] = reinterpret_cast<const f2 *>(kp.r16_tw)[threadIdx.x];
    if (threadIdx.x < (unsigned)kp.K)
        priorl[threadIdx.x] = kp.prior[threadIdx.x];
    for (int e = threadIdx.x; e < 31 * 64; e += 1024) {  // W_C^{-l k} = conj(kp.tw[l k])
        const int k = (e >> 6) + 1, l = e & 63;
        const f2 t = tw[l * k];
        tbl[e] = f2{t.x, -t.y};
    }
    const int lane = (int)threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    // the wave's two pairs' table entries, read once here: a byte of kp
    // indexed per pair is a VMEM load, and its vmcnt wait inside the frame
    // loop would also wait for the next frame's words prefetched before the pairs
    auto rfl = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
    const int q1 = wv + 16 < P ? wv + 16 : wv;
    const int mi0 = rfl(kp.pair_i[wv]), mj0 = rfl(kp.pair_j[wv]);
    const int mi1 = rfl(kp.pair_i[q1]), mj1 = rfl(kp.pair_j[q1]);
    const int lo0 = rfl(kp.wc_lo[wv]), w0 = rfl(kp.wc_w[wv]), of0 = rfl(kp.wc_off[wv]);
    const int lo1 = rfl(kp.wc_lo[q1]), w1 = rfl(kp.wc_w[q1]), of1 = rfl(kp.wc_off[q1]);
    const f2 w2l = tw2[lane];       // W_2C^l: the pre-twiddle's lane factor
    const f2 oml = tw[32 * lane];   // W_64^l = W_C^{32 l}
    const f2 *tt = ttl;  // visible after the first barrier (the DC sum's)
#ifdef TDOA_DIAG
    constexpr int NSTAMP = 32;
    unsigned long long stamp[NSTAMP] = {};
    int nst = 0;
    const int64_t diag_fr = blockIdx.x + (B >= (int64_t)(F16_DIAG_FRAME + 1) * gridDim.x ? F16_DIAG_FRAME : 0) *
                                             (int64_t)gridDim.x;
#else
    constexpr int64_t diag_fr = -1;
#endif
    uint32_t w[8];
    auto fetch = [&](int64_t f) {
        const uint32_t *x = reinterpret_cast<const uint32_t *>(frames + (f * M + g) * (int64_t)C) +
                            ((int)threadIdx.x - g * T);
#pragma unroll
        for (int s = 0; s < 8; s++)
            w[s] = __builtin_nontemporal_load(x + T * s);
    };
    fetch(blockIdx.x);
    for (int64_t fr = blockIdx.x; fr < B; fr += gridDim.x) {
        const int tid = opaque_idx((int)threadIdx.x), j = tid - g * T, pj = pidx(j);
        if (fr == diag_fr) {
#ifdef TDOA_DIAG
            stamp[30] = __builtin_amdgcn_s_memrealtime();
#endif
            F16W_MARK();
        }
        const uint32_t wr0[8] = {};
        frame16_forward<C, 0>(w, win, wr0, buf, red, tt, tid, g, j, pj, kp.log2N, [] {});
        if (fr == diag_fr)
            F16W_MARK();  // forward transforms done
        // ---- 2. split + unit normalisation: thread b reads Z_m[b], Z_m[C - b]
        // (pidx layout), then, after a barrier, writes U_m[b] and U_m[C - b]
        // at their plain indices (b = 0: U_m[0], U_m[C]): the pairs' lane-
        // consecutive reads of the plain layout are bank-conflict free
        {
            const int b = tid;
            const f2 wb = tw2[b];
            const int pb = pidx(b), pr = pidx((C - b) & (C - 1));
            f2 ub[M], un[M];
#pragma unroll
            for (int m = 0; m < M; m++) {
                const f2 *zb = bufs + m * SLOT;
                const f2 z = F16_LD(zb + pb), zp = F16_LD(zb + pr);
                const f2 e = c_addconj(z, zp);
                const f2 od = c_mul(c_subconj(z, zp), wb);
                ub[m] = c_unit(c_add_mi(e, od), e2);
                un[m] = c_unit(c_conj_add_i(e, od), e2);
            }
            f2 uh = f2{0.0f, 0.0f};
            if (tid < M) {  // X[C/2] = conj(Z[C/2]) (x2): self-paired bin
                const f2 v = F16_LD(bufs + tid * SLOT + pidx(C / 2));
                uh = c_unit(f2{2.0f * v.x, -2.0f * v.y}, e2);
            }
            __syncthreads();
#pragma unroll
            for (int m = 0; m < M; m++) {
                bufs[m * SLOT + b] = ub[m];
                bufs[m * SLOT + C - b] = un[m];
            }
            if (tid < M)
                bufs[tid * SLOT + C / 2] = uh;
        }
        __syncthreads();
        if (fr == diag_fr)
            F16W_MARK();  // unit spectra in the slots
#if F16W_PREFETCH_EARLY
        {
            const int64_t fn = fr + gridDim.x;
            fetch(fn < B ? fn : fr);  // the next frame's words (or a harmless re-read)
        }
#endif
        // ---- 3. pairs wv and wv + 16 of this wave, no barriers
        const float invL = 1.0f / (float)(2 * C);
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            const int p = wv + 16 * h;
            if (p >= P)
                break;
            const f2 *Ui = bufs + (h ? mi1 : mi0) * SLOT, *Uj = bufs + (h ? mj1 : mj0) * SLOT;
            // the lane index re-derived per pair: the lag / address arithmetic
            // below stays here instead of being hoisted (and spilled) above the frames
            const int ln = opaque_idx((int)threadIdx.x) & 63;
            const f2 yv = frame16w_inverse<C>(Ui, Uj, tbl, w2l, oml, ln);
            const int n = ln < 32 ? ln : ln - 64;
            const int ka = 2 * n + S, kb = 2 * n + 1 + S;
            const bool oka = ka >= 0 && ka < K, okb = kb >= 0 && kb < K;
            const float sa = yv.x * invL, sb = yv.y * invL;
            // first maximum (the lowest lag wins ties), by keys to every lane
            int bkey = INT_MIN, bk = INT_MAX;
            if (oka) {
                bkey = fkey(sa);
                bk = ka;
            }
            if (okb && fkey(sb) > bkey) {
                bkey = fkey(sb);
                bk = kb;
            }
            wave_argmax_key(bkey, bk);
            bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);
            const size_t gb = (size_t)(fr * P + p) * K;
            float *wc = kernarg_out()->weighted_c;
            const int wlo = h ? lo1 : lo0, ww = h ? w1 : w0;
            float *wcp = wc ? wc + (size_t)fr * kp.wc_CK + (h ? of1 : of0) - wlo : nullptr;
            if (oka) {
                const int dd = ka > bk ? ka - bk : bk - ka;
                const float wa = sa * priorl[dd];
                if (out.scores_f)
                    out.scores_f[gb + ka] = sa;
                if (out.weighted_f)
                    out.weighted_f[gb + ka] = wa;
                if (wcp && ka >= wlo && ka < wlo + ww)
                    wcp[ka] = wa;
            }
            if (okb) {
                const int dd = kb > bk ? kb - bk : bk - kb;
                const float wb = sb * priorl[dd];
                if (out.scores_f)
                    out.scores_f[gb + kb] = sb;
                if (out.weighted_f)
                    out.weighted_f[gb + kb] = wb;
                if (wcp && kb >= wlo && kb < wlo + ww)
                    wcp[kb] = wb;
            }
            if (float *pk3 = kernarg_out()->peak3) {
                float *dst = pk3 + (size_t)(fr * P + p) * 3 + 1 - bk;
                if (oka && ka >= bk - 1 && ka <= bk + 1)
                    dst[ka] = sa;
                if (okb && kb >= bk - 1 && kb <= bk + 1)
                    dst[kb] = sb;
            }
            if (ln == 0) {
                out.lags[fr * P + p] = bk - S;
                lagl[p] = bk - S;
            }
            if (fr == diag_fr)
                F16W_MARK();  // a pair done
        }
#if !F16W_PREFETCH_EARLY
        {
            const int64_t fn = fr + gridDim.x;
            fetch(fn < B ? fn : fr);
        }
#endif
        __syncthreads();  // the slots are rewritten by the next frame
        if (tid == 0 && out.gate) {
            int tot = 0;
            for (int q = 0; q < P; q++)
                tot += lagl[q] * lagl[q];
            out.gate[fr] = tot > 4 ? 1 : 0;  // sample_compute.h:124-134
        }
#ifdef TDOA_DIAG
        if (fr == diag_fr) {
            stamp[31] = __builtin_amdgcn_s_memrealtime();
            stamp[29] = __builtin_amdgcn_s_memtime();
        }
#endif
    }
#ifdef TDOA_DIAG
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 128)
        for (int i = 0; i < 32; i++)
            g_diag_f16[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 32 + i] = stamp[i];
#endif
}
#undef F16W_MARK

template <int C, int M>
int launch_frame16w(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B, float e2,
                    hipStream_t st)
{
    if (B <= 0)
        return 0;
    const int res = tdoa_resident_blocks((const void *)k_frame16w<C, M>, 1024, 0);
    if (res < 1)
        return tdoa_set_error(-2, "k_frame16w: no resident workgroup (LDS / registers)");
    const int64_t grid = B < (int64_t)res ? B : (int64_t)res;
    hipLaunchKernelGGL((k_frame16w<C, M>), dim3((unsigned)grid), dim3(1024), 0, st, kp, out, frames, B, e2);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof msg, "k_frame16w launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, msg);
    }
    return 0;
}
#endif  // TDOA_AB

// k_frame16w (one wave per pair) or k_frame16 (a group of waves per pair) for
// config 4's shape: TDOA_F16=w | grp, default grp (measured: 106.2 vs 103.2
// ms per config-4 step, both with volatile LDS reads)
bool frame16w_pick()
{
#if !TDOA_AB
    return false;  // the product library has only k_frame16
#endif
    static const int pick = [] {
        const char *e = getenv("TDOA_F16");
        return e && !strcmp(e, "w") ? 1 : 0;
    }();
    return pick == 1;
}

}  // namespace
// the fused per-frame kernel's shapes (one group of threads per mic)
bool frame16_shape(const tdoa_kparams &kp)
{
    return (kp.N == 4096 && (kp.M == 3 || kp.M == 4)) || (kp.N == 2048 && (kp.M == 4 || kp.M == 8));
}
bool tdoa_phat_r16_fits(int M, int N, int S);
// a grid-requesting launch of this shape solves the grid in k_frame16 (FG):
// no weighted-score scratch and no k_grid_bb launch (tdoa_capi.cpp run_batch)
bool tdoa_frame16_fused_grid(const tdoa_kparams &kp)
{
    if (!tdoa_phat_r16_fits(kp.M, kp.N, kp.S) || !frame16_shape(kp))
        return false;
    if (kp.N == 2048 && kp.M == 8)
        return !frame16w_pick() && frame16_fg<2048, 8>(kp);
    if (kp.N == 4096 && kp.M == 4)
        return frame16_fg<4096, 4>(kp);
    if (kp.N == 4096 && kp.M == 3)
        return frame16_fg<4096, 3>(kp);
    if (kp.N == 2048 && kp.M == 4)
        return frame16_fg<2048, 4>(kp);
    return false;
}
// the name of the fused kernel a frame16_shape launch runs
const char *frame16_kernel_name(const tdoa_kparams &kp)
{
    return kp.N == 2048 && kp.M == 8 && frame16w_pick() ? "k_frame16w" : "k_frame16";
}
namespace {

__global__ void k_r16_gate(const int32_t *__restrict__ lags, uint8_t *__restrict__ gate, int64_t B, int P)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B)
        return;
    int tot = 0;
    for (int p = 0; p < P; p++) {
        const int b = lags[f * P + p];
        tot += b * b;
    }
    gate[f] = tot > 4 ? 1 : 0;  // sample_compute.h:124-134
}

template <int C>
int launch_r16(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
               float e2, void *scratch, size_t scratch_bytes, hipStream_t st)
{
    const int M = kp.M, P = kp.P;
    const size_t per_frame = (size_t)M * r16_row<C>() * sizeof(f2);
    const int64_t chunk = (int64_t)(scratch_bytes / per_frame);
    if (chunk < 1)
        return tdoa_set_error(-1, "GCC_PHAT: spectrum scratch smaller than one frame");
    const size_t lds = (size_t)(C + C / 16) * sizeof(f2);
    const size_t lds_pair = (size_t)(C / 2 + C / 32) * sizeof(f2);  // half-size buffer (k_pair16)
    for (int64_t c0 = 0; c0 < B; c0 += chunk) {
        const int64_t nf = (B - c0) < chunk ? (B - c0) : chunk;
        if (nf * P > INT_MAX)
            return tdoa_set_error(-1, "GCC_PHAT: chunk too large for one launch");
        hipLaunchKernelGGL(k_spec16<C>, dim3((unsigned)(nf * M)), dim3(C / 16), lds, st, kp, frames, c0 * M,
                           (f2 *)scratch, e2);
        hipLaunchKernelGGL(k_pair16<C>, dim3((unsigned)(nf * P)), dim3(C / 16), lds_pair, st, kp, out,
                           (const f2 *)scratch, c0, nf * P);
    }
    if (out.gate) {
        const int64_t g = (B + 255) / 256;
        hipLaunchKernelGGL(k_r16_gate, dim3((unsigned)g), dim3(256), 0, st, out.lags, out.gate, B, P);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof msg, "GCC_PHAT r16 launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, msg);
    }
    return 0;
}

}  // namespace

bool tdoa_phat_r16_fits(int M, int N, int S)
{
    return (N == 2048 || N == 4096) && M >= 2 && M <= TDOA_MAX_MICS_K && S <= 63;
}

// the least-squares refinement's peak scores come from the kernel (peak3)
bool tdoa_phat_r16_peak3(const tdoa_kparams &kp)
{
    return tdoa_phat_r16_fits(kp.M, kp.N, kp.S) && frame16_shape(kp);
}

int tdoa_launch_phat_r16(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
                         float phat_eps, void *scratch, size_t scratch_bytes, void *stream)
{
    if (!tdoa_phat_r16_fits(kp.M, kp.N, kp.S))
        return tdoa_set_error(-1, "GCC_PHAT r16: unsupported shape");
    if (!scratch)
        return tdoa_set_error(-1, "GCC_PHAT: context has no spectrum scratch");
    // per-mic clamp |X_m| >= sqrt(eps) in the oracle's units (x / 2^15, X / 2):
    // |X|^2 >= eps * 2^32 in the kernel's int16 units with the split's factor 2
    float e2 = phat_eps * 4294967296.0f;
    if (!(e2 >= 1e-30f))
        e2 = 1e-30f;
    hipStream_t st = (hipStream_t)stream;
    // the per-frame fused kernel (spectra on chip) for M = 3, 4 at frame_len 4096
    // and M = 4, 8 at 2048 (config 3: 6.41 vs 7.86 ms per 65536 frames, config
    // 4: 161 vs 198 ms per 1e6); other mic counts take the two-pass kernels
    if (kp.N == 4096 && kp.M == 4)
        return launch_frame16<4096, 4>(kp, out, frames, B, e2, st);
    if (kp.N == 4096 && kp.M == 3)
        return launch_frame16<4096, 3>(kp, out, frames, B, e2, st);
    if (kp.N == 2048 && kp.M == 8)
#if TDOA_AB
        if (frame16w_pick())
            return launch_frame16w<2048, 8>(kp, out, frames, B, e2, st);
#endif
        return launch_frame16<2048, 8>(kp, out, frames, B, e2, st);
    if (kp.N == 2048 && kp.M == 4)
        return launch_frame16<2048, 4>(kp, out, frames, B, e2, st);
    return kp.N == 4096 ? launch_r16<4096>(kp, out, frames, B, e2, scratch, scratch_bytes, st)
                        : launch_r16<2048>(kp, out, frames, B, e2, scratch, scratch_bytes, st);
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch_f16b(unsigned long long *host, int n)
{
    if (n > (1 << 16))
        n = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_f16b), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
extern "C" int tdoa_diag_fetch_f16(unsigned long long *host, int n)
{
    if (n > (1 << 16))
        n = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_f16), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
