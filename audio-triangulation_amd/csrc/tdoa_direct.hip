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
#include <cstdlib>

#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

#ifdef TDOA_DIAG
// Diagnostic build only (libtdoa_diag.so): per-workgroup phase stamps.
#define TDOA_DIAG_SLOTS 16
__device__ unsigned long long g_diag[1 << 20];
#define DIAG_STAMP(i)                                                   \
    do {                                                                \
        if (threadIdx.x == 0)                                           \
            g_diag[(size_t)blockIdx.x * TDOA_DIAG_SLOTS + (i)] =        \
                __builtin_amdgcn_s_memtime();                           \
    } while (0)
#define TDOA_GRID_MARK(i) DIAG_STAMP(i)
// the constant 100 MHz clock (one base for every CU): slots 11 / 12
#define DIAG_RT(i)                                                      \
    do {                                                                \
        if (threadIdx.x == 0)                                           \
            g_diag[(size_t)blockIdx.x * TDOA_DIAG_SLOTS + (i)] =        \
                __builtin_amdgcn_s_memrealtime();                       \
    } while (0)
#else
#define DIAG_STAMP(i) \
    do {              \
    } while (0)
#define DIAG_RT(i) \
    do {           \
    } while (0)
#endif

#include "tdoa_device.h"
#include "tdoa_keys.h"

namespace {

template <bool PREPARED, int TWC>
__global__ void __launch_bounds__(1024) k_direct(tdoa_kparams kp, tdoa_kout out,
                                                 const int16_t *__restrict__ frames, int64_t B,
                                                 const int32_t *__restrict__ count)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Smem sm = carve(smem, kp, blockDim.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kp.F;
    DIAG_STAMP(10);
    if (count) {  // batch size known on the device only (streaming pipeline)
        const int64_t c = *count;
        B = c < B ? c : B;
        if (f0 >= B)
            return;
    }
    const int nf = (int)((B - f0) < kp.F ? (B - f0) : kp.F);
    DIAG_STAMP(0);
    stage_frames<PREPARED>(kp, sm, frames, f0, nf);
    DIAG_STAMP(1);
    xcorr_phase(kp, sm, nf);
    DIAG_STAMP(2);
    argmax_prior_phase<int64_t>(kp, sm.scores, sm.best, out, f0, nf);
    DIAG_STAMP(3);
    DIAG_STAMP(4);  // grid solve runs in k_grid (tdoa_grid.hip)
}

// ------------------------------------------------ exact xcorr on the matrix cores
// k_direct_mfma: the same stage / argmax / prior / gate as k_direct, with the
// int64 cross-correlation (correlations.c:9-18) on v_mfma_i32_16x16x64_i8.
//   Offset byte limbs: every int16 x is stored as z = x ^ 0x0080, whose high
//   byte h = x >> 8 and low byte l = (x & 255) - 128 are int8 with
//   x' = x - 128 = 256 h + l.  a'.b' = 65536 ah.bh + 256 (ah.bl + al.bh)
//   + al.bl; each limb product accumulates exactly in int32 (<= 2 (N+64) 128^2).
//   Lag s = 16 (n - n0) + w is C[w][n] of a Toeplitz product summed over
//   NB 64-sample blocks beta:  A[w][k] = a[64 beta + k - w],  B[k][n] =
//   b[64 beta + k + 16 (n - n0)]  (every i = 64 beta + k - w once), over a
//   window of L = 64 NB indices that holds the whole a-row and b[16 (n - n0)..N).
//   Padding (x = 0) is z = 0x0080, so over the window
//   sum a b = sum a'b' + 128 (sum a + sum_window b) - 128^2 L  exactly.
// Lane l holds A row w = l & 15, B column n = l & 15, k = 16 (l >> 4) + j in
// byte j of its 16-byte operands (A and B pair byte for byte), and C rows
// 4 (l >> 4) + e of column l & 15.
constexpr int MF_GR = 4;      // keyed grid: tuple words held per thread (the 16-wave form)
constexpr int MF_GR_EMA = 5;  // ... and in the 8-wave streaming workgroup (U <= 5 x 512)
// zero words each side of a staged row: 2 PADW bytes per plane and side.  For
// S <= 63 the a reads span [-16, N + 68) and the b reads [-64, N + 112) samples
// (a: q0 = 64 beta + 16 g - r >= -15, five dwords from q0 & ~3; b: qb = 64 beta
// + 16 (g + rr - n0), rr - n0 <= ceil((S + 1) / 16) - 1 <= 3, one 16-B read), so
// 56 words (112 bytes) suffice; 2 PADW stays a multiple of 16 (aligned b reads).
// (96 before round 5: the config-5 workgroup's 44.6 KB of LDS allowed 3 per CU)
constexpr int MF_PADW = 56;

typedef int v4i_mf __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i_mf mf_limbs(const uint32_t (&w)[8], uint32_t sel)
{
    v4i_mf r;
#pragma unroll
    for (int d = 0; d < 4; d++)
        r[d] = (int)__builtin_amdgcn_perm(w[2 * d + 1], w[2 * d], sel);
    return r;
}

// LDS score table of the matrix-core kernel: [F][P][K], or for single-word
// tuples (F = 4) frame-interleaved [P][K][4] -- the grid solve then reads a
// slot's four frames with two 16-B reads instead of four 8-B reads
template <bool IL>
__device__ __forceinline__ int sidx(int f, int p, int k, int P, int K)
{
    return IL ? ((p * K + k) << 2) + f : (f * P + p) * K + k;
}

// argmax + lag prior + gate (correlations.c:20-33, sample_compute.h:124-134)
// for the matrix-core kernel: one wave per (frame, pair), DPP key reduction
template <bool IL>
__device__ void argmax_prior_mf(const tdoa_kparams &kp, int64_t *scores, int *bestlag, const float *prior,
                                const tdoa_kout &out, int64_t f0, int nf)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P;
    for (int fp = wave; fp < nf * P; fp += nwaves) {
        const int ff = fp / P, pp = fp - ff * P;
        int64_t *sc = scores + sidx<IL>(ff, pp, 0, P, K);
        constexpr int KS = IL ? 4 : 1;  // stride of consecutive lags
        const int k1 = lane, k2 = lane + 64;
        const int64_t v1 = k1 < K ? sc[KS * k1] : 0, v2 = k2 < K ? sc[KS * k2] : 0;
        uint64_t key = k1 < K ? vkey<7>(v1, k1) : 0;
        if (k2 < K) {
            const uint64_t k2k = vkey<7>(v2, k2);
            key = k2k > key ? k2k : key;
        }
        const int bk = key_index<7>(lane63_u64(wave_umax_dpp(key)));
        const size_t gbase = (size_t)(f0 * P + fp) * K;
        if (k1 < K) {
            const int d = k1 > bk ? k1 - bk : bk - k1;
            const int64_t wv = apply_prior(v1, prior[d]);
            sc[KS * k1] = wv;
            store_score(out, gbase + k1, v1, wv);
        }
        if (k2 < K) {
            const int d = k2 > bk ? k2 - bk : bk - k2;
            const int64_t wv = apply_prior(v2, prior[d]);
            sc[KS * k2] = wv;
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

// grid solve (vga_heatmap.h:99-108) of the workgroup's <= 4 frames for
// single-word tuples: the thread's <= GR tuple words and first cells were
// loaded at the kernel's start (q, cl); per frame the key maximum over the
// thread's tuples, the wave (DPP) and the workgroup (LDS, one barrier)
// PC: the pair count at compile time (0: kp.P at run time) -- a fixed count
// unrolls the pair loop, so a tuple's 2 P reads issue back to back instead of
// one LDS round trip per pair (config 2 / 5: P = 3)
template <int GR, int PC>
__device__ void grid_mf(const tdoa_kparams &kp, const int64_t *scores, uint64_t *red, const uint32_t (&q)[GR],
                        const int32_t (&cl)[GR], const tdoa_kout &out, int64_t f0, int nf,
                        uint32_t omask = 0xFFFFFFFFu)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6, nt = blockDim.x;
    const int K = kp.K, P = PC ? PC : kp.P, U = kp.U;
    uint64_t best[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < GR; r++) {
        if (tid + r * nt < U) {
            // frame-interleaved table: the slot's four frames in two 16-B reads
            typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
            i64x2 L01 = {0, 0}, L23 = {0, 0};
#pragma unroll
            for (int p = 0; p < (PC ? PC : 4); p++) {  // single-word tuples: P <= 4
                if (!PC && p >= P)
                    break;
                const i64x2 *sl = reinterpret_cast<const i64x2 *>(
                    scores + sidx<true>(0, p, (q[r] >> (8 * p)) & 0xFFu, P, K));
                L01 += sl[0];
                L23 += sl[1];
            }
            const int64_t L[4] = {L01.x, L01.y, L23.x, L23.y};
#pragma unroll
            for (int f = 0; f < 4; f++) {
                const uint64_t k = vkey<16>(L[f], cl[r]);
                best[f] = k > best[f] ? k : best[f];
            }
        }
    }
    TDOA_GRID_MARK(8);
#pragma unroll
    for (int f = 0; f < 4; f++)
        best[f] = wave_umax_dpp(best[f]);
    if (lane == 63)
#pragma unroll
        for (int f = 0; f < 4; f++)
            red[wave * 4 + f] = best[f];
    __syncthreads();
    TDOA_GRID_MARK(9);
    if (tid < nf && ((omask >> tid) & 1u)) {  // omask: the frames whose outputs are written
        const int f = tid;
        uint64_t k = red[f];
        for (int w = 1; w < nwaves; w++) {
            const uint64_t o = red[w * 4 + f];
            k = o > k ? o : k;
        }
        const int cell = key_index<16>(k);
        const int64_t fi = f0 + f;
        if (out.cell)
            out.cell[fi] = cell;
        if (out.max_L)
            out.max_L[fi] = key_value<16>(k);
        if (out.xy) {
            const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
            out.xy[2 * fi] = (float)(cx - kp.half_w) / kp.grid_scale;
            out.xy[2 * fi + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
        }
    }
}

// Streaming (tdoa_stream.cpp, BASELINE config 5): the EMA of correlations.c:
// 38-63 on the stream state of the batch's gated frames (sample_compute.h:134),
// on the weighted scores still in LDS -- which then hold the EMA scores the
// grid solve runs on (vga_heatmap.h reads corr_*) -- and the EMA argmax per
// pair (ema_best).  The clock now = end * 10^6 / fs.  Replaces k_stream_update's
// per-slot pass for the shapes this kernel solves (no fresh-score round trip).
// The stream states are requested at the kernel's start (ema_ids / ema_states: the
// thread's EMA_E elements of the workgroup's [F][P][K] block), so their HBM
// latency hides behind the staging and the xcorr.
// the streaming kernel's grid tables requested after the xcorr (see k_direct_mfma;
// 81.35 -> 79.5 us per config-5 hop, same box)
#ifndef MF_EMA_LATE_TABLES
#define MF_EMA_LATE_TABLES 1
#endif
// waves per SIMD the streaming (EMA) kernel is compiled for: 6 caps it at 80 VGPRs
#ifndef MF_EMA_WPE
#define MF_EMA_WPE 8
#endif
constexpr int EMA_E = 3;  // state elements per thread: F P K <= EMA_E x threads (host-checked)

struct EmaPre {
    int64_t ev[EMA_E];
};

// in two steps: the stream ids (requested with the staging's slot records),
// then the states.  Clamped, unguarded loads: a guarded load is a branch the
// wait-count pass cannot look through (one round trip per element)
struct EmaIds {
    int sid[EMA_E];
};
__device__ __forceinline__ EmaIds ema_ids(const tdoa_kparams &kp, const tdoa_stream_params &sp, int64_t f0, int nf)
{
    EmaIds e;
    const int PK = kp.P * kp.K;
#pragma unroll
    for (int i = 0; i < EMA_E; i++) {
        const int f = ((int)threadIdx.x + i * (int)blockDim.x) / PK;
        e.sid[i] = sp.ids[f0 + (f < nf ? f : nf - 1)];
    }
    return e;
}
__device__ __forceinline__ EmaPre ema_states(const tdoa_kparams &kp, const tdoa_stream_params &sp, const EmaIds &ids,
                                             int nf)
{
    EmaPre e;
    const int PK = kp.P * kp.K;
#pragma unroll
    for (int i = 0; i < EMA_E; i++) {
        const int x = (int)threadIdx.x + i * (int)blockDim.x;
        const int f = x / PK;
        const int64_t v = sp.est[(size_t)ids.sid[i] * PK + (f < nf ? x - f * PK : 0)];
        e.ev[i] = f < nf ? v : 0;
    }
    return e;
}

template <bool IL>
__device__ uint32_t ema_mf(const tdoa_kparams &kp, const tdoa_stream_fuse &ef, const EmaPre &pre,
                           int64_t *scores, const int *bestlag, float *decl, int64_t f0, int nf)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int K = kp.K, P = kp.P, PK = P * K;
    const tdoa_stream_params &sp = ef.sp;
    uint32_t gmask = 0;
    for (int f = 0; f < nf; f++) {  // sum_p best^2 > 4 (sample_compute.h:124-134)
        int tot = 0;
        for (int q = 0; q < P; q++) {
            const int b = bestlag[f * P + q];
            tot += b * b;
        }
        gmask |= (tot > 4 ? 1u : 0u) << f;
    }
    uint64_t now = 0;
    int s = 0;
    if (tid < nf) {  // the frame's decay (correlations.c:40-43), shared through LDS
        const int64_t slot = f0 + tid;
        s = sp.ids[slot];
        now = (uint64_t)sp.end[slot] * 1000000u / (uint64_t)sp.fs;
        decl[tid] = tdoa_decay_dev(now, sp.last[s]);
    }
    __syncthreads();
    // the EMA, element by element, of the states requested at the start
#pragma unroll
    for (int i = 0; i < EMA_E; i++) {
        const int x = tid + i * (int)blockDim.x;
        const int f = x / PK;
        if (f < nf && ((gmask >> f) & 1u)) {
            const int p = (x - f * PK) / K, k = x - f * PK - p * K;
            int64_t *sc = scores + sidx<IL>(f, p, k, P, K);
            const int64_t ev = pre.ev[i];
            const float delta = (float)(*sc - ev) * decl[f];
            const float sum = (float)ev + delta;
            const int64_t nv = (int64_t)sum;
            sp.est[(size_t)sp.ids[f0 + f] * PK + (x - f * PK)] = nv;
            *sc = nv;
        }
    }
    __syncthreads();  // EMA scores in LDS
    if (ef.so.ema_best) {
        constexpr int KS = IL ? 4 : 1;
        for (int fp = wave; fp < nf * P; fp += nwaves) {
            const int f = fp / P, p = fp - f * P;
            if (!((gmask >> f) & 1u))
                continue;
            const int64_t *sc = scores + sidx<IL>(f, p, 0, P, K);
            uint64_t key = 0;
            for (int k = lane; k < K; k += 64) {
                const uint64_t kk = vkey<7>(sc[KS * k], k);  // |EMA| <= 2^42 < 2^47 (tdoa_keys.h)
                key = kk > key ? kk : key;
            }
            const int bk = key_index<7>(lane63_u64(wave_umax_dpp(key)));
            if (lane == 0)
                ef.so.ema_best[(f0 + f) * P + p] = bk - kp.S;
        }
    }
    if (tid < nf) {
        const int64_t slot = f0 + tid;
        if ((gmask >> tid) & 1u)
            sp.last[s] = now;
        else if (ef.so.cell)
            ef.so.cell[slot] = -1;  // not gated: no update, no solve (sample_compute.h:134)
        if (ef.so.stream_id)
            ef.so.stream_id[slot] = s;
        if (ef.so.end)
            ef.so.end[slot] = sp.end[slot];
    }
    if (tid == 0 && gmask)
        atomicAdd((unsigned long long *)&sp.stats[1], (unsigned long long)__builtin_popcount(gmask));
    return gmask;
}

// the hop's bookkeeping (k_stream_update's block 0): the device sample clock,
// the running trigger count, the hop's trigger count
__device__ __forceinline__ void ema_hop(const tdoa_stream_fuse &ef, int cnt)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *ef.sp.pos += ef.sp.H;  // the trigger kernel has read it
        ef.sp.stats[0] += cnt;
        if (ef.so.count)
            *ef.so.count = cnt;
    }
}

// LDS side tables of k_direct_mfma beyond Smem (byte offsets, host-computed):
// rsum [F*M][4] the prepared rows' sums (whole row, first 16 / 32 / 48
// samples); prior [K] the lag prior; red [16][4] u64 grid keys per wave
struct MfTabs {
    int rsum, prior, red;
};

// Frames -> LDS in the offset-byte form the matrix cores read (x ^ 0x0080 per
// sample: high byte and low byte - 128 both int8), fused into one pass per
// chunk (16 B = 8 samples):
//   every global read of the phase (frame chunks, window chunks, the prior,
//   grid tables) is issued first -- one HBM latency, not one per pass;
//   the raw row sums (rolling_buffer.c:48-62 floor mean) by wave sums + one LDS
//   atomic per wave and row; then, from the chunks still in registers, the
//   prep (rolling_buffer.c:64-66, buffer.c:13-16, buffer.c:4-11), the prepared
//   rows' sums for the offset correction, and the offset form, stored once.
// CH: chunks per thread (>= ceil(F*M*N/8 / threads), host-checked).
// WS: the workgroup's thread count is a multiple of the chunks per row, so
// every chunk of a thread sits at the same row offset and reads the same
// window chunk: one window load per thread (8 registers fewer per chunk)
// between(): once the frames' first loads are requested (ring_chunks3) -- the
// streaming kernel's EMA state loads
template <bool PREPARED, int CH, bool WS = false, typename Between = NoBetween>
__device__ __forceinline__ void stage_mf(const tdoa_kparams &kp, const Smem &sm, char *smem, const MfTabs &tb,
                                         const int16_t *__restrict__ frames, int64_t f0, int nf,
                                         Between between = Between())
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int rows = nf * kp.M, NW = kp.N / 2, padw = kp.PADW, RS = kp.RS;
    int *rsum = reinterpret_cast<int *>(smem + tb.rsum);
    const int cpr = kp.N / 8;  // 16-byte chunks per row
    const int nchunk = rows * cpr;
    const int width = cpr < 64 ? cpr : 64;  // lanes of one wave that share a row
    constexpr int CW = WS ? 1 : CH;  // window chunks held per thread
    uint4 v[CH], w[CW];
    if constexpr (WS) {
        w[0] = make_uint4(0, 0, 0, 0);
        if (!PREPARED)
            w[0] = reinterpret_cast<const uint4 *>(kp.window)[tid % cpr];
    }
    if (WS && CH <= 3 && kp.frame_ring && kp.M == 3) {
        ring_chunks3<CH>(kp, f0, tid, nt, nchunk, cpr, v, between);
    } else {
    between();
#pragma unroll
    for (int i = 0; i < CH; i++) {
        const int c = tid + nt * i;
        v[i] = make_uint4(0, 0, 0, 0);
        if constexpr (!WS)
            w[i] = make_uint4(0, 0, 0, 0);
        if (c < nchunk) {
            const int r = c / cpr, k = c - r * cpr;
            if (kp.frame_ring) {  // streaming batch: frame f0 + r / M from its stream's ring
                const int fl = r / kp.M, m = r - fl * kp.M;
                v[i] = ring_chunk(kp, f0 + fl, m, k);
            } else if (kp.frames_u8) {
                v[i] = frame_chunk(kp, frames, f0 * kp.M + r, k);
            } else {
                v[i] = reinterpret_cast<const uint4 *>(frames + f0 * kp.M * kp.N)[c];
            }
            if constexpr (!WS)
                if (!PREPARED)
                    w[i] = reinterpret_cast<const uint4 *>(kp.window)[k];
        }
    }
    }
    // the prior: requested now, written once the frames have arrived
    const float pr = tid < kp.K ? kp.prior[tid] : 0.0f;
    // each row as two byte planes of its offset-form samples z = x ^ 0x0080
    // (plane 0: high bytes h = x >> 8, plane 1: low bytes l = (x & 255) - 128,
    // both int8 -- the matrix cores' operands, read without any byte
    // shuffles), RS words = 2 planes x (2 padw + N) bytes per row.  Pads are
    // zero samples: h = 0x00, l = 0x80.
    uint32_t *Xw = sm.X;
    const int pdw = padw / 2;  // pad dwords per side and plane (2 padw samples)
    const int PLD = RS / 2;    // dwords per plane
    for (int i = tid; i < rows * 4 * pdw; i += nt) {
        const int r = i / (4 * pdw), k = i - r * 4 * pdw;  // k: plane (k / 2pdw), side, dword
        const int pl = k >= 2 * pdw, kk = k - pl * 2 * pdw;
        Xw[r * RS + pl * PLD + (kk < pdw ? kk : NW / 2 + kk)] = pl ? 0x80808080u : 0u;
    }
    for (int i = tid; i < rows; i += nt)
        sm.sums[i] = 0;
    for (int i = tid; i < 4 * rows; i += nt)
        rsum[i] = 0;
    __syncthreads();  // sums zeroed
    DIAG_STAMP(6);
    // lane `width - 1` of each group of lanes sharing a row adds its group's sum
    auto wsum = [&](int x) { return group_sum_dpp(x, width); };
    const bool adder = (tid & (width - 1)) == width - 1;
    if (!PREPARED) {
#pragma unroll
        for (int i = 0; i < CH; i++) {
            const int c = tid + nt * i;
            if (nt * i < nchunk) {  // uniform: the wave's lanes join the shuffles
                const int s = wsum(sum_word(v[i].x) + sum_word(v[i].y) + sum_word(v[i].z) + sum_word(v[i].w));
                if (c < nchunk && adder)
                    atomicAdd(&sm.sums[c / cpr], s);
            }
        }
        __syncthreads();  // row sums complete
    }
    DIAG_STAMP(7);
    if (tid < kp.K)
        reinterpret_cast<float *>(smem + tb.prior)[tid] = pr;
#pragma unroll
    for (int i = 0; i < CH; i++) {
        const int c = tid + nt * i;
        if (nt * i < nchunk) {
            const bool ok = c < nchunk;
            const int r = ok ? c / cpr : 0, k = c - r * cpr;
            uint4 x = v[i];
            if (!PREPARED) {
                // floor mean: int64 `total >> BITS` == int32 arithmetic shift here
                const uint32_t off16 = (uint32_t)(sm.sums[r] >> kp.log2N) & 0xFFFFu;
                const uint4 wi = w[WS ? 0 : i];
                x.x = prep_word(x.x, off16, wi.x);
                x.y = prep_word(x.y, off16, wi.y);
                x.z = prep_word(x.z, off16, wi.z);
                x.w = prep_word(x.w, off16, wi.w);
            }
            const int ps = ok ? sum_word(x.x) + sum_word(x.y) + sum_word(x.z) + sum_word(x.w) : 0;
            const int s = wsum(ps);
            if (ok) {
                if (adder)
                    atomicAdd(&rsum[4 * r], s);
                // first 16 / 32 / 48 samples: chunks 0-1 / 0-3 / 0-5 of the row
                if (k < 6) {
                    if (k < 2)
                        atomicAdd(&rsum[4 * r + 1], ps);
                    if (k < 4)
                        atomicAdd(&rsum[4 * r + 2], ps);
                    atomicAdd(&rsum[4 * r + 3], ps);
                }
                x.x ^= 0x00800080u;
                x.y ^= 0x00800080u;
                x.z ^= 0x00800080u;
                x.w ^= 0x00800080u;
                // samples 8k .. 8k + 7: their high bytes and low bytes, 8 B per plane
                const uint32_t h0 = __builtin_amdgcn_perm(x.y, x.x, 0x07050301u);
                const uint32_t h1 = __builtin_amdgcn_perm(x.w, x.z, 0x07050301u);
                const uint32_t l0 = __builtin_amdgcn_perm(x.y, x.x, 0x06040200u);
                const uint32_t l1 = __builtin_amdgcn_perm(x.w, x.z, 0x06040200u);
                uint32_t *rw = Xw + r * RS + pdw + 2 * k;
                *reinterpret_cast<uint2 *>(rw) = make_uint2(h0, h1);
                *reinterpret_cast<uint2 *>(rw + PLD) = make_uint2(l0, l1);
            }
        }
    }
    __syncthreads();
}

template <bool PREPARED, int TWC, int CH, bool EMA>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(EMA && CH <= 4 ? MF_EMA_WPE : 1))) k_direct_mfma(tdoa_kparams kp, tdoa_kout out,
                                                      const int16_t *__restrict__ frames, int64_t B,
                                                      const int32_t *__restrict__ count, int n0, int nq,
                                                      MfTabs tb, tdoa_stream_fuse ef)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Smem sm = carve(smem, kp, blockDim.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kp.F;
    DIAG_STAMP(10);
    DIAG_RT(11);
    if (count) {  // batch size known on the device only (streaming pipeline)
        // at most B slots (one per stream): a corrupted counter is clamped
        // before any reader (ema_hop's stats, the batch bound) sees it
        int64_t c = *count;
        c = c < 0 ? 0 : (c > B ? B : c);
        if constexpr (EMA)
            ema_hop(ef, (int)c);
        B = c;
        if (f0 >= B)
            return;
    }
    const int nf = (int)((B - f0) < kp.F ? (B - f0) : kp.F);
    DIAG_STAMP(0);
    // single-word tuples (P <= 4): this thread's grid tuples and their first
    // cells, requested now and consumed by the grid solve at the end
    constexpr int GR = EMA ? MF_GR_EMA : MF_GR;  // the 8-wave streaming workgroup holds more tuples per thread
    constexpr bool KEYGRID = TWC == 1;
    uint32_t gq[GR];
    int32_t gc[GR];
    const bool do_grid = out.cell || out.xy || out.max_L;
    auto grid_tables = [&] {
#pragma unroll
        for (int r = 0; r < GR; r++) {
            const int u = (int)threadIdx.x + r * (int)blockDim.x;
            gq[r] = do_grid && u < kp.U ? kp.tuples[u] : 0u;
            gc[r] = do_grid && u < kp.U ? kp.tuple_cell[u] : 0;
        }
    };
    if constexpr (KEYGRID && !(EMA && MF_EMA_LATE_TABLES))
        grid_tables();
    EmaPre epre{};
    EmaIds eids{};
    if constexpr (EMA)
        eids = ema_ids(kp, ef.sp, f0, nf);
    // EMA launches: threads % (N / 8) == 0; their states are requested as soon
    // as the ids are in (with the slot records)
    stage_mf<PREPARED, CH, EMA>(kp, sm, smem, tb, frames, f0, nf, [&]() __attribute__((always_inline)) {
        if constexpr (EMA)
            epre = ema_states(kp, ef.sp, eids, nf);
    });
    DIAG_STAMP(1);
    DIAG_STAMP(2);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const int *rsum = reinterpret_cast<const int *>(smem + tb.rsum);
    const int RS = kp.RS;

    const int g = lane >> 4, r = lane & 15;
    const int K = kp.K, S = kp.S, P = kp.P, NB = kp.N / 64 + 1;
    // xcorr units.  Per pair (a, b): the tile's 16 rows are a's fine shifts, its
    // columns b's coarse 16-lag blocks, nq of them used.  xc3 (three mics, 2 nq
    // <= 16): per (frame, first mic a) -- a = 0 puts pairs (0,1) and (0,2) side by
    // side (columns 0 .. nq - 1 mic 1, nq .. 2 nq - 1 mic 2), a = 1 pair (1,2):
    // two tiles per frame instead of three, and the streaming workgroup's eight
    // waves take F = 4 frames' eight units in one pass (twelve units took two)
    const bool xc3 = kp.xc3 != 0;
    const int nu = xc3 ? 2 * nf : nf * P;
    for (int it = wave; it < nu; it += nwaves) {
        const int f = xc3 ? it >> 1 : it / P;
        const int ma = xc3 ? it & 1 : kp.pair_i[it - f * P];
        // this lane's column: pair p, partner row, coarse block cb (< nq: valid)
        int p, mb, cb;
        bool valid;
        if (xc3) {
            const int two = ma == 0 && r >= nq;  // a = 0: the second partner's columns
            const int c = r - two * nq;
            valid = c < nq;
            cb = c < nq ? c : nq - 1;
            p = ma == 0 ? two : 2;
            mb = ma == 0 ? 1 + two : 2;
        } else {
            p = it - f * P;
            mb = kp.pair_j[p];
            valid = r < nq;
            cb = r < nq ? r : nq - 1;
        }
        const int rowa = f * kp.M + ma, rowb = f * kp.M + mb;
        // byte planes (stage_mf): sample n's high byte at byte 2 padw + n of
        // plane 0, its offset low byte at the same byte of plane 1
        const char *ra = reinterpret_cast<const char *>(sm.X + rowa * RS) + 2 * kp.PADW;
        const char *rb = reinterpret_cast<const char *>(sm.X + rowb * RS) + 2 * kp.PADW;
        const int PLB = RS * 2;  // bytes per plane
        v4i_mf hh = {0, 0, 0, 0}, xx = {0, 0, 0, 0}, ll = {0, 0, 0, 0};
#pragma unroll 2
        for (int beta = 0; beta < NB; beta++) {
            // A: samples q0 .. q0 + 15, q0 = 64 beta + 16 g - w (w = r; any alignment,
            // may be negative): five aligned dwords per plane, byte-aligned in registers
            const int q0 = 64 * beta + 16 * g - r;
            const uint32_t *pa = reinterpret_cast<const uint32_t *>(ra + (q0 & ~3));
            const uint32_t sh = (uint32_t)(q0 & 3);
            uint32_t uh[5], ul[5];
#pragma unroll
            for (int m = 0; m < 5; m++) {
                uh[m] = pa[m];
                ul[m] = pa[PLB / 4 + m];
            }
            v4i_mf ah, al;
#pragma unroll
            for (int d = 0; d < 4; d++) {
                ah[d] = (int)__builtin_amdgcn_alignbyte(uh[d + 1], uh[d], sh);
                al[d] = (int)__builtin_amdgcn_alignbyte(ul[d + 1], ul[d], sh);
            }
            // B: samples 64 beta + 16 (g + n - n0) .. + 15: one aligned 16-B read per plane
            const int qb = 64 * beta + 16 * (g + cb - n0);
            const v4i_mf bh = *reinterpret_cast<const v4i_mf *>(rb + qb);
            const v4i_mf bl = *reinterpret_cast<const v4i_mf *>(rb + PLB + qb);
            hh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bh, hh, 0, 0, 0);
            xx = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bl, xx, 0, 0, 0);
            xx = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bh, xx, 0, 0, 0);
            ll = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bl, ll, 0, 0, 0);
        }
        if (valid) {
            // 128 (sum a + sum_window b) - 128^2 L; the b window starts at 16 (cb - n0)
            const int d = cb - n0;
            const int sb = rsum[4 * rowb] - (d > 0 ? rsum[4 * rowb + d] : 0);
            const int64_t corr = 128 * ((int64_t)rsum[4 * rowa] + sb) - (int64_t)16384 * 64 * NB;
            int64_t *dst = sm.scores + sidx<KEYGRID>(f, p, S, P, K);
            constexpr int KS = KEYGRID ? 4 : 1;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int sl = 16 * d + 4 * g + e;
                if (sl >= -S && sl <= S)
                    dst[KS * sl] = (int64_t)hh[e] * 65536 + (int64_t)xx[e] * 256 + (int64_t)ll[e] + corr;
            }
        }
    }
    __syncthreads();
    DIAG_STAMP(3);
    if constexpr (KEYGRID && EMA && MF_EMA_LATE_TABLES) {
        // the streaming kernel requests its grid tables here, after the xcorr,
        // and waits for them before the batch's first output store: held from
        // the kernel's start they spilled at the 80-VGPR cap, and the reloads
        // after the EMA stores waited for the stores' acknowledgements
        grid_tables();
#pragma unroll
        for (int r = 0; r < GR; r++)
            asm volatile("" : "+v"(gq[r]), "+v"(gc[r]));
    }
    argmax_prior_mf<KEYGRID>(kp, sm.scores, sm.best, reinterpret_cast<const float *>(smem + tb.prior), out, f0, nf);
    DIAG_STAMP(4);
    // streaming: the EMA of the gated frames replaces their scores in LDS, and
    // only gated frames are solved
    uint32_t omask = 0xFFFFFFFFu;
    if constexpr (EMA)
        omask = ema_mf<KEYGRID>(kp, ef, epre, sm.scores, sm.best,
                                reinterpret_cast<float *>(smem + tb.red + 16 * 4 * 8), f0, nf);
    // grid solve (vga_heatmap.h:99-108) on the weighted scores still in LDS:
    // no [B][P][K] round trip through HBM and no second launch
    if (do_grid) {
        if constexpr (KEYGRID)
        {
            uint64_t *red = reinterpret_cast<uint64_t *>(smem + tb.red);
            if (kp.P == 3)
                grid_mf<GR, 3>(kp, sm.scores, red, gq, gc, out, f0, nf, omask);
            else
                grid_mf<GR, 0>(kp, sm.scores, red, gq, gc, out, f0, nf, omask);
        }
        else
            grid_phase_t<int64_t, 4, TWC>(kp, sm.scores, sm.redv, sm.redi, out, f0, nf, nullptr, nullptr, omask);
    }
    DIAG_STAMP(5);
    DIAG_RT(12);
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
        if (bu < 0 || bu >= kp.U)
            bu = 0;
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
                                                    int log2n, int16_t *__restrict__ s1,
                                                    int16_t *__restrict__ s2)
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
            if (s1) {  // the next two ops of the frame path on this output (ops 1, 2 below)
                const int16_t y1 = (int16_t)(uint16_t)(((uint32_t)(uint16_t)y << 8) & 0xFFFFu);
                s1[i] = y1;
                s2[i] = (int16_t)(uint16_t)((uint32_t)(((int32_t)y1 * (int32_t)window[i]) >> 15) & 0xFFFFu);
            }
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

// workgroup shape of k_direct_mfma: F frames per workgroup (one wave per
// (frame, pair) up to 16 waves) and the 16-B staging chunks per thread.  The
// streaming EMA launch (ema) caps the workgroup at 8 waves (its waves loop over
// the F P (frame, pair) units): config 5's 12-wave workgroups ran 2 per CU, 512
// at once, for a batch of ~850 -- two generations, the second two-thirds full;
// at 8 waves, 3 per CU (768 at once).  TDOA_EMA_WAVES=12 keeps the old shape.
static void mf_shape(const tdoa_kparams &kp, int &F, int &threads, int &chunks, bool ema = false)
{
    static const int ema_waves = [] {
        const char *e = getenv("TDOA_EMA_WAVES");
        return e ? atoi(e) : 8;
    }();
    F = kp.P >= 16 ? 1 : 16 / kp.P > 4 ? 4 : 16 / kp.P;
    int w = F * kp.P < 16 ? F * kp.P : 16;
    if (ema && ema_waves > 0 && w > ema_waves)
        w = ema_waves;
    threads = 64 * w;
    chunks = (F * kp.M * kp.N / 8 + threads - 1) / threads;
}

// the matrix-core kernel (config 2..4 shapes) runs the grid solve itself; a
// shape whose frames exceed its staging registers (e.g. 2 mics x 4096: one
// wave per frame holds 16 chunks per thread) takes the VALU k_direct and the
// separate grid launch
bool tdoa_direct_fused_grid(const tdoa_kparams &kp)
{
    if (!(kp.N % 64 == 0 && kp.N >= 64 && kp.S <= 63))
        return false;
    int F, threads, chunks;
    mf_shape(kp, F, threads, chunks);
    return chunks <= 8;
}

// ... and can also run the streaming EMA (k_direct_mfma<.., EMA>): the
// workgroup's stream states fit its prefetch registers
bool tdoa_direct_ema_fits(const tdoa_kparams &kp)
{
    if (!tdoa_direct_fused_grid(kp))
        return false;
    int F, threads, chunks;
    mf_shape(kp, F, threads, chunks, true);
    // (threads a multiple of the row's chunks: stage_mf's shared window chunk)
    return chunks <= 8 && F * kp.P * kp.K <= EMA_E * threads && threads % (kp.N / 8) == 0;
}

int tdoa_launch_direct(const tdoa_kparams &kp_in, const tdoa_kout &out, const int16_t *frames,
                       int64_t B, bool prepared, void *stream, int *lds_bytes_out,
                       const int32_t *count_dev, const tdoa_stream_fuse *ema)
{
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    tdoa_kparams kp = kp_in;
    int threads = 0;
    if (tdoa_direct_fused_grid(kp)) {
        const int n0 = (kp.S + 15) / 16, nq = n0 + (kp.S + 1 + 15) / 16;  // lag columns -16 n0 .. 16 (nq - n0) - 1
        kp.PADW = MF_PADW;
        // (frame, first mic) xcorr units at three mics (k_direct_mfma); TDOA_DIRECT_XC3=0: one unit per pair
        static const bool xc3_off = [] {
            const char *e = getenv("TDOA_DIRECT_XC3");
            return e && e[0] == '0';
        }();
        kp.xc3 = kp.M == 3 && 2 * nq <= 16 && !xc3_off ? 1 : 0;
        kp.RS = kp.N / 2 + 2 * MF_PADW;
        int chunks = 0;
        mf_shape(kp, kp.F, threads, chunks, ema != nullptr);
        MfTabs tb;
        size_t o = smem_bytes(kp, threads / 64);
        tb.rsum = (int)o;
        o += (size_t)16 * kp.F * kp.M;
        tb.prior = (int)o;
        o += (size_t)128 * 4;
        tb.red = (int)o;
        o += (size_t)16 * 4 * 8 + 16 * 4;  // + the EMA's per-frame decay (ema_mf)
        // the keyed grid (TWC = 1): single-word tuples, <= 4 per thread held in
        // registers, the score table frame-interleaved for four frames, cells in
        // the key's 16 index bits; other shapes (wide geometries with more
        // tuples, grids beyond 65536 cells) take the generic grid
        const bool keyed = kp.TW == 1 && kp.U <= (ema ? MF_GR_EMA : MF_GR) * threads && kp.F == 4 && kp.G <= 65536;
        const size_t lds = (o + 15) & ~(size_t)15;
        if (lds > 160 * 1024)
            return tdoa_set_error(-1, "DIRECT: shape needs more than 160 KiB LDS per workgroup");
        if (lds_bytes_out)
            *lds_bytes_out = (int)lds;
        const int64_t grid = (B + kp.F - 1) / kp.F;
        if (grid > INT_MAX)
            return tdoa_set_error(-1, "DIRECT: batch too large for one launch");
        hipStream_t st = (hipStream_t)stream;
        // A/B library only, a measurement: TDOA_DIRECT_RESGRID=1 launches the
        // streaming EMA kernel on the resident workgroups only -- what the
        // launch's empty workgroups (one per possible batch; ~3.4 k of 16384
        // streams trigger at config 5) cost.  Wrong once a hop triggers more
        // frames than the grid holds, so never in the product
        auto dev_grid = [&](const void *fn) -> unsigned {
#if TDOA_AB
            static const bool res_grid = [] {
                const char *e = getenv("TDOA_DIRECT_RESGRID");
                return e && *e && e[0] != '0';
            }();
            if (res_grid && count_dev) {
                const int res = tdoa_resident_blocks(fn, threads, lds);
                return (unsigned)(res > 0 && res < grid ? res : grid);
            }
#endif
            (void)fn;
            return (unsigned)grid;
        };
        constexpr int TWX = (TDOA_MAX_PAIRS + 3) / 4;
        const tdoa_stream_fuse ef = ema ? *ema : tdoa_stream_fuse{};
        if (ema && (!count_dev || prepared))
            return tdoa_set_error(-1, "DIRECT: the EMA launch takes a device-sized batch of raw frames");
        if (ema && (kp.F * kp.P * kp.K > EMA_E * threads || threads % (kp.N / 8) != 0))
            return tdoa_set_error(-1, "DIRECT: EMA state of a workgroup exceeds its prefetch registers");
#define TDOA_LAUNCH_MF(PREP, TWC, CH)                                                                          \
    do {                                                                                                       \
        if (ema) {                                                                                             \
            const void *fn = (const void *)k_direct_mfma<PREP, TWC, CH, !PREP>;                                \
            hipLaunchKernelGGL((k_direct_mfma<PREP, TWC, CH, !PREP>), dim3(dev_grid(fn)), dim3(threads), lds,  \
                               st, kp, out, frames, B, count_dev, n0, nq, tb, ef);                             \
        } else                                                                                                 \
            hipLaunchKernelGGL((k_direct_mfma<PREP, TWC, CH, false>), dim3((unsigned)grid), dim3(threads),     \
                               lds, st, kp, out, frames, B, count_dev, n0, nq, tb, ef);                        \
    } while (0)
#define TDOA_LAUNCH_MF_CH(PREP, TWC)      \
    do {                                  \
        if (chunks <= 2)                  \
            TDOA_LAUNCH_MF(PREP, TWC, 2); \
        else if (chunks == 3)             \
            TDOA_LAUNCH_MF(PREP, TWC, 3); \
        else if (chunks <= 4)             \
            TDOA_LAUNCH_MF(PREP, TWC, 4); \
        else                              \
            TDOA_LAUNCH_MF(PREP, TWC, 8); \
    } while (0)
        if (keyed) {
            if (prepared)
                TDOA_LAUNCH_MF_CH(true, 1);
            else
                TDOA_LAUNCH_MF_CH(false, 1);
        } else {
            if (prepared)
                TDOA_LAUNCH_MF_CH(true, TWX);
            else
                TDOA_LAUNCH_MF_CH(false, TWX);
        }
#undef TDOA_LAUNCH_MF_CH
#undef TDOA_LAUNCH_MF
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "k_direct_mfma launch");
    }
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
#define TDOA_LAUNCH_DIRECT(PREP, TWC)                                                       \
    hipLaunchKernelGGL((k_direct<PREP, TWC>), dim3((unsigned)grid), dim3(threads), lds, st, kp, \
                       out, frames, B, count_dev)
    if (kp.TW == 1) {
        if (prepared)
            TDOA_LAUNCH_DIRECT(true, 1);
        else
            TDOA_LAUNCH_DIRECT(false, 1);
    } else {
        if (prepared)
            TDOA_LAUNCH_DIRECT(true, 7);
        else
            TDOA_LAUNCH_DIRECT(false, 7);
    }
#undef TDOA_LAUNCH_DIRECT
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

int tdoa_launch_ref_buffer(int op, int16_t *buf, const int16_t *ring, int head, int64_t *power,
                           const int16_t *window, int n, void *stream, int16_t *s1, int16_t *s2)
{
    int log2n = 0;
    while ((1 << log2n) < n)
        log2n++;
    hipLaunchKernelGGL(k_ref_buffer, dim3(1), dim3(256), 0, (hipStream_t)stream, op, buf, ring,
                       head, power, window, n, log2n, s1, s2);
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
