// tdoa_internal.h -- layout contract between the host side (tdoa_capi.cpp)
// and the gfx950 kernels (tdoa_kernels.hip).  Not part of the public ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include <hip/hip_runtime.h>

// Lanes of one wave exchanging data through LDS (transpose tiles, score
// tables, staging rows): the wave's DS instructions execute in issue order,
// but the compiler models each lane as a thread of its own and may move one
// lane's LDS write past a later read it cannot prove disjoint.  The wavefront-
// scope release/acquire fences order the memory operations at the IR level
// (they emit no instruction for LDS); the wave barrier between them keeps the
// lanes together (rocPRIM's wave-sync pattern).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The least-squares refinement's sub-sample lag (tdoa_ls.hip, oracle
// orc_ls_refine): the argmax plus the parabolic vertex of the raw scores
// y0, y1, y2 at lags best - 1, best, best + 1, clamped to +-0.5; none at the
// lag range's ends (inside = false) or without a maximum (den >= 0).  One
// definition for k_ls and the kernels that keep the scores on chip, rounded
// as the C oracle (no contraction whatever the TU's flags).
__device__ __forceinline__ double ls_tau3(double y0, double y1, double y2, int best, bool inside)
{
#pragma clang fp contract(off)
    double d = 0.0;
    if (inside) {
        const double den = y0 - 2.0 * y1 + y2;
        if (den < 0.0) {
            d = 0.5 * (y0 - y2) / den;
            d = d < -0.5 ? -0.5 : (d > 0.5 ? 0.5 : d);
        }
    }
    return (double)best + d;
}

// correlations.c:40-43: the EMA decay from the stream clock, in the
// reference's float / double steps (no contraction whatever the TU's flags)
__device__ __forceinline__ float tdoa_decay_dev(uint64_t now, uint64_t last)
{
#pragma clang fp contract(off)
    const float dt = (float)(now - last) / 1e6f;
    const float arg = -dt / 0.5f;
    return (float)(1.0 - exp((double)arg));
}

#define TDOA_MAX_PAIRS 28  // 8 mics
#define TDOA_MAX_MICS_K 8
#define TDOA_LS_ITERS 10   // least-squares refinement steps (tdoa_ls.hip)

// Lag tiling of the DIRECT kernel: each work item owns TDOA_LT consecutive
// lags (an even start lag, so even lags read word-aligned sample pairs and odd
// lags read the one-sample-shifted pairs) over a TDOA_SEGW-word (2*SEGW
// sample) segment of the frame.  SEGW <= 128 keeps every int32 partial of the
// hi/lo byte-split products exact (256 * 32768 * 255 < 2^31).
#define TDOA_LT 16
#define TDOA_LT2 (TDOA_LT / 2)
#define TDOA_SEGW 64

struct tdoa_kparams {
    // shape
    int32_t M, N, log2N, P, K, S;  // S = max_shift, K = 2S+1
    int32_t G, U;                  // grid cells, unique lag tuples
    int32_t grid_W, half_w, half_h;
    float grid_scale;
    // DIRECT tiling
    int32_t sbase;   // first (even) lag of tile 0
    int32_t T;       // lag tiles per pair
    int32_t NSEG;    // segments per frame row (N/2 / SEGW)
    int32_t PADW;    // zero words left/right of every staged row
    int32_t RS;      // staged row stride in words = N/2 + 2*PADW
    int32_t F;       // frames per workgroup
    int32_t TW;      // tuple words per lag tuple = ceil(P/4)
    int32_t xc3;     // k_direct_mfma, three mics: a workgroup's xcorr units are (frame, first mic), the
                     // partners' lag columns side by side in one MFMA tile (0: one unit per pair)
    uint8_t pair_i[TDOA_MAX_PAIRS];
    uint8_t pair_j[TDOA_MAX_PAIRS];
    // device tables
    const int16_t *window;     // [N] Q15
    const float *prior;        // [K] scale by |s - best|
    const uint32_t *tuples;    // [U][TW] packed lag indices (byte p = pair p)
    const int32_t *tuple_cell; // [U] first row-major cell of each tuple
    const float *tw;           // GCC_PHAT: e^{-2 pi i k/N}, k < N   (re, im)
    const float *tw2;          // GCC_PHAT: e^{-2 pi i k/2N}, k <= N (re, im)
    const float *r16_tw;       // GCC_PHAT long frames: [3][16][16] W_N^{(N/256) r k}, W_N^{r l}, W_N^{16 r h}
    const uint8_t *lut;        // [P][G] lag index per cell (heat map)
    const void *p1k_img;       // config-2 GCC-PHAT kernel: its LDS table image (16-B units)
    int32_t p1k_img_bytes;
    const void *w64_img;       // ... and of its one-frame-per-wave form (k_p1k_w64)
    int32_t w64_img_bytes;
    // exact branch-and-bound grid (k_grid_bb): the distinct tuples regrouped
    // by the 8 x 8-cell tile of their first cell (<= 64 tuples per entry);
    // per entry and pair the lag range [lo, hi] of its tuples
    int32_t bb_NT;             // tile entries (0: no table, k_grid only)
    const int32_t *bb_tile;    // [NT][2] first tuple (regrouped order), count
    const uint16_t *bb_rng;    // [NT][P] lo | hi << 8
    const uint32_t *bb_tuples; // [U][TW] regrouped tuples
    const int32_t *bb_uidx;    // [U] their index in first-cell order
    const uint16_t *bb_q;      // [NT][P] the ranges as sparse-table queries (bb_query)
    int32_t bb_wide;           // some range is wider than a query encodes (k_grid instead)
    // compact weighted-score scratch (k_frame16 -> k_grid_bb): per frame only
    // the lags some grid tuple uses, pair p's lags [wc_lo, wc_lo + wc_w) at
    // wc_off[p] (a multiple of 4 floats), wc_CK floats per frame; k_grid_bb
    // expands it in LDS by 16-B chunks: wc_chunks[c] = LDS element of the
    // chunk's first lag (p * K + lag) | valid floats << 16
    int32_t wc_CK, wc_nch;
    uint16_t wc_off[TDOA_MAX_PAIRS];
    uint8_t wc_lo[TDOA_MAX_PAIRS], wc_w[TDOA_MAX_PAIRS];
    const uint32_t *wc_chunks;
    // the grid solve fused into k_frame16 (tdoa_phat_r16.hip, "FG"): every
    // (entry, pair) range of the k_grid_bb tables as a query into sparse-table
    // levels of the compact layout above: e | lv << 11 | d << 13 with e =
    // wc_off[p] + lo - wc_lo[p] the first window's element of level lv
    // (2^lv <= n = hi - lo + 1 < 2^(lv+1); level 0 = the scores) and d = n - 2^lv
    // the second window's distance; rows of 32 (P <= 28 used)
    const uint16_t *fg_q;      // [bb_NT][32]
    const uint16_t *fg_tup;    // [U][32] the regrouped tuples as compact element indices (wc_off + lag - wc_lo)
    int32_t fg_ok;             // the tables exist (n <= 15, wc_CK <= 2048, bb_NT <= 256, P <= 32)
    // DIRECT on the streaming batch read straight from the capture ring (the
    // persistent trigger lists the firing streams and copies nothing): frame f
    // of the batch is stream frame_ids[f]'s samples from ring index
    // frame_ring_at[f] (absolute sample frame_end[f] - N; earlier than the
    // stream's first sample reads as 0); frame_ring null: frame f is frames[f]
    const int32_t *frame_ids;
    const uint8_t *frame_ring;     // [S][ring_len][M] 8-bit ADC bytes, round-robin
    int64_t ring_len;
    const int64_t *frame_end;      // [B] samples consumed at the trigger
    const int64_t *frame_ring_at;  // [B] ring index of the frame's first sample
    // the streaming batch's frames are 8-bit ADC samples ([.][M][N] bytes, the
    // capture ring's values: half the bytes of int16 copies), widened to int16
    // when staged
    int32_t frames_u8;
    // least-squares refinement (tdoa_ls.hip)
    const float *mic_xy;       // [M][2] metres
    float fs, c, height;
};

struct tdoa_kout {
    int32_t *lags;
    uint8_t *gate;
    int32_t *cell;
    float *xy;
    int64_t *max_L;
    float *max_Lf;
    int64_t *scores;
    int64_t *weighted;
    float *scores_f;
    float *weighted_f;
    // per pair the raw scores at lags best - 1, best, best + 1 (the least-
    // squares refinement's parabolic vertex, tdoa_ls.hip): [B][P][3]; written by
    // the kernels that keep the scores on chip (k_frame16) instead of scores_f
    // (slots outside the lag range are not written and not read)
    float *peak3;
    // the compact weighted-score scratch ([B][kp.wc_CK], see tdoa_kparams),
    // written by k_frame16 and read by k_grid_bb in place of weighted_f
    float *weighted_c;
};

// Streaming state of one pipeline (tdoa_stream.hip); all device pointers.
struct tdoa_stream_params {
    int32_t M, N, H, log2N, fs;
    int64_t capture_len;      // samples per stream in the capture ring
    const uint8_t *capture;   // [S][capture_len][M] 8-bit ADC bytes, round-robin
    int64_t *pos;             // [1] samples consumed (device clock)
    int64_t *ring_start;      // [S] sample index of the last trigger (rings restart there)
    int32_t *count;           // [1] frames triggered this step
    int32_t *count_next;      // [1] the next step's counter: zeroed by this step's trigger
                              // (two counters alternate by hop parity: no memset node)
    int32_t *ids;             // [S] compact slot -> stream
    int64_t *end;             // [S] samples consumed at the trigger
    int64_t *ring_at;         // [S] ring index of the slot's first frame sample
                              // (persistent trigger: DIRECT reads the ring)
    int16_t *frames;          // [S][M][N] triggered frames, compact (k_stream_trigger)
    int64_t *fresh;           // [S][P][K] their weighted scores (k_direct)
    int32_t *fresh_lags;      // [S][P]
    uint8_t *fresh_gate;      // [S]
    int64_t *est;             // [S][P][K] EMA scores per stream
    uint64_t *last;           // [S] EMA clock per stream (us)
    int64_t *stats;           // [2] running totals: triggered frames, gated frames
};

struct tdoa_stream_kout {
    int32_t *count;
    int32_t *stream_id;
    int64_t *end;
    int32_t *lags;
    uint8_t *gate;
    int32_t *ema_best;
    int32_t *cell;
    float *xy;
    int64_t *max_L;
};

// Resident workgroups of `kernel` (threads, dynamic LDS) on the current device:
// blocks per CU from the occupancy query x CUs, cached per (device, kernel,
// threads, LDS) under a mutex (contexts on different host threads / devices).
int tdoa_resident_blocks(const void *kernel, int threads, size_t lds);

// Host-side launchers implemented in the .hip files.
// count_dev (optional): device int32 batch size, B then only bounds the grid.
// ema (optional, streaming): the launch also runs the EMA of the gated frames
// and the grid on the EMA scores (k_direct_mfma only: tdoa_direct_fused_grid)
struct tdoa_stream_fuse {
    tdoa_stream_params sp;
    tdoa_stream_kout so;
};
int tdoa_launch_direct(const tdoa_kparams &kp, const tdoa_kout &out,
                       const int16_t *frames, int64_t B, bool prepared,
                       void *stream, int *lds_bytes_out,
                       const int32_t *count_dev = nullptr, const tdoa_stream_fuse *ema = nullptr);
// the DIRECT launch for this shape also solves the grid (k_direct_mfma)
bool tdoa_direct_fused_grid(const tdoa_kparams &kp);
// ... and can also run the streaming EMA (tdoa_stream_fuse)
bool tdoa_direct_ema_fits(const tdoa_kparams &kp);
int tdoa_launch_heatmap(const tdoa_kparams &kp, const void *weighted, const void *max_L,
                        bool is_float, int64_t B, uint8_t *classes, void *stream);
int tdoa_launch_ls(const tdoa_kparams &kp, const void *scores, bool is_float, const float *peak3,
                   const int32_t *lags, const int32_t *cells, float *xy_ls, float *rms,
                   int64_t B, void *stream);
size_t tdoa_stream_trigger_lds(int M, int N, int H);
// *by_id: the launch wrote each triggered frame at its stream's index
// (k_stream_trigger_p) instead of its compact slot -- the layout DIRECT reads
int tdoa_launch_stream_trigger(const tdoa_stream_params &sp, int64_t S, void *stream, bool *by_id);
int tdoa_launch_stream_update(const tdoa_stream_params &sp, const tdoa_kparams &kp,
                              const tdoa_stream_kout &out, int64_t S, void *stream);
int tdoa_launch_average(const tdoa_kparams &kp, int64_t S, int64_t *est,
                        const int64_t *fresh, const float *decay, int32_t *best,
                        const tdoa_kout *solve, void *stream);
int tdoa_launch_grid(const tdoa_kparams &kp, const tdoa_kout &out, const void *weighted,
                     bool is_float, int64_t B, void *stream);
int tdoa_launch_gcc_phat(const tdoa_kparams &kp, const tdoa_kout &out,
                         const int16_t *frames, int64_t B, float phat_eps,
                         void *spec_scratch, size_t spec_bytes, void *stream);
// GCC-PHAT shapes the fused kernels cannot hold (M > 3 or N > 2048): two
// passes per chunk of frames through a spectrum scratch (tdoa_phat_split.hip)
bool tdoa_gcc_phat_needs_split(int M, int N);
// config-2 GCC-PHAT kernel (tdoa_phat1024.hip): host-built LDS table image
// from the twiddles ([N] e^{-2 pi i k/N} then [N+1] e^{-2 pi i k/2N}),
// Q15 window, lag prior and distinct lag tuples with their first cells; empty
// if the shape differs
void tdoa_phat1024_image(int M, int N, int K, int U, const float *tw, const int32_t *win,
                         const float *prior, const uint32_t *tuples, const int32_t *tuple_cell,
                         std::vector<uint8_t> &img);
// the one-frame-per-wave config-2 kernel (tdoa_p1k_w64.hip): its image
void tdoa_p1k_w64_image(int M, int N, int K, int U, const int32_t *win, const float *prior,
                        const uint32_t *tuples, std::vector<uint8_t> &img);
bool tdoa_gcc_phat_fused_grid(const tdoa_kparams &kp);
// the first kernel a GCC-PHAT batch runs for this shape (tdoa_batch_kernel)
const char *tdoa_gcc_phat_kernel_name(const tdoa_kparams &kp);
// the float grid runs k_grid_bb and can read the compact scratch (tdoa_grid.hip)
bool tdoa_grid_bb_compact(const tdoa_kparams &kp);
bool tdoa_gcc_phat_grid_in_kernel(const tdoa_kparams &kp);
bool tdoa_gcc_phat_peak3(const tdoa_kparams &kp);
int tdoa_launch_gcc_phat_split(const tdoa_kparams &kp, const tdoa_kout &out,
                               const int16_t *frames, int64_t B, float eps2_int16,
                               void *scratch, size_t scratch_bytes, void *stream);
