/*
 * tdoa.h -- batched C ABI of the MI355X TDOA localizer (libtdoa.so).
 *
 * The reference (yuan-xy/Audio-Triangulation) processes one 3-mic frame at a
 * time inside protothread_sample_and_compute (src/sample_compute.h:105-139)
 * and solves the position on a 101x101 grid in vga_draw_heatmap
 * (src/components/vga/vga_heatmap.h:95-108).  This header is the batched,
 * error-returning form of that path: one call runs, for B frames at once,
 *
 *   rolling_buffer_write_out DC removal  rolling_buffer.c:64-66
 *   buffer_normalize_range (<<8 wrap)     buffer.c:13-18
 *   buffer_window (Q15 DPSS NW=2)         buffer.c:4-11, window.ipynb:43-60
 *   correlations_init (scores, argmax,    correlations.c:4-36
 *                      Gaussian lag prior)
 *   shift gate sum(best^2) > 4            sample_compute.h:124-134
 *   grid L = sum_p corr_p[LUT_p] max pass vga_heatmap.h:48-108
 *
 * as hand-written gfx950 kernels.  The per-frame reference symbols live in
 * tdoa_reference_abi.h and are implemented on top of this API.
 *
 * Conventions: all pointers in tdoa_outputs and the frames pointer of
 * tdoa_localize_batch are DEVICE pointers on the context's device; `stream`
 * is a hipStream_t (NULL = default stream).  Every function returns
 * TDOA_OK (0) or a negative tdoa_status; tdoa_last_error() describes the
 * last failure on the calling thread.  A context is bound to one device and
 * is not thread-safe: use one context per host thread / GPU.
 */
#ifndef TDOA_H
#define TDOA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDOA_ABI_VERSION 1
#define TDOA_MAX_MICS 8

typedef enum tdoa_status {
    TDOA_OK = 0,
    TDOA_ERR_INVALID = -1,   /* bad argument / config */
    TDOA_ERR_HIP = -2,       /* HIP runtime error (message in tdoa_last_error) */
    TDOA_ERR_NO_DEVICE = -3, /* no gfx950 device visible */
    TDOA_ERR_NOMEM = -4
} tdoa_status;

typedef enum tdoa_engine {
    /* Exact integer time-domain cross-correlation: the reference's
     * correlations_init semantics bit-for-bit (int64 scores). */
    TDOA_ENGINE_DIRECT = 0,
    /* Generalised cross-correlation with PHAT weighting (fp32 radix-4 FFT,
     * |X| normalised cross-spectrum, inverse FFT), the north-star
     * formulation.  Float scores; lags equal DIRECT's on clean integer
     * delays, otherwise checked against a float64 GCC-PHAT oracle. */
    TDOA_ENGINE_GCC_PHAT = 1
} tdoa_engine;

typedef struct tdoa_config {
    int32_t num_mics;        /* M, 2..TDOA_MAX_MICS              (reference: 3) */
    int32_t frame_len;       /* N, power of two 256..4096        (buffer.h:5-6: 1024) */
    int32_t sample_rate_hz;  /* fs                               (constants.h:10: 50000) */
    int32_t max_shift;       /* <= 0 -> fs*32/34300              (constants.h:12: 46) */
    float speed_of_sound;    /* m/s                              (constants.h:14: 343) */
    int32_t engine;          /* tdoa_engine */
    /* mic positions [M][2] in metres; NULL -> microphones_init()'s triangle
     * (microphones.c:9-33) for M == 3, otherwise required. Copied. */
    const float *mic_xy;
    /* grid (vga.h:29-35, vga_heatmap.h:2-3): (2*half_w+1) x (2*half_h+1)
     * cells at grid_scale cells per metre, projected on a hemisphere of
     * radius height_offset. */
    int32_t grid_half_w;     /* 50 */
    int32_t grid_half_h;     /* 50 */
    float grid_scale;        /* 24.0f */
    float height_offset;     /* 1.2f */
    /* Q15 window [N]; NULL -> the reference's table: for N <= 1024 the
     * 1024-point DPSS(NW=2) table (window_function.h) subsampled as
     * buffer.c:8 indexes it, W[i << (10 - log2 N)]; for N > 1024 (where
     * buffer.c:8 is undefined) DPSS(N, NW=2) normalised to max 1, x32767,
     * rounded (window.ipynb procedure).  Copied. */
    const int32_t *window_q15;
    float phat_eps;          /* GCC_PHAT: floor of |X_i^* X_j| (samples scaled by 2^-15), default 1e-12 */
} tdoa_config;

/* Per-frame results (device pointers; any may be NULL unless noted). */
typedef struct tdoa_outputs {
    int32_t *lags;           /* [B][P] best shift per pair (required)       */
    uint8_t *gate;           /* [B] sum_p lag^2 > 4 (sample_compute.h:134)   */
    int32_t *cell;           /* [B] first row-major argmax cell of L         */
    float *xy;               /* [B][2] ((x-hw)/scale, (hh-y)/scale) metres   */
    int64_t *max_L;          /* [B] DIRECT: max of L (vga_heatmap.h:99-108)  */
    float *max_Lf;           /* [B] GCC_PHAT: max of L                       */
    int64_t *scores;         /* [B][P][K] DIRECT raw int64 scores (debug)    */
    int64_t *weighted;       /* [B][P][K] DIRECT scores after the lag prior  */
    float *scores_f;         /* [B][P][K] GCC_PHAT raw correlation (debug)   */
    float *weighted_f;       /* [B][P][K] GCC_PHAT after the lag prior       */
    /* Least-squares refinement of the grid argmax (extension; absent in the
     * reference): sub-sample lags (parabolic vertex of the raw scores) fitted
     * by 10 Levenberg-Marquardt steps in double precision on the LUT's
     * hemisphere geometry, starting at the argmax cell, clamped to the grid. */
    float *xy_ls;            /* [B][2] refined (x, y) metres, grid frame     */
    float *ls_rms;           /* [B] rms lag residual (samples)               */
} tdoa_outputs;

typedef struct tdoa_ctx tdoa_ctx;

/* Fills the reference defaults (3 mics, 1024, 50 kHz, 46, DIRECT, ...). */
int tdoa_config_default(tdoa_config *cfg);

/* Validates cfg, builds the window, mic geometry, lag prior table and the
 * grid LUT on the host, uploads them to `device`. */
int tdoa_create(const tdoa_config *cfg, int device, tdoa_ctx **out);
int tdoa_destroy(tdoa_ctx *ctx);

/* Derived sizes of a context. */
int tdoa_get_dims(const tdoa_ctx *ctx, int32_t *M, int32_t *N, int32_t *P,
                  int32_t *K, int32_t *G);

/* Stateless batch: frames = device int16 [B][M][N] raw (pre-DC) samples, mic
 * rows contiguous.  Asynchronous on `stream`. */
int tdoa_localize_batch(tdoa_ctx *ctx, const int16_t *frames, int64_t B,
                        const tdoa_outputs *out, void *stream);

/* Same as tdoa_localize_batch for frames that already went through DC
 * removal, normalisation and the window (the inputs correlations_init sees).
 * Used by the per-frame reference symbols. */
int tdoa_correlate_prepared(tdoa_ctx *ctx, const int16_t *prepared, int64_t B,
                            const tdoa_outputs *out, void *stream);

/* Temporal averaging (correlations.c:38-63) for S independent streams:
 * est[S][P][K] (device, in/out) <- (int64)((float)est + (float)(fresh-est)*decay[s]),
 * best[S][P] re-argmaxed.  decay (device float[S]) comes from
 * tdoa_decay_us on the host.  If solve is non-NULL the grid solve runs on the
 * averaged scores (the reference solves on corr_*, vga_heatmap.h:102-104). */
int tdoa_average_batch(tdoa_ctx *ctx, int64_t S, int64_t *est,
                       const int64_t *fresh, const float *decay, int32_t *best,
                       const tdoa_outputs *solve, void *stream);

/* Heat-map classes of vga_draw_heatmap's colouring pass (vga_heatmap.h:
 * 110-130) for B frames: classes[B][G] = 4 (white, L >= (max*63)>>6),
 * 3 (green, (max*31)>>5), 2 (red, (max*15)>>4), 1 (blue, (max*7)>>3), else 0,
 * L = sum_p weighted_p[LUT_p].  weighted [B][P][K] and max_L [B] are device
 * int64 (is_float = 0; the reference's integer thresholds) or float
 * (is_float = 1; max * n / 2^b), e.g. a localize call's weighted / max_L
 * outputs or EMA scores with their grid max.  B <= 65535. */
int tdoa_heatmap(tdoa_ctx *ctx, const void *weighted, const void *max_L, int is_float,
                 int64_t B, uint8_t *classes, void *stream);

/* Host helper: decay of correlations.c:42-43 from integer-us timestamps. */
float tdoa_decay_us(uint64_t now_us, uint64_t last_us);

/* Host copies of the context's tables (for tests / tooling). */
int tdoa_get_window(const tdoa_ctx *ctx, int32_t *window /* [N] */);
int tdoa_get_mics(const tdoa_ctx *ctx, float *mic_xy /* [M][2] */);
int tdoa_get_lut(const tdoa_ctx *ctx, uint8_t *lut /* [P][G] */);
int tdoa_get_prior(const tdoa_ctx *ctx, float *scale /* [K] by |d| */);

/* DPSS(N, NW) first Slepian taper, Q15 as in window.ipynb. */
int tdoa_dpss_q15(int32_t n, double nw, int32_t *out);

/* ---- Streaming pipeline (sample_compute.h:53-146; BASELINE config 5) ----
 * S independent mic-array streams whose 8-bit ADC bytes (dma_sampler.c:17-23:
 * one u8 per mic, round-robin; read as sample_t at sample_compute.h:67-73)
 * land in a device capture ring capture[S][capture_len][M].  Each
 * tdoa_stream_step consumes the next `hop` samples of every stream:
 *   trigger   after every sample, once N samples arrived since the stream's
 *             last trigger (the rings restart empty, sample_compute.h:55-57),
 *             fire when sum_m outgoing > 2 << 2(log2 N - 1) + sum_m incoming
 *             (rolling_buffer.c:16-41,73-85; sample_compute.h:75-91), first
 *             firing sample of the hop;
 *   frame     the N samples before it through the DIRECT path (write_out,
 *             normalize, window, xcorr, prior, gate);
 *   EMA       gated frames only: correlations.c:38-63 on the stream's scores
 *             with the clock now_us = end * 1e6 / fs (end = samples consumed
 *             at the trigger; the EMA clock starts at 0 like corr_*'s static
 *             zero init), then the grid solve on the EMA scores (the VGA
 *             thread solves on corr_*, vga_heatmap.h:99-108).
 * The step is a fixed kernel sequence reading its position from a device
 * clock, so with use_graph it is captured once into a hipGraph and replayed.
 * The producer keeps capture_len >= N + 2*hop samples of history per stream.
 * Requires a DIRECT context; hop <= N. */
typedef struct tdoa_stream tdoa_stream;

typedef struct tdoa_stream_outputs { /* device pointers; slot order is arbitrary */
    int32_t *count;     /* [1] frames triggered this step: slots 0..count-1 */
    int32_t *stream_id; /* [S] stream of each slot                           */
    int64_t *end;       /* [S] samples consumed at the trigger (frame = [end-N, end)) */
    int32_t *lags;      /* [S][P] best lags of the fresh frame               */
    uint8_t *gate;      /* [S] sum_p lag^2 > 4                               */
    int32_t *ema_best;  /* [S][P] EMA best lags (gated slots)                */
    int32_t *cell;      /* [S] grid argmax on the EMA scores; -1 if not gated */
    float *xy;          /* [S][2] (gated slots)                              */
    int64_t *max_L;     /* [S] (gated slots)                                 */
} tdoa_stream_outputs;

int tdoa_stream_create(tdoa_ctx *ctx, int32_t num_streams, int32_t hop,
                       const uint8_t *capture, int64_t capture_len, int use_graph,
                       tdoa_stream **out);
/* One hop for every stream, asynchronous on `stream` (graph mode needs a
 * non-NULL stream; the captured graph is reused while `out` and `stream`
 * stay the same). */
int tdoa_stream_step(tdoa_stream *st, const tdoa_stream_outputs *out, void *stream);
/* Back to the start: position 0, rings empty, EMA scores 0, EMA clocks 0. */
int tdoa_stream_reset(tdoa_stream *st, void *stream);
/* Synchronous snapshot: samples consumed, EMA scores [S][P][K], EMA clocks
 * [S] and running totals {triggered, gated} frames [2] (host pointers; any
 * may be NULL). */
int tdoa_stream_state(tdoa_stream *st, int64_t *pos, int64_t *est, uint64_t *last,
                      int64_t *stats);
int tdoa_stream_destroy(tdoa_stream *st);

const char *tdoa_last_error(void);
int tdoa_abi_version(void);
/* Name of the kernel a tdoa_localize_batch call of this context runs first
 * (diagnostics: profile and HBM-traffic attribution); "" if none applies. */
const char *tdoa_batch_kernel(const tdoa_ctx *ctx);
/* 1 if a grid-requesting tdoa_localize_batch of this context solves the grid
 * inside that first kernel (no weighted-score scratch, no separate grid
 * launch), 0 if a grid kernel follows it (diagnostics, like tdoa_batch_kernel). */
int tdoa_batch_grid_fused(const tdoa_ctx *ctx);
/* Measurement: the shader clock (MHz) `device` holds under VALU load -- every
 * CU's waves run FMA chains for about `ms` milliseconds (0 < ms <= 100) on
 * `stream` and compare s_memtime with the 100 MHz s_memrealtime; the median
 * over waves.  Synchronous.  bench.py records it after its timed region so a
 * slow box and a regression can be told apart. */
int tdoa_gpu_clock_mhz(int device, void *stream, double ms, double *mhz);

#ifdef __cplusplus
}
#endif
#endif /* TDOA_H */
