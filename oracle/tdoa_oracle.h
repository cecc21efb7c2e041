/*
 * tdoa_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * THIS IS THE CHECKER, NOT THE PRODUCT.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path
 * (audio-triangulation_amd/, libtdoa.so) never links or calls it.
 *
 * Restates yuan-xy/Audio-Triangulation's integer/float semantics, generalised
 * to M mics, N samples (power of two), P = M(M-1)/2 pairs, K = 2*max_shift+1:
 *   rolling_buffer.c:3-85   ring, half powers, linearise + floor-mean DC removal
 *   buffer.c:4-18           <<8 (int16 wrap) and Q15 window
 *   correlations.c:4-63     int64 xcorr, first-max argmax, Gaussian prior, EMA
 *   microphones.c:9-33      3-mic law-of-cosines geometry
 *   vga_heatmap.h:48-108    per-cell lag LUT and L = sum_p corr_p[LUT_p] max pass
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - rolling buffer, normalize, window, microphones: pinned bit-exact against
 *     the reference's own buffer.c / rolling_buffer.c / microphones.c compiled
 *     unchanged into oracle/_ref (oracle/Makefile) -- tests/test_oracle_pin.py.
 *   - window tables: pinned against window_function.h:5-70 (N=1024) and the
 *     notebook's stored output window.ipynb:73-202 (N=2048).
 *   - correlations.c / vga_heatmap.h: the reference TUs need Pico SDK headers
 *     (pico/time.h, lib/vga/...) that this image lacks, so they are
 *     UNBUILDABLE here: those stages are "parity unpinned" by reference output
 *     and are checked by an independent numpy restatement plus known-answer
 *     (injected integer delay) cases.
 *
 * Compile with -ffp-contract=off and without -ffast-math: FMA contraction
 * changes correlations_average.
 */
#ifndef TDOA_ORACLE_H
#define TDOA_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- a3: linearised-frame DC removal (rolling_buffer.c:43-71) ---- */
void orc_dc_remove(const int16_t *in, int16_t *out, int n, int64_t *power);

/* ---- rolling ring restatement (rolling_buffer.c:3-85) ---- */
typedef struct orc_ring {
    int head;
    int64_t incoming_power, incoming_total;
    int64_t outgoing_power, outgoing_total;
    int is_full;
    int n;
    int16_t *buf; /* n samples, caller-owned */
} orc_ring;
void orc_ring_init(orc_ring *r, int16_t *storage, int n);
void orc_ring_push(orc_ring *r, int16_t sample);
void orc_ring_write_out(const orc_ring *r, int16_t *dst, int64_t *power);
int64_t orc_ring_incoming_power(const orc_ring *r);
int64_t orc_ring_outgoing_power(const orc_ring *r);

/* ---- a4/a5: buffer.c:13-18 and buffer.c:4-11 ---- */
void orc_normalize(int16_t *x, int n);
void orc_window(int16_t *x, const int32_t *w, int n);

/* ---- a6/a7: correlations.c:4-36 ---- */
void orc_xcorr(const int16_t *a, const int16_t *b, int n, int max_shift,
               int64_t *scores, int32_t *best);
float orc_prior_scale(int d2); /* (float)exp(-d2/36.f)   correlations.c:30 */
void orc_prior(int64_t *scores, int max_shift, int best);

/* ---- a9: correlations.c:38-63 ---- */
float orc_decay(uint64_t now_us, uint64_t last_us);
void orc_average(int64_t *est, const int64_t *fresh, int K, float decay,
                 int32_t *best);

/* ---- a10: microphones.c:9-33 (reference triangle, MIRROR on, ROTATE off) ---- */
void orc_microphones_ref(float xy[6]);

/* ---- a11: vga_heatmap.h:48-93 generalised to M mics, lexicographic pairs ---- */
void orc_build_lut(const float *mic_xy, int M, int half_w, int half_h,
                   float grid_scale, float height, float speed_of_sound,
                   int fs, int max_shift, uint8_t *lut /* [P][H][W] */);

/* ---- a12: vga_heatmap.h:99-108 max pass + argmax extension ---- */
void orc_grid_solve(const int64_t *weighted /* [P][K] */, int P, int K,
                    const uint8_t *lut /* [P][G] */, int G,
                    int64_t *max_L, int32_t *cell);

/* ---- full stateless pipeline over a batch (sample_compute.h:105-134 +
 *      vga_heatmap.h:99-108), OpenMP over frames ---- */
typedef struct orc_batch_out {
    int64_t *scores;   /* [B][P][K] raw, may be NULL */
    int64_t *weighted; /* [B][P][K] after prior, may be NULL */
    int32_t *lags;     /* [B][P] */
    uint8_t *gate;     /* [B] */
    int32_t *cell;     /* [B] */
    int64_t *max_L;    /* [B] */
    float *xy;         /* [B][2] */
} orc_batch_out;

int orc_localize_batch(const int16_t *frames /* [B][M][N] raw */, int64_t B,
                       int M, int N, int max_shift, const int32_t *window,
                       const uint8_t *lut, int half_w, int half_h,
                       float grid_scale, int do_grid, int threads,
                       orc_batch_out *out);

/* ---- a13 + a9 + a12 streaming: sample_compute.h:53-146 for S independent
 *      streams, driven sample by sample from 8-bit round-robin ADC bytes
 *      (dma_sampler.c:17-23, sample_compute.h:67-73).  Per stream: rings
 *      restart empty; after every pushed sample, once full, trigger when
 *      sum_m outgoing > (2 << 2*(log2 N - 1)) + sum_m incoming; the frame
 *      (ring oldest..newest) runs write_out -> normalize -> window -> xcorr
 *      -> prior -> gate; gated frames update the EMA (correlations.c:38-63,
 *      clock now_us = end * 1e6 / fs, end = samples consumed, EMA last = 0
 *      at start) and the grid solve runs on the EMA scores (vga_heatmap.h:
 *      99-108, the VGA thread's corr_*).  Records per trigger, in order. ---- */
typedef struct orc_stream_out {
    int32_t *n_trig;   /* [S] */
    int64_t *end;      /* [S][max_trig] samples consumed at the trigger */
    int32_t *lags;     /* [S][max_trig][P] fresh best lags */
    uint8_t *gate;     /* [S][max_trig] */
    int32_t *ema_best; /* [S][max_trig][P] EMA best lags (gated; else 0) */
    int32_t *cell;     /* [S][max_trig] grid argmax on EMA (gated; else -1) */
    int64_t *max_L;    /* [S][max_trig] */
    int64_t *est;      /* [S][P][K] final EMA state, may be NULL */
    uint64_t *last;    /* [S] final EMA clock, may be NULL */
} orc_stream_out;

int orc_stream_run(const uint8_t *adc /* [S][T][M] */, int64_t S, int64_t T, int M,
                   int N, int fs, int max_shift, const int32_t *window,
                   const uint8_t *lut, int half_w, int half_h, int max_trig,
                   int threads, orc_stream_out *out);

/* ---- f4: vga_heatmap.h:110-130 colouring as classes 4..0 (white, green,
 *      red, blue, black) with the reference's int64 thresholds. ---- */
void orc_heatmap(const int64_t *weighted /* [P][K] */, int P, int K, const uint8_t *lut,
                 int G, uint8_t *classes /* [G] */);

/* ---- a15 (north-star extension, absent in the reference): least-squares
 *      refinement of the grid argmax from sub-sample lags, double precision.
 *      tau_p = best_p + parabolic vertex of the raw scores at best-1..best+1
 *      (0 at the lag-window edges or a non-concave triple, clamped to
 *      +-0.5); model pred_p(u, v) = (d_j - d_i) fs / c with the LUT's
 *      geometry (grid metres (u, v), hemisphere projection of radius h,
 *      vga_heatmap.h:55-65); `iters` Levenberg-Marquardt steps
 *      (lambda = 1e-3 trace(J'J) + 1e-12) from the argmax cell's (u, v),
 *      clamped to the grid.  Outputs (u, v) and the rms lag residual. ---- */
void orc_ls_refine(const double *scores /* [P][K] raw */, const int32_t *best /* [P] */,
                   int M, int K, const float *mic_xy, int32_t cell, int half_w,
                   int half_h, double grid_scale, double height, double fs, double c,
                   int iters, double *u, double *v, double *rms);

#ifdef __cplusplus
}
#endif
#endif
