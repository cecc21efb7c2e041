/*
 * tdoa_oracle.c -- CPU restatement of the reference hot path.
 * TEST INFRASTRUCTURE ONLY (see tdoa_oracle.h for the pinning status).
 *
 * Every function cites the reference file:line whose semantics it restates.
 * Implementation-defined conversions the reference relies on (int64->int16,
 * int->int16 wrap, arithmetic >> of negatives, << of negative int16) are
 * written as explicit two's-complement operations so this file has no UB.
 */
#include "tdoa_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int ilog2(int n)
{
    int b = 0;
    while ((1 << b) < n)
        b++;
    return b;
}

/* Two's-complement narrowing, the GCC meaning of (int16_t)v. */
static inline int16_t wrap16(int64_t v) { return (int16_t)(uint16_t)(uint64_t)v; }

/* Arithmetic right shift (GCC's >> on negative signed values). */
static inline int64_t asr64(int64_t v, int s) { return v >> s; }

/* rolling_buffer.c:43-71 -- the ring is already linearised here
 * (oldest..newest); total is int64, offset = (sample_t)(total >> BITS) i.e. a
 * FLOOR mean, and each sample is (sample_t)(x - offset) with int16 wrap. */
void orc_dc_remove(const int16_t *in, int16_t *out, int n, int64_t *power)
{
    const int bits = ilog2(n);
    int64_t total = 0;
    for (int i = 0; i < n; i++)
        total += in[i];
    const int16_t off = wrap16(asr64(total, bits));
    int64_t p = 0;
    for (int i = 0; i < n; i++) {
        out[i] = wrap16((int32_t)in[i] - (int32_t)off);
        p += (int64_t)out[i] * out[i];
    }
    if (power)
        *power = p;
}

/* rolling_buffer.c:3-14 */
void orc_ring_init(orc_ring *r, int16_t *storage, int n)
{
    r->head = 0;
    r->incoming_power = r->incoming_total = 0;
    r->outgoing_power = r->outgoing_total = 0;
    r->is_full = 0;
    r->n = n;
    r->buf = storage;
    memset(storage, 0, (size_t)n * sizeof(int16_t));
}

/* rolling_buffer.c:16-41 -- the sample leaving the newer half (at head-N/2)
 * moves into the older half; the sample at head leaves the older half. */
void orc_ring_push(orc_ring *r, int16_t sample)
{
    const int n = r->n, half = n >> 1;
    int mid = r->head - half;
    if (mid < 0)
        mid += n;
    const int64_t m = r->buf[mid];
    const int64_t o = r->buf[r->head];
    r->outgoing_total += m - o;
    r->outgoing_power += m * m - o * o;
    r->incoming_total += (int64_t)sample - m;
    r->incoming_power += (int64_t)sample * sample - m * m;
    r->buf[r->head] = sample;
    if (++r->head >= n) {
        r->head = 0;
        r->is_full = 1;
    }
}

/* rolling_buffer.c:43-62 linearisation then orc_dc_remove (:64-70). */
void orc_ring_write_out(const orc_ring *r, int16_t *dst, int64_t *power)
{
    const int n = r->n;
    int16_t *lin = (int16_t *)malloc((size_t)n * sizeof(int16_t));
    for (int i = 0; i < n; i++)
        lin[i] = r->buf[(r->head + i) % n];
    orc_dc_remove(lin, dst, n, power);
    free(lin);
}

/* rolling_buffer.c:73-85 -- (power << (BITS-1)) - total^2 */
int64_t orc_ring_incoming_power(const orc_ring *r)
{
    const int hb = ilog2(r->n) - 1;
    return (int64_t)((uint64_t)r->incoming_power << hb) - r->incoming_total * r->incoming_total;
}
int64_t orc_ring_outgoing_power(const orc_ring *r)
{
    const int hb = ilog2(r->n) - 1;
    return (int64_t)((uint64_t)r->outgoing_power << hb) - r->outgoing_total * r->outgoing_total;
}

/* buffer.c:13-18 -- `x <<= 8` on int16: only the low byte survives.  The
 * max-abs rescale at buffer.c:20-48 is unreachable (early return). */
void orc_normalize(int16_t *x, int n)
{
    for (int i = 0; i < n; i++)
        x[i] = wrap16((int64_t)(((uint32_t)(uint16_t)x[i]) << 8));
}

/* buffer.c:4-11 -- tmp = (int32)x * W[i]; x = (int16)(tmp >> 15).
 * For N != 1024 the caller passes the DPSS(N, 2) Q15 table of length N
 * (the reference's i << (10 - BITS) indexing is only defined for N <= 1024). */
void orc_window(int16_t *x, const int32_t *w, int n)
{
    for (int i = 0; i < n; i++) {
        const int32_t tmp = (int32_t)x[i] * w[i];
        x[i] = wrap16(tmp >> 15);
    }
}

/* correlations.c:7-24 -- for s = -S..S: score[s] = sum a[i+max(0,-s)] *
 * b[i+max(0,s)] over N-|s| terms in int64; best = first strictly greater. */
void orc_xcorr(const int16_t *a, const int16_t *b, int n, int max_shift,
               int64_t *scores, int32_t *best)
{
    int64_t best_score = INT64_MIN;
    int32_t best_s = -max_shift;
    for (int s = -max_shift; s <= max_shift; s++) {
        const int16_t *p = s < 0 ? a - s : a;
        const int16_t *q = s < 0 ? b : b + s;
        const int cnt = n - (s < 0 ? -s : s);
        int64_t score = 0;
        for (int i = 0; i < cnt; i++)
            score += (int32_t)p[i] * (int32_t)q[i];
        scores[s + max_shift] = score;
        if (score > best_score) {
            best_score = score;
            best_s = s;
        }
    }
    *best = best_s;
}

/* correlations.c:27-30 -- int diff = (s-best)^2; scale = exp(-diff / 36.f):
 * (float)(-diff) / 36.f in float, exp in double, narrowed to float. */
float orc_prior_scale(int d2)
{
    const float arg = (float)(-d2) / 36.f;
    return (float)exp((double)arg);
}

/* correlations.c:26-33 -- score = (int64)((float)score * scale), truncating. */
void orc_prior(int64_t *scores, int max_shift, int best)
{
    for (int s = -max_shift; s <= max_shift; s++) {
        const int d = s - best;
        const float scale = orc_prior_scale(d * d);
        const float v = (float)scores[s + max_shift] * scale;
        scores[s + max_shift] = (int64_t)v;
    }
}

/* correlations.c:40-43 -- dt = (float)(now-last)/1e6f;
 * decay = (float)(1.0 - exp((double)(-dt / 0.5f))). */
float orc_decay(uint64_t now_us, uint64_t last_us)
{
    const float dt = (float)(now_us - last_us) / 1e6f;
    const float arg = -dt / 0.5f;
    return (float)(1.0 - exp((double)arg));
}

/* correlations.c:45-60 -- est += (new-est)*decay as C compound assignment on
 * an int64 lvalue with a float rhs: (int64)((float)est + (float)(new-est)*decay),
 * two separate float roundings (no FMA); then first-max re-argmax. */
void orc_average(int64_t *est, const int64_t *fresh, int K, float decay,
                 int32_t *best)
{
    for (int i = 0; i < K; i++) {
        const int64_t e = est[i];
        const float delta = (float)(fresh[i] - e) * decay;
        const float sum = (float)e + delta;
        est[i] = (int64_t)sum;
    }
    const int S = K / 2;
    int64_t best_score = INT64_MIN;
    int32_t bs = -S;
    for (int s = -S; s <= S; s++) {
        if (est[s + S] > best_score) {
            best_score = est[s + S];
            bs = s;
        }
    }
    *best = bs;
}

/* microphones.c:9-33 with constants.h:17-19,26,28 (AB=.132, BC=.15, CA=.20,
 * MIRROR on, ROTATE off). Output xy = {Ax, Ay, Bx, By, Cx, Cy}. */
void orc_microphones_ref(float xy[6])
{
    const float dAB = 0.132f, dBC = 0.15f, dCA = 0.20f;
    const float xC = (dAB * dAB + dCA * dCA - dBC * dBC) / (2.0f * dAB);
    const float yC = sqrtf(fmaxf(0.0f, dCA * dCA - xC * xC));
    const float ax = 0.0f, ay = 0.0f, bx = dAB, by = 0.0f;
    const float cx_ = xC, cy_ = yC * -1.0f;
    const float cx = (ax + bx + cx_) / 3.0f;
    const float cy = (ay + by + cy_) / 3.0f;
    xy[0] = ax - cx;
    xy[1] = ay - cy;
    xy[2] = bx - cx;
    xy[3] = by - cy;
    xy[4] = cx_ - cx;
    xy[5] = cy_ - cy;
}

/* vga_heatmap.h:11-13 -- sqrtf(x*x + y*y + z*z), left to right, no FMA. */
static inline float hyp3(float x, float y, float z)
{
    return sqrtf(x * x + y * y + z * z);
}

/* vga_heatmap.h:48-93 generalised: pair (i<j) lexicographic, dt = (d_j-d_i)/c,
 * s = (int)roundf(dt * fs) clamped to +-max_shift, idx = s + max_shift. */
void orc_build_lut(const float *mic_xy, int M, int half_w, int half_h,
                   float grid_scale, float height, float speed_of_sound,
                   int fs, int max_shift, uint8_t *lut)
{
    const int W = 2 * half_w + 1, H = 2 * half_h + 1, G = W * H;
    float d[64];
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            float xm = (float)(x - half_w) / grid_scale;
            float ym = (float)(half_h - y) / grid_scale;
            float zm = height;
            const float k = height / hyp3(zm, xm, ym);
            xm *= k;
            ym *= k;
            zm *= k;
            for (int m = 0; m < M; m++)
                d[m] = hyp3(zm, xm - mic_xy[2 * m], ym - mic_xy[2 * m + 1]);
            int p = 0;
            for (int i = 0; i < M; i++)
                for (int j = i + 1; j < M; j++, p++) {
                    const float dt = (d[j] - d[i]) / speed_of_sound;
                    int s = (int)roundf(dt * (float)fs);
                    if (s < -max_shift)
                        s = -max_shift;
                    else if (s > max_shift)
                        s = max_shift;
                    lut[(size_t)p * G + (size_t)y * W + x] = (uint8_t)(s + max_shift);
                }
        }
    }
}

/* vga_heatmap.h:99-108 -- row-major scan, strict '>' keeps the first max. */
void orc_grid_solve(const int64_t *weighted, int P, int K, const uint8_t *lut,
                    int G, int64_t *max_L, int32_t *cell)
{
    int64_t best = INT64_MIN;
    int32_t bc = 0;
    for (int c = 0; c < G; c++) {
        int64_t L = 0;
        for (int p = 0; p < P; p++)
            L += weighted[(size_t)p * K + lut[(size_t)p * G + c]];
        if (L > best) {
            best = L;
            bc = c;
        }
    }
    *max_L = best;
    *cell = bc;
}

/* sample_compute.h:105-134 (write_out -> normalize -> window -> correlate
 * every pair -> gate) + vga_heatmap.h:99-108 on the fresh weighted scores. */
int orc_localize_batch(const int16_t *frames, int64_t B, int M, int N,
                       int max_shift, const int32_t *window, const uint8_t *lut,
                       int half_w, int half_h, float grid_scale, int do_grid,
                       int threads, orc_batch_out *out)
{
    const int P = M * (M - 1) / 2, K = 2 * max_shift + 1;
    const int W = 2 * half_w + 1, G = W * (2 * half_h + 1);
    if (M < 2 || M > 16 || N < 2 * K)
        return -1;
#ifdef _OPENMP
    if (threads > 0)
        omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        int16_t *x = (int16_t *)malloc((size_t)M * N * sizeof(int16_t));
        int64_t *sc = (int64_t *)malloc((size_t)P * K * sizeof(int64_t));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t f = 0; f < B; f++) {
            const int16_t *fr = frames + (size_t)f * M * N;
            for (int m = 0; m < M; m++) {
                int16_t *xm = x + (size_t)m * N;
                orc_dc_remove(fr + (size_t)m * N, xm, N, NULL);
                orc_normalize(xm, N);
                orc_window(xm, window, N);
            }
            int p = 0, gate = 0;
            for (int i = 0; i < M; i++)
                for (int j = i + 1; j < M; j++, p++) {
                    int32_t best;
                    int64_t *s = sc + (size_t)p * K;
                    orc_xcorr(x + (size_t)i * N, x + (size_t)j * N, N, max_shift, s, &best);
                    if (out->scores)
                        memcpy(out->scores + ((size_t)f * P + p) * K, s, K * sizeof(int64_t));
                    orc_prior(s, max_shift, best);
                    if (out->weighted)
                        memcpy(out->weighted + ((size_t)f * P + p) * K, s, K * sizeof(int64_t));
                    out->lags[(size_t)f * P + p] = best;
                    gate += best * best;
                }
            out->gate[f] = gate > 4;
            if (do_grid) {
                int64_t mL;
                int32_t c;
                orc_grid_solve(sc, P, K, lut, G, &mL, &c);
                out->max_L[f] = mL;
                out->cell[f] = c;
                out->xy[2 * f] = (float)(c % W - half_w) / grid_scale;
                out->xy[2 * f + 1] = (float)(half_h - c / W) / grid_scale;
            }
        }
        free(x);
        free(sc);
    }
    return 0;
}

/* sample_compute.h:53-146, one stream at a time (see tdoa_oracle.h). */
int orc_stream_run(const uint8_t *adc, int64_t S, int64_t T, int M, int N, int fs,
                   int max_shift, const int32_t *window, const uint8_t *lut, int half_w,
                   int half_h, int max_trig, int threads, orc_stream_out *out)
{
    const int P = M * (M - 1) / 2, K = 2 * max_shift + 1;
    const int W = 2 * half_w + 1, G = W * (2 * half_h + 1);
    const int hb = ilog2(N) - 1;
    const int64_t thr = (int64_t)2 << (2 * hb); /* POWER_THRESHOLD, sample_compute.h:21 */
    if (M < 2 || M > 16 || N < 2 * K || (N & (N - 1)))
        return -1;
#ifdef _OPENMP
    if (threads > 0)
        omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        int16_t *store = (int16_t *)malloc((size_t)M * N * sizeof(int16_t));
        int16_t *x = (int16_t *)malloc((size_t)M * N * sizeof(int16_t));
        int64_t *sc = (int64_t *)malloc((size_t)P * K * sizeof(int64_t));
        int64_t *est = (int64_t *)malloc((size_t)P * K * sizeof(int64_t));
        int32_t *bst = (int32_t *)malloc((size_t)P * sizeof(int32_t));
        orc_ring *rb = (orc_ring *)malloc((size_t)M * sizeof(orc_ring));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t s = 0; s < S; s++) {
            const uint8_t *a = adc + (size_t)s * T * M;
            int nt = 0;
            uint64_t last = 0;
            memset(est, 0, (size_t)P * K * sizeof(int64_t));
            for (int m = 0; m < M; m++)
                orc_ring_init(&rb[m], store + (size_t)m * N, N);
            for (int64_t t = 0; t < T; t++) {
                int full = 1;
                for (int m = 0; m < M; m++) {
                    orc_ring_push(&rb[m], (int16_t)a[(size_t)t * M + m]);
                    full &= rb[m].is_full;
                }
                if (!full)
                    continue;
                int64_t po = 0, pi = 0;
                for (int m = 0; m < M; m++) {
                    po += orc_ring_outgoing_power(&rb[m]);
                    pi += orc_ring_incoming_power(&rb[m]);
                }
                if (!(po > thr + pi))
                    continue;
                /* triggered after sample t: the frame ends at t + 1 */
                const int64_t end = t + 1;
                const uint64_t now = (uint64_t)end * 1000000u / (uint64_t)fs;
                int gate = 0;
                for (int m = 0; m < M; m++) {
                    int16_t *xm = x + (size_t)m * N;
                    orc_ring_write_out(&rb[m], xm, NULL);
                    orc_normalize(xm, N);
                    orc_window(xm, window, N);
                }
                const size_t r = (size_t)s * max_trig + nt;
                int p = 0;
                for (int i = 0; i < M; i++)
                    for (int j = i + 1; j < M; j++, p++) {
                        int32_t b;
                        orc_xcorr(x + (size_t)i * N, x + (size_t)j * N, N, max_shift,
                                  sc + (size_t)p * K, &b);
                        orc_prior(sc + (size_t)p * K, max_shift, b);
                        if (nt < max_trig)
                            out->lags[r * P + p] = b;
                        gate += b * b;
                    }
                int32_t cell = -1;
                int64_t mL = 0;
                if (gate > 4) {
                    const float decay = orc_decay(now, last);
                    for (p = 0; p < P; p++)
                        orc_average(est + (size_t)p * K, sc + (size_t)p * K, K, decay, &bst[p]);
                    last = now;
                    if (lut)
                        orc_grid_solve(est, P, K, lut, G, &mL, &cell);
                }
                if (nt < max_trig) {
                    out->end[r] = end;
                    out->gate[r] = gate > 4;
                    for (p = 0; p < P; p++)
                        out->ema_best[r * P + p] = gate > 4 ? bst[p] : 0;
                    out->cell[r] = cell;
                    out->max_L[r] = mL;
                }
                nt++;
                for (int m = 0; m < M; m++) /* sample_compute.h:55-57 */
                    orc_ring_init(&rb[m], store + (size_t)m * N, N);
            }
            out->n_trig[s] = nt;
            if (out->est)
                memcpy(out->est + (size_t)s * P * K, est, (size_t)P * K * sizeof(int64_t));
            if (out->last)
                out->last[s] = last;
        }
        free(store);
        free(x);
        free(sc);
        free(est);
        free(bst);
        free(rb);
    }
    return 0;
}

/* a15: see tdoa_oracle.h.  Sub-sample lag of pair p from its raw scores. */
static double ls_tau(const double *s, int K, int best)
{
    const int S = K / 2, kb = best + S;
    double d = 0.0;
    if (kb > 0 && kb < K - 1) {
        const double y0 = s[kb - 1], y1 = s[kb], y2 = s[kb + 1];
        const double den = y0 - 2.0 * y1 + y2;
        if (den < 0.0) {
            d = 0.5 * (y0 - y2) / den;
            d = d < -0.5 ? -0.5 : (d > 0.5 ? 0.5 : d);
        }
    }
    return (double)best + d;
}

void orc_ls_refine(const double *scores, const int32_t *best, int M, int K,
                   const float *mic_xy, int32_t cell, int half_w, int half_h,
                   double grid_scale, double height, double fs, double c, int iters,
                   double *u_out, double *v_out, double *rms_out)
{
    const int P = M * (M - 1) / 2, W = 2 * half_w + 1;
    double tau[64 * 63 / 2];
    for (int p = 0; p < P; p++)
        tau[p] = ls_tau(scores + (size_t)p * K, K, best[p]);
    double u = (double)(cell % W - half_w) / grid_scale;
    double v = (double)(half_h - cell / W) / grid_scale;
    const double lu = (double)half_w / grid_scale, lv = (double)half_h / grid_scale;
    const double h = height, kf = fs / c;
    double ss = 0.0;
    for (int it = 0; it <= iters; it++) {
        /* point on the hemisphere and its derivatives */
        const double n2 = u * u + v * v + h * h, n = sqrt(n2), n3 = n2 * n;
        const double k = h / n;
        const double px = k * u, py = k * v, pz = k * h;
        const double dxu = h * (1.0 / n - u * u / n3), dyu = h * (-v * u / n3), dzu = h * (-h * u / n3);
        const double dxv = h * (-u * v / n3), dyv = h * (1.0 / n - v * v / n3), dzv = h * (-h * v / n3);
        double d[64], du[64], dv[64];
        for (int m = 0; m < M; m++) {
            const double ex = px - (double)mic_xy[2 * m], ey = py - (double)mic_xy[2 * m + 1], ez = pz;
            d[m] = sqrt(ex * ex + ey * ey + ez * ez);
            du[m] = (ex * dxu + ey * dyu + ez * dzu) / d[m];
            dv[m] = (ex * dxv + ey * dyv + ez * dzv) / d[m];
        }
        double a11 = 0.0, a12 = 0.0, a22 = 0.0, g1 = 0.0, g2 = 0.0;
        ss = 0.0;
        int p = 0;
        for (int i = 0; i < M; i++)
            for (int j = i + 1; j < M; j++, p++) {
                const double r = (d[j] - d[i]) * kf - tau[p];
                const double ju = (du[j] - du[i]) * kf, jv = (dv[j] - dv[i]) * kf;
                a11 += ju * ju;
                a12 += ju * jv;
                a22 += jv * jv;
                g1 += ju * r;
                g2 += jv * r;
                ss += r * r;
            }
        if (it == iters)
            break;
        const double lam = 1e-3 * (a11 + a22) + 1e-12;
        const double b11 = a11 + lam, b22 = a22 + lam;
        const double det = b11 * b22 - a12 * a12;
        u -= (b22 * g1 - a12 * g2) / det;
        v -= (b11 * g2 - a12 * g1) / det;
        u = u < -lu ? -lu : (u > lu ? lu : u);
        v = v < -lv ? -lv : (v > lv ? lv : v);
    }
    *u_out = u;
    *v_out = v;
    *rms_out = sqrt(ss / (double)P);
}

/* vga_heatmap.h:97-130: max pass, thresholds (max*63)>>6, (max*31)>>5,
 * (max*15)>>4, (max*7)>>3 (int64, arithmetic shifts), then the class of
 * every cell. */
void orc_heatmap(const int64_t *weighted, int P, int K, const uint8_t *lut, int G,
                 uint8_t *classes)
{
    int64_t hi = INT64_MIN;
    for (int c = 0; c < G; c++) {
        int64_t L = 0;
        for (int p = 0; p < P; p++)
            L += weighted[(size_t)p * K + lut[(size_t)p * G + c]];
        if (L > hi)
            hi = L;
    }
    const int64_t tw = asr64(hi * 63, 6), tg = asr64(hi * 31, 5), tr = asr64(hi * 15, 4),
                  tb = asr64(hi * 7, 3);
    for (int c = 0; c < G; c++) {
        int64_t L = 0;
        for (int p = 0; p < P; p++)
            L += weighted[(size_t)p * K + lut[(size_t)p * G + c]];
        classes[c] = L >= tw ? 4 : L >= tg ? 3 : L >= tr ? 2 : L >= tb ? 1 : 0;
    }
}
