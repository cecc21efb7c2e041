/*
 * tdoa_host.c -- plain-C host for libtdoa.
 *
 * Part 1 replays the reference's protothread_sample_and_compute
 * (src/sample_compute.h:45-150) without protothreads or Pico hardware: a
 * synthetic 3-mic source stands in for the ADC/DMA bytes
 * (dma_sample_array, dma_sampler.c:3,17-20), and every call goes to the
 * reference-named entry points exported by libtdoa (tdoa_reference_abi.h):
 *   rolling_buffer_* -> trigger (sample_compute.h:62-99)
 *   write_out / normalize / window / correlations_init (GPU)   (:105-122)
 *   gate, correlations_average (GPU)                           (:124-139)
 *
 * Part 2 runs the batched API (tdoa.h) on a device-resident batch.
 *
 *   gcc -O2 -I../../include tdoa_host.c -L../tdoa -ltdoa -Wl,-rpath,... -lamdhip64
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "tdoa.h"
#include "tdoa_reference_abi.h"

/* sample_compute.h:21: POWER_THRESHOLD = 2 << (2 * BUFFER_HALF_SIZE_BITS) */
#define POWER_THRESHOLD (((power_t)2) << 18)

/* deterministic us clock advanced by the sample loop (20 us per sample) */
static absolute_time_t g_now = 1000000;
static absolute_time_t host_clock(void) { return g_now; }

/* xorshift + Box-Muller */
static uint64_t g_rng = 0x5EED0001ull;
static double urand(void)
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return ((g_rng >> 11) + 0.5) / 9007199254740992.0;
}
static double nrand(void) { return sqrt(-2.0 * log(urand())) * cos(6.283185307179586 * urand()); }

/* A quiet room, then a 700-sample broadband burst reaching mic j delayed by
 * tau[j].  The reference's trigger (sample_compute.h:89) fires once the burst
 * sits in the ring's older half and the newer half has gone quiet. */
static void synth_samples(long t, const int tau[3], long burst_at, uint8_t out[3])
{
    static double src[1 << 16];
    static int init = 0;
    if (!init) {
        for (int i = 0; i < (1 << 16); i++)
            src[i] = nrand();
        init = 1;
    }
    for (int m = 0; m < 3; m++) {
        double v = 128.0 + 0.5 * nrand();
        long u = t - tau[m] - burst_at;
        if (u >= 0 && u < 700)
            v += 40.0 * src[u & 0xFFFF];
        v = v < 0 ? 0 : v > 255 ? 255 : v;
        out[m] = (uint8_t)lrint(v);
    }
}

static int fail_hip(const char *what, int rc)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, tdoa_last_error());
    return 1;
}

int main(void)
{
    tdoa_ref_set_clock(host_clock);
    microphones_init();
    printf("mics: A(%.6f, %.6f) B(%.6f, %.6f) C(%.6f, %.6f)\n", mic_a_location.x,
           mic_a_location.y, mic_b_location.x, mic_b_location.y, mic_c_location.x,
           mic_c_location.y);

    /* ---- part 1: the reference loop, one trigger at a time ---- */
    static struct rolling_buffer_t rb[3];
    static struct buffer_t buf[3];
    static struct correlations_t corr[3], fresh[3];
    const int taus[3][3] = {{0, 5, 9}, {0, -7, 3}, {0, 12, -4}};
    long t = 0;
    for (int ev = 0; ev < 3; ev++) {
        for (int m = 0; m < 3; m++)
            rolling_buffer_init(&rb[m]);
        const long burst_at = t + 3000;
        int triggered = 0;
        for (long guard = 0; guard < 20000; guard++, t++) {
            uint8_t s[3];
            synth_samples(t, taus[ev], burst_at, s);
            for (int m = 0; m < 3; m++)
                rolling_buffer_push(&rb[m], (sample_t)s[m]);
            if (rb[0].is_full && rb[1].is_full && rb[2].is_full) {
                power_t out = 0, in = 0;
                for (int m = 0; m < 3; m++) {
                    out += rolling_buffer_get_outgoing_power(&rb[m]);
                    in += rolling_buffer_get_incoming_power(&rb[m]);
                }
                if (out > POWER_THRESHOLD + in) {
                    triggered = 1;
                    break;
                }
            }
            g_now += 20; /* SAMPLE_PERIOD_US */
        }
        if (!triggered) {
            printf("event %d: no trigger\n", ev);
            continue;
        }
        for (int m = 0; m < 3; m++) {
            rolling_buffer_write_out(&rb[m], &buf[m]);
            buffer_normalize_range(&buf[m]);
            buffer_window(&buf[m]);
        }
        correlations_init(&fresh[0], &buf[0], &buf[1]);
        correlations_init(&fresh[1], &buf[0], &buf[2]);
        correlations_init(&fresh[2], &buf[1], &buf[2]);
        const int ab = fresh[0].best_shift, ac = fresh[1].best_shift, bc = fresh[2].best_shift;
        const int gate = ab * ab + ac * ac + bc * bc > 4;
        if (gate)
            for (int p = 0; p < 3; p++)
                correlations_average(&corr[p], &fresh[p]);
        printf("event %d: trigger at t=%ld  lags ab=%d ac=%d bc=%d (injected %d %d %d)  gate=%d  "
               "avg best %d %d %d\n",
               ev, t, ab, ac, bc, taus[ev][1], taus[ev][2], taus[ev][2] - taus[ev][1], gate,
               corr[0].best_shift, corr[1].best_shift, corr[2].best_shift);
        t += 5000;
        g_now += 100000;
    }

    /* ---- part 2: batched API, device-resident frames ---- */
    tdoa_config cfg;
    tdoa_config_default(&cfg);
    cfg.engine = TDOA_ENGINE_GCC_PHAT;
    tdoa_ctx *ctx = NULL;
    int rc = tdoa_create(&cfg, 0, &ctx);
    if (rc)
        return fail_hip("tdoa_create", rc);
    const int B = 1024, M = 3, N = 1024, P = 3;
    int16_t *h = (int16_t *)malloc(sizeof(int16_t) * B * M * N);
    int32_t *lags = (int32_t *)malloc(sizeof(int32_t) * B * P);
    static double src[1024 + 64];
    for (int b = 0; b < B; b++) {
        const int d[3] = {0, (b % 31) - 15, (b % 19) - 9};
        for (int u = 0; u < N + 64; u++)
            src[u] = nrand();
        for (int m = 0; m < M; m++)
            for (int n = 0; n < N; n++) {
                double v = 128.0 + 40.0 * src[n + 32 - d[m]] + 4.0 * nrand();
                v = v < 0 ? 0 : v > 255 ? 255 : v;
                h[((size_t)b * M + m) * N + n] = (int16_t)lrint(v);
            }
    }
    int16_t *d_frames = NULL;
    int32_t *d_lags = NULL;
    float *d_xy = NULL;
    if (hipMalloc((void **)&d_frames, sizeof(int16_t) * B * M * N) != hipSuccess ||
        hipMalloc((void **)&d_lags, sizeof(int32_t) * B * P) != hipSuccess ||
        hipMalloc((void **)&d_xy, sizeof(float) * B * 2) != hipSuccess)
        return fail_hip("hipMalloc", -4);
    hipMemcpy(d_frames, h, sizeof(int16_t) * B * M * N, hipMemcpyHostToDevice);
    tdoa_outputs o;
    memset(&o, 0, sizeof o);
    o.lags = d_lags;
    o.xy = d_xy;
    rc = tdoa_localize_batch(ctx, d_frames, B, &o, NULL);
    if (rc)
        return fail_hip("tdoa_localize_batch", rc);
    hipMemcpy(lags, d_lags, sizeof(int32_t) * B * P, hipMemcpyDeviceToHost);
    int ok = 0;
    for (int b = 0; b < B; b++) {
        const int d1 = (b % 31) - 15, d2 = (b % 19) - 9;
        ok += lags[b * P] == d1 && lags[b * P + 1] == d2 && lags[b * P + 2] == d2 - d1;
    }
    printf("batched GCC-PHAT: %d/%d frames recovered all three injected lags\n", ok, B);
    hipFree(d_frames);
    hipFree(d_lags);
    hipFree(d_xy);
    free(h);
    free(lags);
    tdoa_destroy(ctx);
    return ok > B * 9 / 10 ? 0 : 2;
}
