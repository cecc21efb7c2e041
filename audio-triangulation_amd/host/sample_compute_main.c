/*
 * sample_compute_main.c -- the reference's own sample loop, UNCHANGED, on the
 * host: this file includes the reference's src/sample_compute.h as it stands
 * (protothread_sample_and_compute, sample_compute.h:45-150) and links its
 * component calls -- rolling_buffer_*, buffer_*, correlations_* -- against
 * libtdoa.so (include/tdoa_reference_abi.h), whose write_out / normalize /
 * window / correlations_init / correlations_average run on the GPU.
 *
 * The Pico side the north star replaces is host/pico_host/ (time, gpio,
 * spin locks, UART, FIFO) plus, here, the capture: dma_sample_array (the
 * ADC round robin, dma_sampler.c:17-55) is refilled from a synthetic 3-mic
 * source every time the sample loop waits for its next 20 us deadline, and
 * a host thread plays the VGA thread's hand-off (vga_debug.h:16-36).
 *
 * Build (the reference's headers are needed at compile time only):
 *   gcc -std=gnu11 -Ihost/pico_host -I<reference>/src -I../include \
 *       host/sample_compute_main.c -Ltdoa -ltdoa -lamdhip64 -lm
 * Run: ./sample_compute_host [frames]   (needs a gfx950 GPU)
 *
 * Environment:
 *   TDOA_REF_HOST=1    libtdoa's host path for the per-frame symbols
 *                      (tdoa_ref_set_device(-1): no HIP call, runs without a GPU)
 *   TDOA_REF_LOG=path  at every hand-off, the loop's state as the reference's own
 *                      structs (int64 sample, u64 now_us, then mic_a/b/c_rb,
 *                      buffer_a/b/c, new_corr_ab/ac/bc, corr_ab/ac/bc) for
 *                      tests/test_reference_loop.py to check against the oracle
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <sample_compute.h> /* the reference's file, unchanged */

/* libtdoa's clock hook (tdoa_reference_abi.h): the EMA's get_absolute_time() */
void tdoa_ref_set_clock(absolute_time_t (*now_us)(void));
int tdoa_ref_set_device(int device);

static FILE *g_log;

volatile uint8_t dma_sample_array[3];

/* ---------------------------------------------------------- capture side */
static absolute_time_t g_now = 1000000;
static long g_sample;
static const int g_tau[3] = {0, 5, 9}; /* injected delays: ab = 5, ac = 9, bc = 4 */

static uint64_t g_rng = 0x5EED0001ull;
static double urand(void)
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return ((g_rng >> 11) + 0.5) / 9007199254740992.0;
}
static double nrand(void) { return sqrt(-2.0 * log(urand())) * cos(6.283185307179586 * urand()); }

/* quiet floor with a 700-sample broadband burst every 4000 samples, mic m
 * hearing it tau[m] samples late */
static void capture_next(void)
{
    static double src[1 << 16];
    static int init;
    if (!init) {
        for (int i = 0; i < (1 << 16); i++)
            src[i] = nrand();
        init = 1;
    }
    for (int m = 0; m < 3; m++) {
        const long u = (g_sample - g_tau[m]) % 4000;
        double v = 128.0 + 0.5 * nrand();
        if (u >= 0 && u < 700)
            v += 40.0 * src[(g_sample - g_tau[m]) & 0xFFFF];
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        dma_sample_array[m] = (uint8_t)lrint(v);
    }
    g_sample++;
}

absolute_time_t host_now_us(void) { return g_now; }

void host_wait_until_us(absolute_time_t t)
{
    if (t > g_now)
        g_now = t;
    capture_next(); /* the ADC's next round-robin triple lands */
}

spin_lock_t *host_spin_lock(unsigned int n)
{
    static spin_lock_t locks[32];
    return &locks[n & 31];
}

/* ------------------------------------------------- the VGA thread's hand-off */
static int g_frames, g_want = 8;

static PT_THREAD(protothread_host_consumer(struct pt *pt))
{
    PT_BEGIN(pt);
    while (true) {
        PT_SEM_WAIT(pt, &vga_semaphore);
        g_frames++;
        if (g_log) {
            const int64_t smp = g_sample;
            const uint64_t now = (uint64_t)g_now;
            fwrite(&smp, sizeof smp, 1, g_log);
            fwrite(&now, sizeof now, 1, g_log);
            fwrite(&mic_a_rb, sizeof mic_a_rb, 1, g_log);
            fwrite(&mic_b_rb, sizeof mic_b_rb, 1, g_log);
            fwrite(&mic_c_rb, sizeof mic_c_rb, 1, g_log);
            fwrite(&buffer_a, sizeof buffer_a, 1, g_log);
            fwrite(&buffer_b, sizeof buffer_b, 1, g_log);
            fwrite(&buffer_c, sizeof buffer_c, 1, g_log);
            fwrite(&new_corr_ab, sizeof new_corr_ab, 1, g_log);
            fwrite(&new_corr_ac, sizeof new_corr_ac, 1, g_log);
            fwrite(&new_corr_bc, sizeof new_corr_bc, 1, g_log);
            fwrite(&corr_ab, sizeof corr_ab, 1, g_log);
            fwrite(&corr_ac, sizeof corr_ac, 1, g_log);
            fwrite(&corr_bc, sizeof corr_bc, 1, g_log);
            fflush(g_log);
        }
        printf("frame %d at sample %ld: best shifts ab %d ac %d bc %d (EMA ab %d ac %d bc %d)\n",
               g_frames, g_sample, new_corr_ab.best_shift, new_corr_ac.best_shift,
               new_corr_bc.best_shift, corr_ab.best_shift, corr_ac.best_shift, corr_bc.best_shift);
        if (g_frames >= g_want)
            exit(new_corr_ab.best_shift == 5 && new_corr_ac.best_shift == 9 &&
                         new_corr_bc.best_shift == 4
                     ? 0
                     : 1);
        PT_SEM_SIGNAL(pt, &load_audio_semaphore);
    }
    PT_END(pt);
}

int main(int argc, char **argv)
{
    if (argc > 1)
        g_want = atoi(argv[1]);
    const char *host = getenv("TDOA_REF_HOST");
    if (host && atoi(host) == 1 && tdoa_ref_set_device(-1) != 0)
        return 3;
    const char *log = getenv("TDOA_REF_LOG");
    if (log && !(g_log = fopen(log, "wb")))
        return 4;
    tdoa_ref_set_clock(host_now_us);
    capture_next();
    PT_SEM_INIT(&vga_semaphore, 0);
    PT_SEM_INIT(&load_audio_semaphore, 0);
    pt_add_thread(protothread_sample_and_compute);
    pt_add_thread(protothread_host_consumer);
    pt_schedule_start;
    return 0;
}
