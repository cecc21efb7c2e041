/*
 * tdoa_reference_abi.h -- the per-frame entry points of the reference's DSP
 * components, exported by libtdoa.so with the reference's own names, argument
 * meaning and struct layouts, so that the reference's unchanged
 * src/sample_compute.h links against libtdoa instead of
 * src/components/{rolling_buffer,buffer,correlations,microphones}.c.
 *
 *   symbol                          replaces (reference file:line)
 *   rolling_buffer_init             src/components/rolling_buffer.h:27, .c:3-14
 *   rolling_buffer_push             src/components/rolling_buffer.h:28, .c:16-41
 *   rolling_buffer_write_out        src/components/rolling_buffer.h:29, .c:43-71
 *   rolling_buffer_get_incoming_power  rolling_buffer.h:31, .c:73-78
 *   rolling_buffer_get_outgoing_power  rolling_buffer.h:32, .c:80-85
 *   buffer_window                   src/components/buffer.h:14, buffer.c:4-11
 *   buffer_normalize_range          src/components/buffer.h:15, buffer.c:13-49
 *   correlations_init               src/components/correlations.h:18-21, .c:4-36
 *   correlations_average            src/components/correlations.h:23-25, .c:38-63
 *   microphones_init, mic_*_location src/components/microphones.h:6-10, .c:5-61
 *
 * Where each runs:
 *   - write_out, normalize, window, correlations_init, correlations_average
 *     are the hot path and run as one-frame launches on the GPU (device 0,
 *     or tdoa_ref_set_device); they never fall back to a CPU path -- a HIP
 *     failure prints the reason and aborts, since the reference functions
 *     return void.  Throughput work goes through tdoa.h's batched API.
 *   - tdoa_ref_set_device(-1) explicitly selects libtdoa's own host-CPU
 *     implementation of those five (csrc/tdoa_host_path.cpp, bit-exact, no
 *     HIP call; BASELINE config 1 "on host CPU"); tdoa_ref_set_device(0)
 *     switches back.
 *   - rolling_buffer_init / push / get_*_power are the per-sample capture
 *     ring (the ADC/DMA side, sample_compute.h:62-99) and run on the host.
 *   - microphones_init is one-time geometry and runs on the host.
 *
 * The time source used by correlations_* (pico/time.h get_absolute_time in
 * the reference, correlations.c:35,40) is tdoa_ref_set_clock's callback
 * (default: CLOCK_MONOTONIC in microseconds).
 */
#ifndef TDOA_REFERENCE_ABI_H
#define TDOA_REFERENCE_ABI_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* constants.h:6-7 */
typedef int64_t power_t;
typedef int16_t sample_t;
/* pico/time.h: microseconds since boot (non-opaque form) */
typedef uint64_t absolute_time_t;

#define TDOA_REF_BUFFER_SIZE 1024        /* buffer.h:5-6 */
#define TDOA_REF_MAX_SHIFT 46            /* constants.h:12: 50000*32/34300 */
#define TDOA_REF_CORR_SIZE (2 * TDOA_REF_MAX_SHIFT + 1) /* correlations.h:8 */

struct buffer_t {
    sample_t buffer[TDOA_REF_BUFFER_SIZE];
    power_t power;
};

struct rolling_buffer_t {
    int head;
    power_t incoming_power;
    power_t incoming_total;
    power_t outgoing_power;
    power_t outgoing_total;
    bool is_full;
    sample_t buffer[TDOA_REF_BUFFER_SIZE];
};

struct correlations_t {
    power_t correlations[TDOA_REF_CORR_SIZE];
    int best_shift;
    absolute_time_t last_update;
};

typedef struct {
    float x;
    float y;
} point2d_t;

extern point2d_t mic_a_location;
extern point2d_t mic_b_location;
extern point2d_t mic_c_location;

void microphones_init(void);

void rolling_buffer_init(struct rolling_buffer_t *buf);
void rolling_buffer_push(struct rolling_buffer_t *buf, sample_t sample);
void rolling_buffer_write_out(const struct rolling_buffer_t *buf, struct buffer_t *dst);
power_t rolling_buffer_get_incoming_power(const struct rolling_buffer_t *buf);
power_t rolling_buffer_get_outgoing_power(const struct rolling_buffer_t *buf);

void buffer_window(struct buffer_t *buf);
void buffer_normalize_range(struct buffer_t *buf);

void correlations_init(struct correlations_t *corr, const struct buffer_t *buf_a,
                       const struct buffer_t *buf_b);
void correlations_average(struct correlations_t *estimate, struct correlations_t *new_data);

/* libtdoa extensions for the per-frame shim */
void tdoa_ref_set_clock(absolute_time_t (*now_us)(void));
/* device >= 0: before the first GPU-backed call (or the device in use);
 * device < 0: the host-CPU path, at any time */
int tdoa_ref_set_device(int device);

#ifdef __cplusplus
}
#endif
#endif /* TDOA_REFERENCE_ABI_H */
