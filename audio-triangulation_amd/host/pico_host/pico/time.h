/* Host platform layer (replaces the Pico SDK on the capture side, as the
 * north star asks): the time API sample_compute.h and correlations.h use
 * (pico/time.h), on a deterministic synthetic sample clock.  busy_wait_until()
 * is where the host's synthetic ADC advances: it loads the next round-robin
 * sample into dma_sample_array (dma_sampler.c:17-55 on the device). */
#pragma once
#include <stdbool.h>
#include <stdint.h>

typedef uint64_t absolute_time_t;

absolute_time_t host_now_us(void);
void host_wait_until_us(absolute_time_t t);

static inline absolute_time_t get_absolute_time(void) { return host_now_us(); }
static inline uint64_t time_us_64(void) { return host_now_us(); }
static inline absolute_time_t delayed_by_us(absolute_time_t t, uint64_t us) { return t + us; }
static inline void busy_wait_until(absolute_time_t t) { host_wait_until_us(t); }
