/* Host platform layer: the inter-core FIFO (unused by the sample loop: the
 * reference runs both protothreads on core 0). */
#pragma once
#include <stdbool.h>
#include <stdint.h>
static inline bool multicore_fifo_wready(void) { return true; }
static inline bool multicore_fifo_rvalid(void) { return false; }
static inline void multicore_fifo_push_blocking(uint32_t v) { (void)v; }
static inline uint32_t multicore_fifo_pop_blocking(void) { return 0; }
static inline void multicore_fifo_drain(void) {}
