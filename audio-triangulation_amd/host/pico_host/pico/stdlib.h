/* Host platform layer: the pico/stdlib.h subset sample_compute.h uses. */
#pragma once
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <hardware/uart.h>
#include <pico/time.h>

typedef unsigned int uint;

static inline void gpio_put(uint pin, bool value) { (void)pin; (void)value; }  /* scope probe */
