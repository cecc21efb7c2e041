/* Host platform layer: one host thread plays core 0. */
#pragma once
static inline unsigned int get_core_num(void) { return 0; }
