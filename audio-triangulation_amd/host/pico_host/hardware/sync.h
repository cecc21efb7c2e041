/* Host platform layer: hardware spin locks as plain flags (one host thread). */
#pragma once
#include <stdbool.h>
#include <stdint.h>
typedef volatile uint32_t spin_lock_t;
spin_lock_t *host_spin_lock(unsigned int n);
static inline spin_lock_t *spin_lock_init(unsigned int n) { return host_spin_lock(n); }
static inline void spin_lock_unsafe_blocking(spin_lock_t *l) { *l = 1; }
static inline void spin_unlock_unsafe(spin_lock_t *l) { *l = 0; }
static inline bool is_spin_locked(spin_lock_t *l) { return *l != 0; }
