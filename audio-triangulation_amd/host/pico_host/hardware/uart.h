/* Host platform layer: the UART the protothread serial helpers poll (stdio). */
#pragma once
#include <stdbool.h>
#include <stdio.h>
typedef struct uart_inst uart_inst_t;
#define uart0 ((uart_inst_t *)0)
static inline bool uart_is_readable(uart_inst_t *u) { (void)u; return false; }
static inline bool uart_is_writable(uart_inst_t *u) { (void)u; return true; }
static inline char uart_getc(uart_inst_t *u) { (void)u; return 0; }
static inline void uart_putc(uart_inst_t *u, char c) { (void)u; putchar(c); }
