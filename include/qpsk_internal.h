/*
 * qpsk_internal.h -- drop-in replacement of the reference modem surface.
 *
 * Same five prototypes, argument meaning and C linkage as the reference header
 * /root/reference/headers/qpsk_internal.h:79-84 (extern "C" :10-12/86-88).
 * Implemented by libqpsk_hip.so: qpsk_rx_frame() runs the MI355X receive path
 * on a one-channel context, the other four are host C.
 *
 * Added (the reference has no init API; its RX/TX state is set
 * up inside main(), src/qpsk.c:361-368, 375-376, 427-434):
 *   qpsk_rx_init()  -- reset the one-channel receiver to main()'s RX start
 *                      state; also run implicitly by the first qpsk_rx_frame().
 *   qpsk_tx_init()  -- reset the transmitter (tx_filter, fbb_tx_phase).
 *   qpsk_surface_error() -- last HIP error of qpsk_rx_frame (0 = none); the
 *                      reference cannot fail, so qpsk_rx_frame itself keeps the
 *                      1/0 return contract and reports failures here.
 */
#pragma once

/* The reference header's includes (headers/qpsk_internal.h:14-21): a caller
 * written against it may rely on them transitively.  <complex.h> is C only;
 * a C++ caller gets the same layout through float _Complex. */
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifndef __cplusplus
#include <complex.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Constants and helpers of headers/qpsk_internal.h:23-75, same names, values
 * and expression types (CYCLES is an int expression there too). */
#define FINE_TIMING_OFFSET 3
#define TX_FILENAME "/tmp/spectrum-filtered.raw"   /* :25, main()'s TX output */
#define RX_FILENAME "/tmp/databits.txt"            /* :26, main()'s RX records */
#define EOF_COST_VALUE 5.0f
#define EQ_LENGTH 5
#define FS 8000.0f
#define RS 1600.0f
#define TS (1.0f / RS)
#define CYCLES (int)(FS / RS)                      /* 5 */
#define CYCLESF 5
#define CENTER 1100.0f
#define NS 8
#define DATA_SYMBOLS 31
#define FRAME_SYMBOLS (DATA_SYMBOLS * NS)
#define DATA_SAMPLES (DATA_SYMBOLS * CYCLES * NS)
#define DATA_SIZE 1240                             /* DATA_SYMBOLS * NS * CYCLES */
#define FRAME_SIZE 1880                            /* preamble + DATA_SIZE */
#define BITS_PER_FRAME 496                         /* DATA_SYMBOLS * 2 * NS */
#define PREAMBLE_LENGTH 128
#define PREAMBLE_SIZE (PREAMBLE_LENGTH * CYCLESF)
#ifndef M_PI
#define M_PI 3.14159265358979323846f
#endif
#define TAU (2.0f * M_PI)
#define ROT45 (M_PI / 4.0f)
#ifndef __cplusplus
/* e^{+-i x} as cos + i sin (C only: needs complex.h's I) */
#define cmplx(float_value) (cosf(float_value) + sinf(float_value) * I)
#define cmplxconj(float_value) (cosf(float_value) + sinf(float_value) * -I)
#endif

/* receiver state of the reference's driver (:72-75; write-only there) */
typedef enum { hunt, process } RXState;

/* headers/qpsk_internal.h:79 -- |val|^2 (re*re + im*im) */
float cnormf(float _Complex val);
/* headers/qpsk_internal.h:81 (src/qpsk.c:251) -- Gray map bits[index+1]=I, bits[index]=Q */
float _Complex qpsk_mod(uint8_t bits[], int index);
/* headers/qpsk_internal.h:82 (src/qpsk.c:268) -- bits[1] = Re<0 (I), bits[0] = Im<0 (Q) */
void qpsk_demod(uint8_t bits[], float _Complex symbol);
/* headers/qpsk_internal.h:83 (src/qpsk.c:133) -- one 1880-sample frame; returns
 * 1 and writes bits[0..61] on a valid frame, else 0 (bits untouched). */
int qpsk_rx_frame(int16_t in[], uint8_t bits[]);
/* headers/qpsk_internal.h:84 (src/qpsk.c:278) -- length symbols -> length*5
 * int16 samples at 1100 Hz; preamble frames at half amplitude. */
int qpsk_tx_frame(int16_t out[], float _Complex symbol[], int length, bool preamble);

void qpsk_rx_init(void);
void qpsk_tx_init(void);
int qpsk_surface_error(void);

#ifdef __cplusplus
}
#endif
