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

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FINE_TIMING_OFFSET 3
#define EQ_LENGTH 5
#define FS 8000.0f
#define RS 1600.0f
#define CYCLES 5
#define CENTER 1100.0f
#define NS 8
#define DATA_SYMBOLS 31
#define FRAME_SIZE 1880
#define BITS_PER_FRAME 496
#define PREAMBLE_LENGTH 128
#define PREAMBLE_SIZE (PREAMBLE_LENGTH * CYCLES)

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
