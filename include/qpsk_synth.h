/*
 * qpsk_synth.h -- synthetic multi-channel input for benchmarks and tests.
 *
 * Channel c is the reference transmitter's packet stream (src/qpsk.c:380-413:
 * 128-symbol preamble at half amplitude, 8 x 31 QPSK data symbols, 903 zero
 * samples; TX filter/phase state carried across packets) with the dibits and a
 * leading delay d_c in [0, 2783) drawn from splitmix64(seed ^ c*0x9E3779B97F4A7C15),
 * truncated to nsamples.  ebn0_db < 100 adds white Gaussian noise of variance
 * 1.25 * P_data / 10^(EbN0/10) (P_data = 5.19e7, the data-section mean square),
 * rounded and saturated to int16.
 */
#pragma once
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Explicit transmitter state: tx_filter (src/qpsk.c:39), fbb_tx_phase (:47). */
typedef struct {
    float fir_mem[49][2];
    float phase[2];
} qpsk_tx_state;

void qpsk_tx_state_init(qpsk_tx_state *st);
/* qpsk_tx_frame (src/qpsk.c:278) on an explicit state; sym = re/im pairs. */
int qpsk_tx_frame_state(qpsk_tx_state *st, int16_t out[], const float *sym, int length,
                        bool preamble);

/* out [nch][nsamples] for channels c0 .. c0+nch-1, nthreads host threads. */
void qpsk_synth_batch(uint64_t seed, uint32_t c0, int nch, double ebn0_db, int16_t *out,
                      long nsamples, int nthreads);

/* The same streams generated on the GPU into device memory d_out [nch][nsamples]
 * (current HIP device), enqueued on `stream` (hipStream_t, NULL = default).
 * Noiseless output is identical to qpsk_synth_batch(); with noise the
 * Box-Muller transcendentals are the device libm's (tests/test_gpu_synth.py
 * compares).  Returns 0, -1 (bad argument), -2 (host allocation) or
 * -1000 - hipError_t.  Blocks until the host-built phase table is uploaded. */
int qpsk_synth_device(uint64_t seed, uint32_t c0, int nch, double ebn0_db, int16_t *d_out,
                      long nsamples, void *stream);
/* Carrier phase (re, im) of transmitted samples 0 .. ntx-1 of every channel
 * (the transmitter's call sequence is the same for all channels). */
void qpsk_tx_phase_table(float *out2, long ntx);

#ifdef __cplusplus
}
#endif
