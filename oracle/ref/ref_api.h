/*
 * ref_api.h -- TEST INFRASTRUCTURE ONLY (oracle).
 *
 * C interface of oracle/_ref/libqpsk_ref.so: the UNMODIFIED reference receiver
 * (/root/reference/src/*.c compiled by oracle/Makefile) driven one channel at a
 * time.  Used to pin the clean-room restatement (oracle/cpu_ref.c), to generate
 * the golden fixtures under tests/golden/, and as the "reference" CPU baseline
 * leg of bench.py.  Never linked into the product library.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t max_index;      /* first train_eq index  (src/qpsk.c:188 -> :114)        */
    int32_t matches;        /* equalize() result      (src/qpsk.c:188)                */
    int32_t valid;          /* qpsk_rx_frame() return (src/qpsk.c:221/238)            */
    int32_t rx_timing;      /* rx_timing after the frame (src/qpsk.c:219)             */
    float soft[31][2];      /* data_eq soft symbols (either branch, src/qpsk.c:209/228) */
    uint8_t raw_dibit[31];  /* qpsk_demod dibit before descramble                     */
    uint8_t pad[1];
} ref_trace_t;

/* Reset every piece of RX state to what main() establishes before its RX loop
 * (src/qpsk.c:361-368, 427-434, statics zeroed).  Returns 0, or -1 when the
 * static layout is not the gcc -O2 "model A" layout. */
int ref_rx_reset(void);
/* One call of the reference qpsk_rx_frame (src/qpsk.c:133).  bits[62] is
 * zeroed first (the reference leaves it untouched on invalid frames). */
int ref_rx_frame(const int16_t in[1880], uint8_t bits[62], ref_trace_t *tr);
/* Reset, then run nframes frames of one channel. */
int ref_rx_stream(const int16_t *in, int nframes, uint8_t *bits, uint8_t *valid,
                  ref_trace_t *tr);
/* Sequentially demodulate nch independent channels (reset per channel);
 * in [nch][nframes][1880], bits [nch][nframes][62], valid [nch][nframes]. */
int ref_rx_batch(const int16_t *in, int nch, int nframes, uint8_t *bits,
                 uint8_t *valid);

/* decimated_frame[0..289] / input_frame[1880..3759] after the last call. */
void ref_peek_dec(float out[290][2]);
void ref_peek_mixed(float out[1880][2]);

/* Reference TX (src/qpsk.c:278-322) after main()'s TX setup; sym re/im pairs. */
void ref_tx_reset(void);
int ref_tx_frame(int16_t *out, const float *sym, int len, int preamble);

/* Byte distance between decimated_frame and input_frame in this build. */
long ref_layout_gap(void);

/* Observability probe: NaN decimated_frame[0..289] outside [mi + lo, mi + hi]
 * before each frame's equalizer (on != 0), see ref_trace.c. */
void ref_poison_set(int on, int lo, int hi);

void ref_trace_begin(ref_trace_t *tr);
void ref_trace_end(void);
void ref_log_set(char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
