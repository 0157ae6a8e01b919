/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (oracle).  Never shipped.
 *
 * Compiles the UNMODIFIED reference receiver by #including it from where it
 * lies (REF_QPSK_C = /root/reference/src/qpsk.c, set by oracle/Makefile), with
 * its main() renamed and its DEBUG2 printf captured.  The reference has no
 * init API: ref_rx_reset() re-establishes exactly the state
 * main() sets up before its RX loop (src/qpsk.c:361-368, 427-434) and zeroes
 * the RX statics, so each channel starts as a fresh process would.
 *
 * Nothing in this TU declares static data, so qpsk.c's .bss layout (the
 * decimated_frame -> input_frame overflow) is unchanged;
 * ref_rx_reset() refuses to run if it is not.
 *
 * -DREF_DEC752 (oracle/_ref/libqpsk_ref752.so): the same unmodified sources,
 * linked with oracle/ref/dec752.ld, which places decimated_frame in a section
 * of its own followed by 1,536 zeroed bytes.  The decimation loop's writes
 * past index 561 (src/qpsk.c:157-162, up to index 751) then land in that pad
 * instead of input_frame, and are read back from it on the next call: the
 * program behaves as if the array had the 752 entries the loop assumes
 * ("intended semantics").  No source line changes.
 */
#include <stdio.h>
#include <string.h>
#include <stdint.h>

int ref_debug_printf(const char *fmt, ...);
#define main qpsk_ref_main
#define printf ref_debug_printf
#include REF_QPSK_C
#undef printf
#undef main

#include "ref_api.h"

#ifdef REF_DEC752
/* symbols of oracle/ref/dec752.ld: decimated_frame's end and the pad's end */
extern char ref_dec752_pad[], ref_dec752_end[];

/* addresses as integers behind an asm barrier: the compiler may not fold
 * comparisons between distinct objects */
static uintptr_t addr_of(const void *p) {
    uintptr_t a = (uintptr_t)p;
    __asm__("" : "+r"(a));
    return a;
}

long ref_layout_gap(void) {   /* bytes of owned storage from decimated_frame on */
    return (long)(addr_of(ref_dec752_end) - addr_of(decimated_frame));
}

int ref_rx_reset(void) {
    /* the pad must directly follow the array and cover index 751 */
    if (addr_of(ref_dec752_pad) != addr_of(decimated_frame) + sizeof decimated_frame ||
        ref_layout_gap() < 752 * (long)sizeof(complex float))
        return -1;
    char *p = (char *)decimated_frame;
    __asm__("" : "+r"(p));
    memset(p, 0, (size_t)ref_layout_gap());
    memset(input_frame, 0, sizeof input_frame);
    memset(rx_filter, 0, sizeof rx_filter);
#else
long ref_layout_gap(void) {
    return (long)((const char *)input_frame - (const char *)decimated_frame);
}

int ref_rx_reset(void) {
    if (ref_layout_gap() != 0x11a0) return -1;  /* 562 cf32 + 2 cf32 padding */

    /* zero decimated_frame, the 16 padding bytes after it, and input_frame */
    char *p = (char *)decimated_frame;
    __asm__("" : "+r"(p));
    memset(p, 0, (size_t)ref_layout_gap() + sizeof input_frame);
    memset(rx_filter, 0, sizeof rx_filter);
#endif

    /* src/qpsk.c:361-365 */
    for (size_t i = 0; i < PREAMBLE_LENGTH; i++) {
        float val = (float)preamblevalues[i];
        preambletable[i] = val + (val * I);
    }
    kalman_init();                                       /* src/qpsk.c:367 */
    fbb_rx_phase = cmplx(0.0f);                          /* src/qpsk.c:427 */
    fbb_rx_rect = cmplx(TAU * (-CENTER + FOFFSET) / FS); /* src/qpsk.c:428 */
    state = hunt;                                        /* src/qpsk.c:432 */
    scramble_init(rx);                                   /* src/qpsk.c:434 */
    rx_timing = FINE_TIMING_OFFSET;                      /* src/qpsk.c:53  */
    preamble_frames_detected = 0;
    return 0;
}

int ref_rx_frame(const int16_t in[1880], uint8_t bits[62], ref_trace_t *tr) {
    int16_t frame[FRAME_SIZE];
    uint8_t ibits[BITS_PER_FRAME];
    memcpy(frame, in, sizeof frame);
    memset(ibits, 0, sizeof ibits);
    ref_trace_begin(tr);
    int valid = qpsk_rx_frame(frame, ibits);              /* src/qpsk.c:447 */
    ref_trace_end();
    if (tr) {
        tr->valid = valid;
        tr->rx_timing = rx_timing;
    }
    memcpy(bits, ibits, 62);
    return valid;
}

int ref_rx_stream(const int16_t *in, int nframes, uint8_t *bits, uint8_t *valid,
                  ref_trace_t *tr) {
    if (ref_rx_reset() != 0) return -1;
    int nvalid = 0;
    for (int n = 0; n < nframes; n++) {
        int v = ref_rx_frame(in + (size_t)n * FRAME_SIZE, bits + (size_t)n * 62,
                             tr ? tr + n : NULL);
        if (valid) valid[n] = (uint8_t)v;
        nvalid += v;
    }
    return nvalid;
}

int ref_rx_batch(const int16_t *in, int nch, int nframes, uint8_t *bits,
                 uint8_t *valid) {
    int total = 0;
    for (int c = 0; c < nch; c++) {
        int r = ref_rx_stream(in + (size_t)c * nframes * FRAME_SIZE, nframes,
                              bits + (size_t)c * nframes * 62,
                              valid + (size_t)c * nframes, NULL);
        if (r < 0) return r;
        total += r;
    }
    return total;
}

/* Stage taps for golden fixtures: the reference's own buffers after a call. */
void ref_peek_dec(float out[290][2]) {           /* decimated_frame[0..289] */
    for (int i = 0; i < 290; i++) {
        out[i][0] = crealf(decimated_frame[i]);
        out[i][1] = cimagf(decimated_frame[i]);
    }
}

void ref_peek_mixed(float out[FRAME_SIZE][2]) {  /* input_frame[1880..3759] */
    for (int i = 0; i < FRAME_SIZE; i++) {
        out[i][0] = crealf(input_frame[FRAME_SIZE + i]);
        out[i][1] = cimagf(input_frame[FRAME_SIZE + i]);
    }
}

/* Reference transmitter (src/qpsk.c:278-322) with main()'s TX setup
 * (src/qpsk.c:361-365, 375-376); sym is interleaved re/im. */
void ref_tx_reset(void) {
    memset(tx_filter, 0, sizeof tx_filter);
    for (size_t i = 0; i < PREAMBLE_LENGTH; i++) {
        float val = (float)preamblevalues[i];
        preambletable[i] = val + (val * I);
    }
    fbb_tx_phase = cmplx(0.0f);
    fbb_tx_rect = cmplx(TAU * CENTER / FS);
}

int ref_tx_frame(int16_t *out, const float *sym, int len, int preamble) {
    complex float s[len];
    for (int i = 0; i < len; i++) s[i] = sym[2 * i] + sym[2 * i + 1] * I;
    return qpsk_tx_frame(out, s, len, preamble != 0);
}
