/*
 * ref_trace.c -- TEST INFRASTRUCTURE ONLY (oracle).  Never shipped, never on
 * the product path.
 *
 * Link-time taps (-Wl,--wrap=...) around the UNMODIFIED reference functions so
 * the harness can record per-frame internals of the reference receiver:
 *   train_eq    /root/reference/src/equalizer.c:45  (first call's index = max_index,
 *                                                    match test of src/qpsk.c:117)
 *   qpsk_demod  /root/reference/src/qpsk.c:268      (soft symbol + raw dibit per data_eq)
 * The taps call straight through (__real_*) and only observe, so the reference's
 * arithmetic and control flow are untouched.  The trace state lives in THIS
 * translation unit so that the reference's own static-data layout in qpsk.c
 * (which its decimated_frame overflow depends on) is exactly
 * that of a plain `gcc -O2 src/*.c` build.
 */
#include <complex.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ref_api.h"

float __real_train_eq(complex float in[], int index, float ref);
void __real_qpsk_demod(uint8_t bits[], complex float symbol);

static ref_trace_t *g_tr;       /* current frame's trace record, or NULL */
static int g_train_calls;
static int g_demod_calls;
static char *g_log;             /* DEBUG2 printf capture */
static size_t g_log_cap, g_log_len;

void ref_trace_begin(ref_trace_t *tr) {
    g_tr = tr;
    g_train_calls = 0;
    g_demod_calls = 0;
    if (tr) memset(tr, 0, sizeof(*tr));
}

void ref_trace_end(void) { g_tr = NULL; }

void ref_log_set(char *buf, size_t cap) {
    g_log = buf;
    g_log_cap = cap;
    g_log_len = 0;
    if (buf && cap) buf[0] = 0;
}

/* The reference qpsk.c is compiled with DEBUG2 (src/qpsk.c:1); its one printf
 * (src/qpsk.c:198-199) is routed here so it can be captured as a golden. */
int ref_debug_printf(const char *fmt, ...) {
    va_list ap;
    char line[256];
    va_start(ap, fmt);
    int n = vsnprintf(line, sizeof line, fmt, ap);
    va_end(ap);
    if (g_log && n > 0 && g_log_len + (size_t)n + 1 < g_log_cap) {
        memcpy(g_log + g_log_len, line, (size_t)n + 1);
        g_log_len += (size_t)n;
    }
    return n;
}

/* Observability probe (tests/test_oracle.py::test_window_observable_range_
 * in_the_reference): when set, before a frame's first train_eq -- after the
 * hunt, src/qpsk.c:172-188 -- every entry of decimated_frame[0..289] (the
 * frame's own dec: the next call rewrites [0, 376) from [376, 752)) outside
 * [index + lo, index + hi] is set to NaN.  index is max_index.  This changes
 * the reference's data, never its code: a probe of which entries reach an
 * output, not a trace. */
static int g_poison, g_plo, g_phi;

void ref_poison_set(int on, int lo, int hi) {
    g_poison = on;
    g_plo = lo;
    g_phi = hi;
}

float __wrap_train_eq(complex float in[], int index, float ref) {
    if (g_poison && g_train_calls == 0) {
        const float nan = __builtin_nanf("");
        for (int k = 0; k < 290; k++)
            if (k < index + g_plo || k > index + g_phi) in[k] = CMPLXF(nan, nan);
    }
    float r = __real_train_eq(in, index, ref);
    if (g_tr) {
        if (g_train_calls == 0) g_tr->max_index = index;
        /* src/qpsk.c:117: match iff train_eq(...) * crealf(ref) > 0 */
        if (r * ref > 0.0f) g_tr->matches++;
    }
    g_train_calls++;
    return r;
}

void __wrap_qpsk_demod(uint8_t bits[], complex float symbol) {
    __real_qpsk_demod(bits, symbol);
    if (g_tr && g_demod_calls < 31) {
        g_tr->soft[g_demod_calls][0] = crealf(symbol);
        g_tr->soft[g_demod_calls][1] = cimagf(symbol);
        g_tr->raw_dibit[g_demod_calls] = (uint8_t)((bits[1] << 1) | bits[0]);
    }
    g_demod_calls++;
}
