/*
 * qpsk_surface.c -- the reference's qpsk_internal.h surface (host C).
 *
 *   cnormf, qpsk_mod, qpsk_demod  -- src/qpsk.c:75-80, 251-256, 268-271
 *   qpsk_tx_frame                 -- src/qpsk.c:278-322 (host TX, reference
 *                                    semantics incl. int16 truncation)
 *   qpsk_rx_frame                 -- src/qpsk.c:133-239, run on the MI355X
 *                                    through a one-channel qpsk_ctx
 * The RX and TX state the reference keeps in file statics (src/qpsk.c:37-53)
 * is kept here in the same single-instance form, so existing single-channel
 * callers link unchanged; the batched API (qpsk_batch.h) is the native one.
 * Compiled with -ffp-contract=off: every fp32 op rounds like the reference.
 */
#include <math.h>
#include <string.h>

#include "qpsk_batch.h"
#include "qpsk_consts.h"
#include "qpsk_internal.h"
#include "qpsk_synth.h"

float cnormf(float _Complex val) {
    float re = __real__ val, im = __imag__ val;
    return re * re + im * im;
}

float _Complex qpsk_mod(uint8_t bits[], int index) {
    float _Complex r;
    __real__ r = (bits[index + 1] == 1) ? -1.0f : 1.0f;  /* I - odd bits  */
    __imag__ r = (bits[index] == 1) ? -1.0f : 1.0f;      /* Q - even bits */
    return r;
}

void qpsk_demod(uint8_t bits[], float _Complex symbol) {
    bits[1] = __real__ symbol < 0.0f;  /* I - odd bits  */
    bits[0] = __imag__ symbol < 0.0f;  /* Q - even bits */
}

/* ---------------------------------------------------------------- TX */

void qpsk_tx_state_init(qpsk_tx_state *st) {
    memset(st, 0, sizeof(*st));
    st->phase[0] = 1.0f;   /* fbb_tx_phase = cmplx(0.0f), src/qpsk.c:375 */
}

/* qpsk_tx_frame() body on an explicit state; sym = interleaved re/im */
int qpsk_tx_frame_state(qpsk_tx_state *st, int16_t out[], const float *sym, int length,
                        bool preamble) {
    /* fbb_tx_rect = cmplx(TAU*CENTER/FS), src/qpsk.c:376: float argument */
    const float arg = (float)(2.0f * 3.14159265358979323846 * 1100.0f / 8000.0f);
    const float rr = cosf(arg), ri = sinf(arg);
    const float scale = preamble ? 8192.0f : 16384.0f;
    for (int j = 0; j < length * CYCLES; j++) {
        /* zero-stuffed symbol stream through fir(tx_filter, ...) src/fir.c:29-43 */
        memmove(st->fir_mem[0], st->fir_mem[1], sizeof(float[2]) * (QK_NTAPS - 1));
        if (j % CYCLES == 0) {
            st->fir_mem[QK_NTAPS - 1][0] = sym[2 * (j / CYCLES)];
            st->fir_mem[QK_NTAPS - 1][1] = sym[2 * (j / CYCLES) + 1];
        } else {
            st->fir_mem[QK_NTAPS - 1][0] = 0.0f;
            st->fir_mem[QK_NTAPS - 1][1] = 0.0f;
        }
        float yr = 0.0f, yi = 0.0f;
        for (int i = 0; i < QK_NTAPS; i++) {
            yr = yr + st->fir_mem[i][0] * QK_RRC[i];
            yi = yi + st->fir_mem[i][1] * QK_RRC[i];
        }
        yr = yr * QK_GAIN;
        yi = yi * QK_GAIN;
        /* shift to 1100 Hz, src/qpsk.c:301-304 */
        const float a = st->phase[0] * rr - st->phase[1] * ri;
        const float b = st->phase[0] * ri + st->phase[1] * rr;
        st->phase[0] = a;
        st->phase[1] = b;
        const float sr = yr * a - yi * b;
        out[j] = (int16_t)(sr * scale);   /* src/qpsk.c:313-319 (truncation) */
    }
    /* fbb_tx_phase /= cabsf(fbb_tx_phase), src/qpsk.c:306 (glibc hypotf) */
    const float mag = (float)sqrt((double)st->phase[0] * st->phase[0] +
                                  (double)st->phase[1] * st->phase[1]);
    st->phase[0] = st->phase[0] / mag;
    st->phase[1] = st->phase[1] / mag;
    return length * CYCLES;
}

static qpsk_tx_state g_tx = {{{0}}, {1.0f, 0.0f}};  /* tx_filter, fbb_tx_phase src/qpsk.c:39,47 */

void qpsk_tx_init(void) { qpsk_tx_state_init(&g_tx); }

int qpsk_tx_frame(int16_t out[], float _Complex symbol[], int length, bool preamble) {
    return qpsk_tx_frame_state(&g_tx, out, (const float *)symbol, length, preamble);
}

/* ---------------------------------------------------------------- RX */

static qpsk_ctx *g_rx;
static int g_rx_err;

void qpsk_rx_init(void) {
    int err = QPSK_OK;
    if (!g_rx) g_rx = qpsk_rx_create(0, 1, &err);
    else err = qpsk_rx_reset(g_rx);
    g_rx_err = g_rx ? err : (err ? err : QPSK_ENODEV);
}

int qpsk_surface_error(void) { return g_rx_err; }

int qpsk_rx_frame(int16_t in[], uint8_t bits[]) {
    if (!g_rx) qpsk_rx_init();
    if (!g_rx) return 0;
    uint8_t b[QK_NBITS], v = 0;
    g_rx_err = qpsk_rx_batch(g_rx, in, 1, b, &v, NULL, NULL);
    if (g_rx_err != QPSK_OK || !v) return 0;
    memcpy(bits, b, QK_NBITS);  /* bits untouched on invalid frames, like the reference */
    return 1;
}
