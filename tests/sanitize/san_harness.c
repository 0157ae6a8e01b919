/* san_harness.c -- TEST ONLY.  Drives the host C of the path under
 * AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitize.py):
 * the oracle restatement (oracle/cpu_ref.c), the host input generator
 * (csrc/qpsk_synth.c), the reference surface (csrc/qpsk_surface.c: TX,
 * qpsk_mod/demod/cnormf, qpsk_rx_frame's host logic) and the record writer
 * (csrc/qpsk_records.c).  qpsk_rx_frame() reaches the GPU through
 * qpsk_rx_create/qpsk_rx_batch; here a host test double answers those calls
 * with the oracle, so the surface's own host logic (init, error propagation,
 * bits left untouched on invalid frames) runs sanitized.  Every output is
 * written to OUTDIR and compared by the Python test with the unsanitized
 * build's results.
 *
 *   san_harness OUTDIR SAMPLE.raw
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cpu_ref.h"
#include "qpsk_batch.h"
#include "qpsk_internal.h"
#include "qpsk_stream.h"
#include "qpsk_synth.h"

/* ---- test double of the batch ABI for qpsk_surface.c (one channel) ---- */
struct qpsk_ctx { qc_chan_t ch; int nch; };

qpsk_ctx *qpsk_rx_create(int device, int nch, int *err) {
    (void)device;
    qpsk_ctx *c = calloc(1, sizeof *c);
    if (!c || nch != 1) { free(c); *err = QPSK_EINVAL; return NULL; }
    qc_chan_init(&c->ch);
    c->nch = nch;
    *err = QPSK_OK;
    return c;
}

int qpsk_rx_reset(qpsk_ctx *c) { qc_chan_init(&c->ch); return QPSK_OK; }

int qpsk_rx_batch(qpsk_ctx *c, const int16_t *in, int nframes, uint8_t *bits, uint8_t *valid,
                  int32_t *trace, float *soft) {
    (void)trace; (void)soft;
    for (int f = 0; f < nframes; f++) {
        uint8_t b[QC_BITS] = {0};
        valid[f] = (uint8_t)qc_rx_frame(&c->ch, in + (size_t)f * QC_FRAME, b, NULL);
        memcpy(bits + (size_t)f * QC_BITS, b, QC_BITS);
    }
    return QPSK_OK;
}

static void put(const char *dir, const char *name, const void *p, size_t n) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(p, 1, n, f) != n) { perror(path); exit(2); }
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s OUTDIR SAMPLE.raw\n", argv[0]); return 2; }
    const char *dir = argv[1];
    enum { NCH = 24, NF = 12 };
    const long ns = (long)NF * QC_FRAME;

    /* host generator, 4 threads (AWGN: the Box-Muller path too) */
    int16_t *x = malloc(sizeof(int16_t) * NCH * ns);
    qpsk_synth_batch(7, 100, NCH, 4.0, x, ns, 4);
    put(dir, "synth.bin", x, sizeof(int16_t) * NCH * ns);

    /* oracle receiver, every mode, threaded, traced */
    uint8_t *bits = malloc((size_t)NCH * NF * QC_BITS), *valid = malloc((size_t)NCH * NF);
    qc_trace_t *tr = malloc(sizeof(qc_trace_t) * NCH * NF);
    for (int mode = 0; mode < 4; mode++) {
        char name[64];
        qc_rx_batch_mode(x, NCH, NF, bits, valid, tr, 4, mode);
        snprintf(name, sizeof name, "rx_bits_m%d.bin", mode);
        put(dir, name, bits, (size_t)NCH * NF * QC_BITS);
        snprintf(name, sizeof name, "rx_valid_m%d.bin", mode);
        put(dir, name, valid, (size_t)NCH * NF);
        snprintf(name, sizeof name, "rx_trace_m%d.bin", mode);
        put(dir, name, tr, sizeof(qc_trace_t) * NCH * NF);
    }

    /* the surface's qpsk_rx_frame over the sample file, records as the
     * reference driver writes them (src/qpsk.c:436-458) */
    FILE *f = fopen(argv[2], "rb");
    if (!f) { perror(argv[2]); return 2; }
    int16_t fr[QC_FRAME];
    uint8_t b[QC_BITS], v;
    uint8_t *recs = malloc(496 * 64);
    size_t nrec = 0;
    qpsk_rx_init();
    while (fread(fr, sizeof fr, 1, f) == 1 && nrec < 64 * 496) {
        memset(b, 0, sizeof b);
        v = (uint8_t)qpsk_rx_frame(fr, b);
        nrec += qpsk_records(b, &v, 1, recs + nrec);
    }
    fclose(f);
    if (qpsk_surface_error() != QPSK_OK) return 3;
    put(dir, "surface_records.bin", recs, nrec);

    /* TX surface: a preamble frame then three data frames, symbols from the
     * reference modulator qpsk_mod() over LCG bits */
    qpsk_tx_init();
    float _Complex sym[QC_PRE];
    int16_t *tx = malloc(sizeof(int16_t) * 4 * QC_PRE * 5);
    uint32_t lcg = 12345u;
    long nt = 0;
    for (int k = 0; k < 4; k++) {
        const int len = k == 0 ? QC_PRE : QC_DSYM;
        for (int s = 0; s < len; s++) {
            uint8_t bb[2];
            lcg = lcg * 1664525u + 1013904223u;
            bb[0] = (uint8_t)((lcg >> 16) & 1u);
            bb[1] = (uint8_t)((lcg >> 17) & 1u);
            sym[s] = qpsk_mod(bb, 0);
        }
        nt += qpsk_tx_frame(tx + nt, sym, len, k == 0);
    }
    put(dir, "tx.bin", tx, sizeof(int16_t) * nt);

    /* qpsk_demod / cnormf over a grid of symbols incl. signed zeros */
    const float vals[] = {-2.5f, -1.0f, -0.0f, 0.0f, 1e-30f, 3.0f};
    uint8_t dm[36 * 2];
    float cn[36];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            float _Complex s;
            __real__ s = vals[i];
            __imag__ s = vals[j];
            qpsk_demod(dm + 2 * (6 * i + j), s);
            cn[6 * i + j] = cnormf(s);
        }
    put(dir, "demod.bin", dm, sizeof dm);
    put(dir, "cnormf.bin", cn, sizeof cn);

    free(x); free(bits); free(valid); free(tr); free(recs); free(tx);
    return 0;
}
