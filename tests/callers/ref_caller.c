/*
 * ref_caller.c -- a caller written against the reference's header surface
 * (/root/reference/headers/qpsk_internal.h) and nothing else: it includes no
 * system header of its own and uses the header's macros, its RXState type,
 * C99 `complex float` and cmplx() the way the reference's own driver does
 * (src/qpsk.c:346-461).  tests/test_header_surface.py compiles it against the
 * repo's include/qpsk_internal.h and links libqpsk_hip.so (INTEGRATION.md:
 * "no source changes"), and compiles its `consts` part against the reference
 * header too, to compare every macro value.
 *
 *   ref_caller consts                 the header's constants, one per line
 *   ref_caller tx SYMS OUT            qpsk_tx_frame over frames read from SYMS
 *                                     (int32 n; then per frame int32 len, int32
 *                                     preamble, len x (float re, float im)); int16 to OUT
 *   ref_caller rx IN OUT              the reference RX loop (src/qpsk.c:436-458):
 *                                     qpsk_rx_frame per 1880-sample frame, a
 *                                     496-byte record per valid frame (GPU)
 */
#include "qpsk_internal.h"

static int consts(void) {
    const complex float rect = cmplx(TAU * -CENTER / FS);   /* fbb_rx_rect, src/qpsk.c:428 */
    const complex float conj45 = cmplxconj(ROT45);
    RXState st = hunt;
    printf("FINE_TIMING_OFFSET %d\n", FINE_TIMING_OFFSET);
    printf("TX_FILENAME %s\nRX_FILENAME %s\n", TX_FILENAME, RX_FILENAME);
    printf("EOF_COST_VALUE %a\nEQ_LENGTH %d\n", (double)EOF_COST_VALUE, EQ_LENGTH);
    printf("FS %a\nRS %a\nTS %a\n", (double)FS, (double)RS, (double)TS);
    printf("CYCLES %d sizeof %zu\nCYCLESF %d\n", CYCLES, sizeof(CYCLES), CYCLESF);
    printf("CENTER %a\nNS %d\nDATA_SYMBOLS %d\n", (double)CENTER, NS, DATA_SYMBOLS);
    printf("FRAME_SYMBOLS %d\nDATA_SAMPLES %d\nDATA_SIZE %d\n", FRAME_SYMBOLS, DATA_SAMPLES, DATA_SIZE);
    printf("FRAME_SIZE %d\nBITS_PER_FRAME %d\n", FRAME_SIZE, BITS_PER_FRAME);
    printf("PREAMBLE_LENGTH %d\nPREAMBLE_SIZE %d\n", PREAMBLE_LENGTH, PREAMBLE_SIZE);
    printf("TAU %a\nROT45 %a\n", (double)TAU, (double)ROT45);
    printf("rect %a %a\n", (double)crealf(rect), (double)cimagf(rect));
    printf("conj45 %a %a\n", (double)crealf(conj45), (double)cimagf(conj45));
    printf("RXState %d %d %zu\n", (int)st, (int)process, sizeof(RXState));
    return 0;
}

#ifndef CONSTS_ONLY
static int tx(const char *syms, const char *out) {
    FILE *fi = fopen(syms, "rb"), *fo = fopen(out, "wb");
    int32_t n;
    if (!fi || !fo || fread(&n, sizeof n, 1, fi) != 1) return 1;
    for (int32_t k = 0; k < n; k++) {
        int32_t len, pre;
        if (fread(&len, sizeof len, 1, fi) != 1 || fread(&pre, sizeof pre, 1, fi) != 1) return 1;
        complex float *sym = malloc(sizeof(complex float) * (size_t)len);
        int16_t *samples = malloc(sizeof(int16_t) * (size_t)len * CYCLES);
        for (int32_t i = 0; i < len; i++) {
            float re, im;
            if (fread(&re, 4, 1, fi) != 1 || fread(&im, 4, 1, fi) != 1) return 1;
            sym[i] = re + im * I;
        }
        const int m = qpsk_tx_frame(samples, sym, len, pre != 0);   /* len * CYCLES samples */
        if (m != len * CYCLES) return 2;
        fwrite(samples, sizeof(int16_t), (size_t)m, fo);
        free(sym);
        free(samples);
    }
    fclose(fi);
    fclose(fo);
    return 0;
}

static int rx(const char *in, const char *out) {
    FILE *fin = fopen(in, "rb"), *fout = fopen(out, "wb");
    int16_t frame[FRAME_SIZE];
    uint8_t ibits[BITS_PER_FRAME];
    RXState state = hunt;
    if (!fin || !fout) return 1;
    while (fread(frame, sizeof(int16_t), FRAME_SIZE, fin) == FRAME_SIZE) {
        memset(ibits, 0, sizeof ibits);
        if (qpsk_rx_frame(frame, ibits)) {
            state = process;
            fwrite(ibits, sizeof(uint8_t), BITS_PER_FRAME, fout);
        } else {
            state = hunt;
        }
    }
    fclose(fin);
    fclose(fout);
    return state == hunt || state == process ? 0 : 1;
}
#endif

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "consts")) return consts();
#ifndef CONSTS_ONLY
    if (argc >= 4 && !strcmp(argv[1], "tx")) return tx(argv[2], argv[3]);
    if (argc >= 4 && !strcmp(argv[1], "rx")) return rx(argv[2], argv[3]);
#endif
    fprintf(stderr, "usage: ref_caller consts | tx SYMS OUT | rx IN OUT\n");
    return 64;
}
