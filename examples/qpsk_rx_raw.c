/*
 * qpsk_rx_raw.c -- the reference RX driver loop (src/qpsk.c:420-461) built
 * against the drop-in library instead of the reference sources.
 *
 *   qpsk_rx_raw in.raw out.bin            single channel, qpsk_rx_frame() per frame
 *                                          (unchanged reference call pattern)
 *   qpsk_rx_raw -b [-m MODE] in1.raw [in2.raw ...] -o PREFIX
 *                                          every file is one channel; all channels are
 *                                          demodulated together through qpsk_rx_batch()
 *                                          and PREFIX<i>.bin is written per channel;
 *                                          MODE = QPSK_MODE_* (qpsk_batch.h, default 0:
 *                                          the reference; 1 dec752, 2 FFT hunt, 3 both)
 * Output: one 496-byte record per valid frame, bits in bytes 0..61 (the
 * reference's /tmp/databits.txt format, src/qpsk.c:455-457).
 * Build: gcc -O2 -Iinclude qpsk_rx_raw.c -Lsinglecarrier_amd -lqpsk_hip -Wl,-rpath,...
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qpsk_batch.h"
#include "qpsk_internal.h"

static int16_t *read_frames(const char *path, int *nframes) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    *nframes = (int)(bytes / (long)(sizeof(int16_t) * FRAME_SIZE));  /* short tail dropped */
    int16_t *buf = malloc(sizeof(int16_t) * (size_t)(*nframes > 0 ? *nframes : 1) * FRAME_SIZE);
    if (buf && fread(buf, sizeof(int16_t) * FRAME_SIZE, (size_t)*nframes, f) != (size_t)*nframes) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    return buf;
}

static int single(const char *in, const char *out) {
    FILE *fin = fopen(in, "rb"), *fout = fopen(out, "wb");
    if (!fin || !fout) return 1;
    int16_t frame[FRAME_SIZE];
    uint8_t ibits[BITS_PER_FRAME];
    qpsk_rx_init();
    if (qpsk_surface_error()) {
        fprintf(stderr, "qpsk: %s\n", qpsk_strerror(qpsk_surface_error()));
        return 3;
    }
    while (fread(frame, sizeof(int16_t), FRAME_SIZE, fin) == FRAME_SIZE) {   /* src/qpsk.c:442 */
        memset(ibits, 0, sizeof ibits);
        int valid = qpsk_rx_frame(frame, ibits);                              /* src/qpsk.c:447 */
        if (qpsk_surface_error()) {
            fprintf(stderr, "qpsk: %s\n", qpsk_strerror(qpsk_surface_error()));
            return 3;
        }
        if (valid) fwrite(ibits, sizeof(uint8_t), BITS_PER_FRAME, fout);        /* src/qpsk.c:455 */
    }
    fclose(fin);
    fclose(fout);
    return 0;
}

static int batch(int nch, char **paths, const char *prefix, int mode) {
    int nf = -1;
    int16_t **ch = calloc((size_t)nch, sizeof(int16_t *));
    for (int c = 0; c < nch; c++) {
        int n;
        ch[c] = read_frames(paths[c], &n);
        if (!ch[c]) return 1;
        if (nf < 0 || n < nf) nf = n;   /* common length: frames every channel has */
    }
    if (nf <= 0) return 1;
    int16_t *in = malloc(sizeof(int16_t) * (size_t)nch * nf * FRAME_SIZE);
    for (int c = 0; c < nch; c++)
        memcpy(in + (size_t)c * nf * FRAME_SIZE, ch[c], sizeof(int16_t) * (size_t)nf * FRAME_SIZE);
    uint8_t *bits = malloc((size_t)nch * nf * 62), *valid = malloc((size_t)nch * nf);
    int err;
    qpsk_ctx *ctx = qpsk_rx_create_mode(0, nch, mode, &err);
    if (!ctx) {
        fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
        return 3;
    }
    err = qpsk_rx_batch(ctx, in, nf, bits, valid, NULL, NULL);
    if (err) {
        fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
        return 3;
    }
    uint8_t rec[BITS_PER_FRAME];
    for (int c = 0; c < nch; c++) {
        char name[4096];
        snprintf(name, sizeof name, "%s%d.bin", prefix, c);
        FILE *fo = fopen(name, "wb");
        if (!fo) return 1;
        for (int n = 0; n < nf; n++) {
            if (!valid[(size_t)c * nf + n]) continue;
            memset(rec, 0, sizeof rec);
            memcpy(rec, bits + ((size_t)c * nf + n) * 62, 62);
            fwrite(rec, 1, sizeof rec, fo);
        }
        fclose(fo);
    }
    qpsk_rx_destroy(ctx);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 3 && strcmp(argv[1], "-b") != 0) return single(argv[1], argv[2]);
    if (argc >= 5 && !strcmp(argv[1], "-b") && !strcmp(argv[argc - 2], "-o")) {
        int first = 2, mode = QPSK_MODE_REFERENCE;
        if (argc >= 7 && !strcmp(argv[2], "-m")) {
            mode = atoi(argv[3]);
            first = 4;
        }
        return batch(argc - 2 - first, argv + first, argv[argc - 1], mode);
    }
    fprintf(stderr, "usage: %s in.raw out.bin | -b [-m MODE] in1.raw [in2.raw ...] -o PREFIX\n",
            argv[0]);
    return 2;
}
