/*
 * qpsk_rx_stream.c -- the reference RX driver loop (src/qpsk.c:420-461) for
 * many channels at once, streaming: every input file is one channel's .raw
 * stream (int16 LE, 1880-sample frames), read chunk by chunk straight into the
 * pinned slots of a qpsk_stream (include/qpsk_stream.h); the receive of one
 * chunk overlaps the file reads and PCIe copies of the next.  Each channel's
 * 496-byte records go to PREFIX<i>.bin, as the reference writes them
 * (src/qpsk.c:455-457).
 *
 *   qpsk_rx_stream [-f FRAMES_PER_CHUNK] in1.raw [in2.raw ...] -o PREFIX
 *
 * Channels end at the shortest file (whole frames only, as the reference).
 * Build: make -C examples
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qpsk_batch.h"
#include "qpsk_internal.h"
#include "qpsk_stream.h"

static void drain(qpsk_stream *s, int nch, int frames, int nf_chunk, FILE **out, uint8_t *rec) {
    const uint8_t *bits, *valid;
    int err = qpsk_stream_retrieve(s, &bits, &valid);
    if (err) {
        fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
        exit(3);
    }
    for (int c = 0; c < nch; c++) {
        size_t n = qpsk_records(bits + (size_t)c * frames * 62, valid + (size_t)c * frames,
                                nf_chunk, rec);
        if (n && fwrite(rec, 1, n, out[c]) != n) exit(1);
    }
}

int main(int argc, char **argv) {
    int frames = 8, a = 1;
    if (argc > 2 && !strcmp(argv[1], "-f")) {
        frames = atoi(argv[2]);
        a = 3;
    }
    if (argc - a < 3 || strcmp(argv[argc - 2], "-o") || frames < 1) {
        fprintf(stderr, "usage: %s [-f FRAMES_PER_CHUNK] in1.raw [in2.raw ...] -o PREFIX\n", argv[0]);
        return 2;
    }
    const int nch = argc - a - 2;
    const char *prefix = argv[argc - 1];
    FILE **in = calloc((size_t)nch, sizeof(FILE *)), **out = calloc((size_t)nch, sizeof(FILE *));
    for (int c = 0; c < nch; c++) {
        char name[4096];
        snprintf(name, sizeof name, "%s%d.bin", prefix, c);
        in[c] = fopen(argv[a + c], "rb");
        out[c] = fopen(name, "wb");
        if (!in[c] || !out[c]) return 1;
    }
    const int nslot = 3;
    int err;
    qpsk_stream *s = qpsk_stream_create(0, nch, frames, nslot, &err);
    if (!s) {
        fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
        return 3;
    }
    uint8_t *rec = malloc((size_t)frames * BITS_PER_FRAME);
    int sizes[4] = {0};   /* frames in each slot's chunk (slots are used in order) */
    long submitted = 0, retrieved = 0;
    for (int done = 0; !done;) {
        if (qpsk_stream_pending(s) == nslot) {
            drain(s, nch, frames, sizes[retrieved % nslot], out, rec);
            retrieved++;
        }
        int16_t *buf = qpsk_stream_acquire(s, &err);
        if (!buf) {
            fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
            return 3;
        }
        /* every channel contributes the same number of whole frames */
        int nf = frames;
        for (int c = 0; c < nch; c++) {
            size_t got = fread(buf + (size_t)c * frames * FRAME_SIZE, sizeof(int16_t) * FRAME_SIZE,
                               (size_t)nf, in[c]);                           /* src/qpsk.c:442 */
            if ((int)got < nf) nf = (int)got;
        }
        if (nf < frames) done = 1;   /* the shortest stream ended inside this chunk */
        if (nf == 0) break;
        /* frames past nf of a short chunk are received too but never written out */
        if ((err = qpsk_stream_submit(s))) {
            fprintf(stderr, "qpsk: %s\n", qpsk_strerror(err));
            return 3;
        }
        sizes[submitted % nslot] = nf;
        submitted++;
    }
    while (retrieved < submitted) {
        drain(s, nch, frames, sizes[retrieved % nslot], out, rec);
        retrieved++;
    }
    qpsk_stream_destroy(s);
    for (int c = 0; c < nch; c++) {
        fclose(in[c]);
        fclose(out[c]);
    }
    free(rec);
    return 0;
}
