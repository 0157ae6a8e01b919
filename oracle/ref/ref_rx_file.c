/*
 * ref_rx_file.c -- TEST INFRASTRUCTURE ONLY (oracle).
 * The reference RX driver loop (src/qpsk.c:420-461) over an arbitrary .raw
 * file: 1880-int16 frames, short tail dropped, a 496-byte record per valid
 * frame (bytes 62..495 zero).  Usage: ref_rx_file in.raw out.bin [log.txt]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ref_api.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s in.raw out.bin [debug.log]\n", argv[0]);
        return 2;
    }
    FILE *fin = fopen(argv[1], "rb");
    FILE *fout = fopen(argv[2], "wb");
    if (!fin || !fout) return 1;
    static char log[1 << 20];
    ref_log_set(log, sizeof log);
    if (ref_rx_reset() != 0) {
        fprintf(stderr, "reference static layout is not model A\n");
        return 3;
    }
    int16_t frame[1880];
    uint8_t rec[496];
    while (fread(frame, sizeof(int16_t), 1880, fin) == 1880) {
        memset(rec, 0, sizeof rec);
        if (ref_rx_frame(frame, rec, NULL)) fwrite(rec, 1, sizeof rec, fout);
    }
    fclose(fin);
    fclose(fout);
    if (argc > 3) {
        FILE *fl = fopen(argv[3], "w");
        if (fl) {
            fputs(log, fl);
            fclose(fl);
        }
    }
    return 0;
}
