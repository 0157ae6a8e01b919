/* qpsk_records.c -- the reference RX driver's output records (include/
 * qpsk_stream.h): one 496-byte record per valid frame, bits in bytes 0..61
 * (src/qpsk.c:455-457), zero elsewhere (the reference writes an uninitialised
 * stack array there; zero in every observed run).
 * Host C (gcc), so the sanitizer build (tests/test_sanitize.py) covers it. */
#include <stdint.h>
#include <string.h>

#include "qpsk_consts.h"
#include "qpsk_stream.h"

size_t qpsk_records(const uint8_t *bits, const uint8_t *valid, int nframes, uint8_t *out) {
    size_t n = 0;
    for (int f = 0; f < nframes; f++) {
        if (!valid[f]) continue;
        memcpy(out + n, bits + (size_t)f * QK_NBITS, QK_NBITS);
        memset(out + n + QK_NBITS, 0, 496 - QK_NBITS);
        n += 496;
    }
    return n;
}
