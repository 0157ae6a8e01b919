/*
 * ref_fft.c -- TEST INFRASTRUCTURE ONLY (oracle).  Never shipped.
 *
 * C interface to the reference's UNMODIFIED kiss_fft (/root/reference/src/fft.c,
 * compiled where it lies by oracle/Makefile into oracle/_ref/libkissfft_ref.so):
 * fft_alloc() + fft() (headers/fft.h:45-46), one transform per call.  Pins the
 * restatement qc_fft() (oracle/cpu_ref.c) and, through it, the GPU FFT.
 */
#include <stdlib.h>

#include "fft.h"

/* in/out: nfft interleaved (re, im) pairs; returns 0, or -1 if fft_alloc fails */
int ref_fft(int nfft, int inverse, const float *in, float *out) {
    fft_cfg cfg = fft_alloc(nfft, inverse, NULL, NULL);   /* src/fft.c:52 */
    if (!cfg) return -1;
    fft(cfg, (const complex float *)in, (complex float *)out);   /* src/fft.c:133 */
    free(cfg);
    return 0;
}

/* The factor list kf_factor() (src/fft.c:433) builds: (p, m) pairs, 0-terminated. */
int ref_fft_factors(int nfft, int *out, int cap) {
    fft_cfg cfg = fft_alloc(nfft, 0, NULL, NULL);
    if (!cfg) return -1;
    int k = 0;
    for (; k + 1 < cap && k < 64; k += 2) {
        out[k] = cfg->factors[k];
        out[k + 1] = cfg->factors[k + 1];
        if (cfg->factors[k + 1] == 1) { k += 2; break; }
    }
    free(cfg);
    return k / 2;
}
