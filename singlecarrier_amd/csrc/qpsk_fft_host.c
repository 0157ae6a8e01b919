/*
 * qpsk_fft_host.c -- host tables of the GPU kiss_fft (qpsk_fft.hip).
 *
 * Built with gcc -O2 like the reference, and written as the reference writes
 * them, so the twiddles are the same bits fft_alloc() makes:
 *   twiddles  src/fft.c:67-74: phase = -TAU * i / nfft (TAU = 2.0f * M_PI,
 *             M_PI being math.h's double, so the product is formed in double
 *             and rounded once to the float phase), cmplx(phase) =
 *             cosf + sinf * I (headers/qpsk_internal.h:67);
 *   perm      the leaf copies of kf_work (src/fft.c:398-402): output position
 *             j of the first stage holds input perm[j].
 */
#include <math.h>
#include <stddef.h>

#include "qpsk_fft_tables.h"

void qpsk_fft_twiddle_table(int nfft, int inverse, float *tw) {
    const double tau = 2.0f * 3.14159265358979323846;
    for (int i = 0; i < nfft; i++) {
        float phase = (float)(-tau * (float)i / (float)nfft);
        if (inverse) phase *= -1.0f;
        tw[2 * i] = cosf(phase);
        tw[2 * i + 1] = sinf(phase);
    }
}

/* kf_factor (src/fft.c:433-459) of a power of two: 4, 4, ..., then 2 */
static void work(int *perm, int out, int in, int fstride, int n) {
    const int p = (n % 4 == 0) ? 4 : 2;   /* n >= 2 here */
    const int m = n / p;
    if (m == 1) {
        for (int j = 0; j < p; j++) perm[out + j] = in + j * fstride;
    } else {
        for (int j = 0; j < p; j++) work(perm, out + j * m, in + j * fstride, fstride * p, m);
    }
}

int qpsk_fft_perm_table(int nfft, int *perm) {
    if (nfft < 2 || (nfft & (nfft - 1)) != 0) return -1;
    work(perm, 0, 0, 1, nfft);
    return 0;
}
