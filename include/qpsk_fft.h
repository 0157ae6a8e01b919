/*
 * qpsk_fft.h -- the reference's complex FFT on the GPU, batched.
 *
 * Replaces fft_alloc() / fft() of the reference's kiss_fft
 * (headers/fft.h:45-46, src/fft.c:52-83, 133-135) for many transforms per
 * call.  Results are bit-identical to the reference's fft() (same
 * factorization, twiddles and butterfly arithmetic; tests/test_gpu_fft.py).
 * The reference itself never calls its FFT; the receive path
 * uses it in the QPSK_MODE_FFT_HUNT receiver variant (qpsk_batch.h).
 *
 * Sizes: nfft a power of two, 4 <= nfft <= 4096 (kiss_fft's radix-4 stages plus
 * one radix-2 stage for odd powers).  Other sizes return QPSK_EINVAL.
 * Layout: [batch][nfft] complex float, interleaved (re, im); unnormalized,
 * inverse = the reference's inverse_fft flag (twiddle sign only).
 * Errors: the QPSK_E* codes of qpsk_batch.h.
 */
#pragma once
#include "qpsk_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qpsk_fft_plan qpsk_fft_plan;

/* fft_alloc(nfft, inverse_fft, NULL, NULL) on HIP device `device`. */
qpsk_fft_plan *qpsk_fft_alloc(int device, int nfft, int inverse, int *err);
void qpsk_fft_free(qpsk_fft_plan *plan);
/* fft(cfg, in, out) for `batch` transforms; device pointers, enqueued on
 * `stream` (hipStream_t, NULL = default), no synchronisation.  in may equal out. */
int qpsk_fft_device(qpsk_fft_plan *plan, const float *d_in, float *d_out, int batch, void *stream);
/* The same from and to host memory (synchronous). */
int qpsk_fft(qpsk_fft_plan *plan, const float *in, float *out, int batch);

#ifdef __cplusplus
}
#endif
