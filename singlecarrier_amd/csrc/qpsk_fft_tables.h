// qpsk_fft_tables.h -- host tables of the GPU kiss_fft (qpsk_fft_host.c)
#pragma once
#ifdef __cplusplus
extern "C" {
#endif
/* fft_alloc()'s twiddles (src/fft.c:67-74): nfft interleaved (re, im) pairs */
void qpsk_fft_twiddle_table(int nfft, int inverse, float *tw);
/* kf_work()'s input permutation for a power of two nfft >= 2; -1 otherwise */
int qpsk_fft_perm_table(int nfft, int *perm);
#ifdef __cplusplus
}
#endif
