/*
 * cpu_ref.h -- TEST INFRASTRUCTURE ONLY (oracle).
 *
 * Clean-room C restatement of the reference receive path qpsk_rx_frame()
 * (/root/reference/src/qpsk.c:133-239 and its callees), in the bit-exact
 * "minimal form" of SURVEY.md App. A, with all per-channel state explicit.
 * It is the checker for the HIP product path (tests/, __graft_entry__.smoke())
 * and the "port" CPU baseline leg of bench.py; nothing in singlecarrier_amd/
 * links it.  Parity of this restatement with the unmodified reference is pinned
 * by tests/test_oracle.py against oracle/_ref (built from /root/reference) and
 * the committed golden fixtures in tests/golden/.
 *
 * Also holds a restatement of the reference transmitter (src/qpsk.c:251-342),
 * used to synthesise test inputs.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QC_FRAME      1880   /* FRAME_SIZE          headers/qpsk_internal.h:45 */
#define QC_DEC        188    /* FRAME_SIZE/CYCLES/2: carried decimated symbols */
#define QC_PRE        128    /* PREAMBLE_LENGTH     headers/qpsk_internal.h:50 */
#define QC_DSYM       31     /* DATA_SYMBOLS        headers/qpsk_internal.h:37 */
#define QC_BITS       62     /* bits written per valid frame                   */
#define QC_NTAPS      49     /* NTAPS               headers/fir.h:16           */
#define QC_PACKET     2783   /* one TX packet: 640 + 8*155 + 903 samples       */

#define QC_DEC752     290    /* observable carried symbols, dec752 mode        */

/* Receiver semantics. */
#define QC_MODE_REF     0    /* the reference as built: gcc -O2 "model A" overflow */
#define QC_MODE_DEC752  1    /* decimated_frame with the 752 entries its loop
                                assumes (src/qpsk.c:157-162): NOT reference
                                parity; pinned by the layout-padded reference
                                build oracle/_ref/libqpsk_ref752.so           */
#define QC_MODE_FFT_HUNT 2   /* flag: the preamble hunt correlates through the
                                reference's kiss_fft (src/fft.c), see qc_fft_hunt */

/* Explicit per-channel receiver state (the reference keeps it in statics,
 * src/qpsk.c:37-53, src/scramble.c:41-42). */
typedef struct {
    int32_t rx_timing;          /* src/qpsk.c:53, starts at 3               */
    uint32_t frame;             /* frames received so far                   */
    int32_t mode;               /* QC_MODE_*                                */
    float dprev[QC_DEC752][2];  /* D_{n-1}: decimated symbols carried over
                                   (model A uses the first QC_DEC)          */
    int16_t hist[2][QC_FRAME];  /* hist[1] = x_{n-1}, hist[0] = x_{n-2}     */
} qc_chan_t;

typedef struct {
    int32_t max_index;
    int32_t matches;
    int32_t valid;
    int32_t rx_timing;          /* after the frame */
    float soft[QC_DSYM][2];     /* valid frames only (zero otherwise) */
} qc_trace_t;

void qc_chan_init(qc_chan_t *ch);
void qc_chan_init_mode(qc_chan_t *ch, int mode);
/* Diagnostics (profiles/decision_steps_drv.c): after qc_rx_frame, the first
 * training step at which the frame's validity was certain (matches > 98, or
 * 30 misses); 128 if only the last step decided it.  Per thread (the batch
 * path runs qc_rx_frame on pthreads). */
extern _Thread_local int qc_decision_step;
/* Test switch (tests/test_oracle.py): when nonzero, every dec entry outside
 * [mi, mi + 162] is set to NaN after the hunt, before the equalizer: the
 * outputs must not change (the window's observable range, which the GPU's
 * split FIR relies on: dec[255..289] only when mi >= 93).  Set it only while
 * no call runs. */
extern int qc_poison_unobservable;
/* One qpsk_rx_frame() call.  bits[62] written (zero when invalid). */
int qc_rx_frame(qc_chan_t *ch, const int16_t in[QC_FRAME], uint8_t bits[QC_BITS],
                qc_trace_t *tr);
/* nch independent channels from a fresh state, nthreads pthreads over channels.
 * in [nch][nframes][1880]; bits [nch][nframes][62]; valid [nch][nframes];
 * tr [nch][nframes] or NULL.  Returns the number of valid frames. */
long qc_rx_batch(const int16_t *in, int nch, int nframes, uint8_t *bits,
                 uint8_t *valid, qc_trace_t *tr, int nthreads);
/* Stage tap: one channel from a fresh state; dec_out [nframes][290][2] gets
 * the observable decimated_frame[0..289] of every call (after decimation,
 * before the hunt), as the reference's buffer holds it.  Returns #valid. */
long qc_rx_stages(const int16_t *in, int nframes, int mode, float *dec_out);
/* Same, with the receiver semantics `mode` (QC_MODE_*). */
long qc_rx_batch_mode(const int16_t *in, int nch, int nframes, uint8_t *bits,
                      uint8_t *valid, qc_trace_t *tr, int nthreads, int mode);

/* Mixer table P[t] = R^(t+1) (fp32 recurrence, src/qpsk.c:139), KAT access. */
void qc_mixer_table(float p[QC_FRAME][2]);
/* RX descrambler keystream bits ks[0..n) (src/scramble.c:57-69, seed 0x4A80). */
void qc_keystream(uint8_t *ks, int n);

/* ---- kiss_fft restatement (src/fft.c; no caller in the reference) ------- */
/* fft_alloc(nfft, inverse) + fft() (headers/fft.h:45-46) on nfft interleaved
 * (re, im) pairs; any nfft >= 1 (radix 4, 2, 3, 5 and generic stages).
 * Returns 0, or -1 for nfft < 1. */
int qc_fft(int nfft, int inverse, const float *in, float *out);
/* the twiddle table fft_alloc() builds (src/fft.c:67-74), nfft pairs */
void qc_fft_twiddles(int nfft, int inverse, float *tw);
/* The FFT-correlation hunt of the QC_MODE_FFT_HUNT receiver variant over
 * dec[0..255] (interleaved pairs):  S = ifft(fft(dec) * Q) with
 * Q = conj(fft(c)), c[i] = conj(preambletable[i]) = (p_i, -p_i) for i < 128
 * and 0 above (256-point kiss_fft, unnormalized; S[l] = 256 x the correlate()
 * sum of src/qpsk.c:88-96 in exact arithmetic); then the reference's hunt
 * loop (src/qpsk.c:172-183) over cnormf(S[l]), l < 128.  Returns max_index. */
int qc_fft_hunt(const float *dec);
/* Q above (256 pairs), for tests */
void qc_fft_hunt_spectrum(float *q);

/* ---- transmitter restatement (src/qpsk.c:251-342) ---------------------- */
typedef struct {
    float fir_mem[QC_NTAPS][2];  /* tx_filter, src/qpsk.c:39   */
    float phase[2];              /* fbb_tx_phase, src/qpsk.c:47 */
} qc_tx_t;

void qc_tx_init(qc_tx_t *tx);
/* qpsk_tx_frame(): len symbols -> 5*len int16 samples. */
int qc_tx_frame(qc_tx_t *tx, int16_t *out, const float (*sym)[2], int len,
                int preamble);

/* Synthetic channel stream: reference TX packets (preamble +
 * 8x31 data symbols + 903 zeros) with dibits and a leading delay drawn from
 * splitmix64(seed ^ c*0x9E3779B97F4A7C15); optional AWGN at ebn0_db
 * (ebn0_db >= 100 -> noiseless).  out gets nsamples int16. */
void qc_synth_channel(uint64_t seed, uint32_t c, double ebn0_db, int16_t *out,
                      long nsamples, uint8_t *txbits /* optional, see .c */);
/* [nch][nsamples] with nthreads threads. */
void qc_synth_batch(uint64_t seed, uint32_t c0, int nch, double ebn0_db,
                    int16_t *out, long nsamples, int nthreads);

#ifdef __cplusplus
}
#endif
