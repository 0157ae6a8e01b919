/*
 * qpsk_batch.h -- batched, multi-channel C-ABI of the MI355X receive path.
 *
 * Replaces the reference's single-channel driver loop (src/qpsk.c:436-458,
 * which calls qpsk_rx_frame() once per 1880-sample frame, src/qpsk.c:447)
 * with one call over many independent channels.  Each channel behaves exactly
 * like a fresh run of the reference receiver fed that channel's stream; the
 * per-channel state the reference keeps in statics (src/qpsk.c:37-53,
 * src/kalman.c:19-35, src/scramble.c:41-42) lives in the context and persists
 * across calls, so a stream may be fed in any number of calls.
 *
 * Layouts (row-major, little endian):
 *   in     int16  [nch][nframes][1880]   raw 8 kHz samples (reference .raw framing)
 *   bits   uint8  [nch][nframes][62]     0/1 per bit, reference order
 *                                         (bits[2s] = Q, bits[2s+1] = I, descrambled);
 *                                         all zero for invalid frames
 *   valid  uint8  [nch][nframes]         qpsk_rx_frame() return value
 *   trace  int32  [nch][nframes][4]      optional: max_index, matches, valid,
 *                                         rx_timing after the frame
 *   soft   float  [nch][nframes][31][2]  optional: data_eq soft symbols (valid
 *                                         frames; zero otherwise)
 * Any optional pointer may be NULL.
 *
 * Errors: functions return 0 on success or a negative QPSK_E* code; HIP errors
 * are QPSK_EHIP - (int)hipError_t.  Contexts are independent and may be used
 * from different host threads; one context must not be used concurrently.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qpsk_ctx qpsk_ctx;

enum {
    QPSK_OK = 0,
    QPSK_EINVAL = -1,     /* bad argument (NULL ctx/in, nch < 1, nframes < 0,
                             nch * nframes >= 2^28 in one call: 1 TB of input) */
    QPSK_ENOMEM = -2,     /* device or host allocation failed */
    QPSK_ENODEV = -3,     /* no such HIP device */
    QPSK_EBUSY = -4,      /* qpsk_stream_acquire() with every slot in flight, or
                             qpsk_rx_reset() / qpsk_rx_state_load() on a stream's
                             context while chunks are pending: retrieve first */
    QPSK_ESTALL = -5,     /* a device-side progress wait of rx_kernel's dual-chain
                             shapes exceeded its bound (~0.1 s): the outputs of
                             the calls since the previous check are undefined.
                             Never expected; it turns a logic error into an
                             error code instead of a hung GPU or wrong bits. */
    QPSK_EHIP = -1000,    /* QPSK_EHIP - hipError_t */
};

/* Receiver semantics of a context. */
enum {
    QPSK_MODE_REFERENCE = 0,  /* bit-identical to the reference as built (gcc -O2:
                                 the decimated_frame[562] overflow of
                                 src/qpsk.c:157-162 aliases input_frame) */
    QPSK_MODE_DEC752 = 1,     /* "intended semantics": decimated_frame with the
                                 752 entries its loop writes.  A working receiver
                                 variant, NOT reference parity; equal to the
                                 unmodified reference sources linked with that
                                 array padded (oracle/ref/dec752.ld) */
    QPSK_MODE_FFT_HUNT = 2,   /* flag, combinable with either of the above: the
                                 preamble hunt correlates through the reference's
                                 kiss_fft (src/fft.c, which the reference never
                                 calls): S = ifft(fft(dec[0..255]) * conj(fft(c))),
                                 c = conj(preambletable) zero-padded to 256, then
                                 the hunt loop of src/qpsk.c:172-183 over
                                 cnormf(S[l]).  Not reference parity. */
};

/* Create a receiver for nch channels on HIP device `device`, in the reference's
 * initial RX state (src/qpsk.c:427-434).  Returns NULL on failure; *err (if
 * non-NULL) receives the error code.  qpsk_rx_create() is
 * qpsk_rx_create_mode(device, nch, QPSK_MODE_REFERENCE, err). */
qpsk_ctx *qpsk_rx_create(int device, int nch, int *err);
qpsk_ctx *qpsk_rx_create_mode(int device, int nch, int mode, int *err);
void qpsk_rx_destroy(qpsk_ctx *ctx);
/* Back to the initial state (all channels), as after qpsk_rx_create.  Waits
 * for the context's calls in flight first (they read the state it clears).
 * On the context of a qpsk_stream (qpsk_stream_ctx) it returns QPSK_EBUSY
 * while the stream has chunks submitted and not retrieved: drain the stream
 * (qpsk_stream_retrieve until qpsk_stream_pending is 0), then reset. */
int qpsk_rx_reset(qpsk_ctx *ctx);
int qpsk_rx_channels(const qpsk_ctx *ctx);
/* QPSK_MODE_* of the context. */
int qpsk_rx_mode(const qpsk_ctx *ctx);
/* Frames received so far by every channel of the context. */
uint64_t qpsk_rx_frames(const qpsk_ctx *ctx);

/* Per-channel state checkpoint / resume.  Between frames the
 * reference carries, per channel, rx_timing (src/qpsk.c:53), the decimated
 * symbols D_{n-1} and the sample history in its statics (decimated_frame /
 * input_frame, src/qpsk.c:40-42) and the descrambler register
 * (src/scramble.c:41-42, a function of the frame index).  The context holds
 * the equivalent per channel in device memory: the history of the last two
 * frames, the next frame's equalizer window (dec[mi .. mi+166]) with its
 * preamble position, and rx_timing; the frame index is the context's.
 *
 *   qpsk_rx_state_size(n)        bytes of a snapshot of n channels
 *   qpsk_rx_state_save(ctx, c0, n, buf, size)
 *                                channels [c0, c0 + n) -> buf (host memory)
 *   qpsk_rx_state_load(ctx, c0, n, buf, size)
 *                                buf -> channels [c0, c0 + n) of ctx
 *
 * A snapshot records the context's mode and frame index.  Loading it into a
 * context of the same mode (on any device, in any process) continues those
 * channels exactly where they stopped: demodulating 7 frames, saving,
 * loading into a fresh context and demodulating 9 more gives the outputs of
 * one 16-frame call.  The frame index is shared by all channels of a
 * context: a context takes the snapshot's index when it has received no
 * frame since create/reset (qpsk_rx_frames() == 0); otherwise the indices
 * must be equal (QPSK_EINVAL).  Loading fewer than all channels into such a
 * fresh context from a snapshot at frame G != 0 moves every channel to frame
 * G, so the context then receives nothing (qpsk_rx_batch*, streams, state
 * saves: QPSK_EINVAL) until each of its channels has been loaded from
 * snapshots at G (any number of ranges, in any order); qpsk_rx_reset()
 * abandons such an assembly.  Both calls wait for the context's calls in
 * flight; on a stream's context they return QPSK_EBUSY while chunks are
 * pending.  n snapshots' channel ranges may differ from the ones loaded into
 * (channel c0 + i of the snapshot goes to channel c0' + i).
 * qpsk_rx_state_save returns QPSK_ESTALL once any call of the context has
 * stalled since create/reset (reported, or still in the device error word,
 * which it reads without taking): that state is undefined.  A snapshot is a
 * function of the channels' state alone (window slots past the last one the
 * equalizer reads are zero). */
size_t qpsk_rx_state_size(int n);
int qpsk_rx_state_save(qpsk_ctx *ctx, int c0, int n, void *buf, size_t size);
int qpsk_rx_state_load(qpsk_ctx *ctx, int c0, int n, const void *buf, size_t size);

/* Host-memory call: copies `in` to the device, demodulates nframes frames of
 * every channel, copies the results back and synchronises; returns
 * qpsk_rx_sync()'s verdict. */
int qpsk_rx_batch(qpsk_ctx *ctx, const int16_t *in, int nframes, uint8_t *bits,
                  uint8_t *valid, int32_t *trace, float *soft);

/* Device-memory call: all pointers are device pointers on the context's device;
 * the work is enqueued on `stream` (a hipStream_t, NULL = default stream) and
 * the call returns without synchronising.  Launches two kernels: rx_kernel
 * (every stage of every frame, persistent over the call's frames) and
 * rx_data_kernel (the 31 data symbols of the valid frames); see DESIGN.md. */
int qpsk_rx_batch_device(qpsk_ctx *ctx, const int16_t *d_in, int nframes,
                         uint8_t *d_bits, uint8_t *d_valid, int32_t *d_trace,
                         float *d_soft, void *stream);

/* Waits for the context's latest qpsk_rx_batch_device call (an event recorded
 * on its stream after its kernels; the stream itself may since be destroyed)
 * and returns QPSK_ESTALL if any call since the previous check reported a
 * device-side failure, else 0.  The device error word is sticky until this
 * reads it, and is read and cleared in one atomic exchange.  Calls on one
 * context depend on each other through the per-channel state, so the caller
 * orders them (one stream, or streams it chains). */
int qpsk_rx_sync(qpsk_ctx *ctx);

/* Kernel-time accounting.  When enabled, every qpsk_rx_batch_device call
 * records HIP events on its stream before rx_kernel, between the two kernels
 * and after rx_data_kernel.  collect() waits for them and returns the summed
 * span of both kernels (ms) and the number of frames demodulated since the
 * previous collect; split() returns the two kernels' spans separately. */
int qpsk_rx_timing_enable(qpsk_ctx *ctx, int on);
int qpsk_rx_timing_collect(qpsk_ctx *ctx, float *ms, int *frames);
int qpsk_rx_timing_split(qpsk_ctx *ctx, float *ms_rx, float *ms_data, int *frames);

/* Message for an error code (static storage). */
const char *qpsk_strerror(int err);

/* Provenance of the receive kernels in this library: the first 16 hex digits of
 * the sha256 of their sources and build rules (singlecarrier_amd/csrc/Makefile
 * KSRC).  Profiled counters record it; bench.py reports them only for a
 * library with the same hash. */
const char *qpsk_kernel_hash(void);

#ifdef __cplusplus
}
#endif
