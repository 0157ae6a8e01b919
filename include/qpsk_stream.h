/*
 * qpsk_stream.h -- streaming ingest for the batched receiver: host-resident
 * input arriving chunk by chunk (the reference's .raw framing, src/qpsk.c:
 * 436-458 reads 1880-sample frames from a file), pipelined over PCIe.
 *
 * A stream owns one qpsk_ctx (include/qpsk_batch.h) and `nslot` chunk slots.
 * Each slot has a pinned host input buffer int16 [nch][frames][1880] that the
 * caller fills in place (no extra copy), device buffers, and pinned host
 * output buffers bits u8 [nch][frames][62] / valid u8 [nch][frames].
 * Submitting a chunk enqueues H2D (copy stream) -> receive (compute stream)
 * -> D2H (copy-back stream), so the copy of chunk k+1 overlaps the receive
 * of chunk k.  Chunks are received in submission order and every channel's
 * state carries from one chunk to the next, exactly as one qpsk_rx_batch()
 * call over the concatenated frames.
 *
 *   s = qpsk_stream_create(dev, nch, frames, 3, &err);
 *   loop: in = qpsk_stream_acquire(s);  fill in[c][f][t];  qpsk_stream_submit(s);
 *         when qpsk_stream_pending(s) == nslot (or at the end):
 *             qpsk_stream_retrieve(s, &bits, &valid);   consume; (valid until the
 *                                                      slot is acquired again)
 *   qpsk_stream_destroy(s);
 *
 * Output records: qpsk_records() writes the reference driver's 496-byte record
 * per valid frame (bits in bytes 0..61, zero elsewhere; src/qpsk.c:455-457).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "qpsk_batch.h"   /* qpsk_ctx, QPSK_E* (QPSK_EBUSY = -4) */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qpsk_stream qpsk_stream;

qpsk_stream *qpsk_stream_create(int device, int nch, int frames, int nslot, int *err);
/* the same with the receiver semantics `mode` (QPSK_MODE_*, qpsk_batch.h) */
qpsk_stream *qpsk_stream_create_mode(int device, int nch, int frames, int nslot, int mode,
                                     int *err);
void qpsk_stream_destroy(qpsk_stream *s);
/* pinned input buffer of the next chunk, or NULL (*err = QPSK_EBUSY) */
int16_t *qpsk_stream_acquire(qpsk_stream *s, int *err);
/* enqueue the acquired chunk; returns 0 or a negative QPSK_E* code */
int qpsk_stream_submit(qpsk_stream *s);
/* chunks submitted and not yet retrieved */
int qpsk_stream_pending(const qpsk_stream *s);
/* wait for the oldest submitted chunk; *bits / *valid point into its pinned
 * output buffers (layouts as qpsk_rx_batch).  Returns QPSK_ESTALL (qpsk_batch.h)
 * when a device-side progress wait of that chunk's receive ran out: its
 * outputs are then undefined (the chunk counts as retrieved either way).  The
 * stall is sticky: every later chunk starts from the per-channel state the
 * stalled one left, so it is reported QPSK_ESTALL too -- every chunk submitted
 * before the next qpsk_rx_reset() on qpsk_stream_ctx(s).  A chunk's epoch is
 * taken when it is submitted, and the reset itself is refused (QPSK_EBUSY)
 * while chunks are pending, so a chunk that ran on the stalled state can
 * never come back QPSK_OK.  The stall also reaches the context's own
 * qpsk_rx_sync(). */
int qpsk_stream_retrieve(qpsk_stream *s, const uint8_t **bits, const uint8_t **valid);
/* the stream's receiver (e.g. for qpsk_rx_frames, or qpsk_rx_reset between
 * streams once qpsk_stream_pending(s) is 0: it returns QPSK_EBUSY before) */
struct qpsk_ctx *qpsk_stream_ctx(qpsk_stream *s);

/* One channel's outputs -> reference records: 496 bytes per valid frame.
 * Returns the bytes written to out (capacity >= 496 * nframes). */
size_t qpsk_records(const uint8_t *bits, const uint8_t *valid, int nframes, uint8_t *out);

#ifdef __cplusplus
}
#endif
