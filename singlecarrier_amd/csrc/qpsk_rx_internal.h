// qpsk_rx_internal.h -- entry points shared inside libqpsk_hip.so (not part of
// the C-ABI in include/).
#pragma once

#include <hip/hip_runtime.h>

#include "qpsk_batch.h"

// qpsk_rx_batch_device() with the device error word the call's progress waits
// report stalls to (nullptr: the context's own, which qpsk_rx_sync() takes).
// qpsk_stream.hip gives each stream slot its own word, so a stall is reported
// by qpsk_stream_retrieve() for the chunk it happened in.
// err_to (nullable): where rx_data_kernel stores the context's error word,
// taken in one atomic exchange once rx_kernel is done (host calls).
int qpsk_rx_launch(qpsk_ctx* c, const int16_t* d_in, int F, uint8_t* d_bits, uint8_t* d_valid,
                   int32_t* d_trace, float* d_soft, hipStream_t s, int* d_err, int* err_to = nullptr);

// The context's own device error word (qpsk_rx_sync() takes it): a stream
// slot's stall is OR-ed into it too, so the context sees every stall.
int* qpsk_rx_err_word(qpsk_ctx* c);
// Bumped by every qpsk_rx_reset(): a stream keeps reporting a stall for every
// later chunk until the per-channel state it corrupted has been reset.
uint64_t qpsk_rx_epoch(const qpsk_ctx* c);
// A stream chunk of epoch `epoch` stalled: if no reset has run since, the
// context's per-channel state is undefined (qpsk_rx_state_save refuses it).
void qpsk_rx_mark_stalled(qpsk_ctx* c, uint64_t epoch);

// The stream that owns a context (qpsk_stream_create_mode): qpsk_rx_reset()
// and qpsk_rx_state_load() refuse with QPSK_EBUSY while it has chunks pending.
struct qpsk_stream;
void qpsk_rx_set_owner(qpsk_ctx* c, const qpsk_stream* s);
extern "C" int qpsk_stream_pending(const qpsk_stream* s);
