// qpsk_stream.hip -- streaming ingest (include/qpsk_stream.h): host chunks in
// pinned slots, H2D / receive / D2H on three HIP streams so consecutive chunks
// overlap.  Host code only; the receive is qpsk_rx_batch_device().
#include <hip/hip_runtime.h>

#include <new>
#include <stdint.h>
#include <string.h>

#include "qpsk_batch.h"
#include "qpsk_consts.h"
#include "qpsk_rx_internal.h"
#include "qpsk_stream.h"

namespace {

constexpr int kMaxSlots = 4;

struct Slot {
    int16_t* h_in = nullptr;     // pinned
    int16_t* d_in = nullptr;
    uint8_t* d_bits = nullptr;
    uint8_t* d_valid = nullptr;
    uint8_t* h_bits = nullptr;   // pinned
    uint8_t* h_valid = nullptr;  // pinned
    int* d_err = nullptr;        // the chunk's device error word (progress-wait stalls)
    int* h_err = nullptr;        // pinned copy, read by qpsk_stream_retrieve
    hipEvent_t copied = nullptr, received = nullptr, done = nullptr;
    uint64_t epoch = 0;          // qpsk_rx_epoch() when the chunk was submitted
};

int herr(hipError_t e) { return e == hipSuccess ? QPSK_OK : QPSK_EHIP - (int)e; }

// a slot's stall also goes into the context's own error word (qpsk_rx_sync)
__global__ void err_merge_kernel(int* ctx_err, const int* slot_err) {
    if (threadIdx.x == 0 && *slot_err != 0) atomicOr(ctx_err, *slot_err);
}

}  // namespace

struct qpsk_stream {
    int device = 0, nch = 0, frames = 0, nslot = 0;
    qpsk_ctx* rx = nullptr;
    hipStream_t s_h2d = nullptr, s_rx = nullptr, s_d2h = nullptr;
    Slot slot[kMaxSlots];
    uint64_t acquired = 0, submitted = 0, retrieved = 0;
    // A stalled chunk leaves every channel's carried state (rx_timing, windows,
    // history) undefined, so every later chunk of the same epoch (submitted
    // before the next qpsk_rx_reset() on the stream's context) is reported
    // QPSK_ESTALL too.  Chunks are retrieved in submission order, so when a
    // chunk is retrieved every earlier chunk's stall is known.
    bool stalled = false;
    uint64_t stall_epoch = 0;
};

#define SCHECK(x) do { const hipError_t e_ = (x); if (e_ != hipSuccess) return herr(e_); } while (0)

static void stream_free(qpsk_stream* s) {
    (void)hipSetDevice(s->device);
    for (int i = 0; i < s->nslot; i++) {
        Slot& q = s->slot[i];
        (void)hipHostFree(q.h_in);
        (void)hipHostFree(q.h_bits);
        (void)hipHostFree(q.h_valid);
        (void)hipHostFree(q.h_err);
        (void)hipFree(q.d_err);
        (void)hipFree(q.d_in);
        (void)hipFree(q.d_bits);
        (void)hipFree(q.d_valid);
        if (q.copied) (void)hipEventDestroy(q.copied);
        if (q.received) (void)hipEventDestroy(q.received);
        if (q.done) (void)hipEventDestroy(q.done);
    }
    if (s->s_h2d) (void)hipStreamDestroy(s->s_h2d);
    if (s->s_rx) (void)hipStreamDestroy(s->s_rx);
    if (s->s_d2h) (void)hipStreamDestroy(s->s_d2h);
    if (s->rx) qpsk_rx_destroy(s->rx);
}

static int stream_alloc(qpsk_stream* s) {
    SCHECK(hipSetDevice(s->device));
    SCHECK(hipStreamCreateWithFlags(&s->s_h2d, hipStreamNonBlocking));
    SCHECK(hipStreamCreateWithFlags(&s->s_rx, hipStreamNonBlocking));
    SCHECK(hipStreamCreateWithFlags(&s->s_d2h, hipStreamNonBlocking));
    const size_t cf = (size_t)s->nch * (size_t)s->frames;
    for (int i = 0; i < s->nslot; i++) {
        Slot& q = s->slot[i];
        SCHECK(hipHostMalloc((void**)&q.h_in, sizeof(int16_t) * cf * QK_FRAME, hipHostMallocDefault));
        SCHECK(hipHostMalloc((void**)&q.h_bits, cf * QK_NBITS, hipHostMallocDefault));
        SCHECK(hipHostMalloc((void**)&q.h_valid, cf, hipHostMallocDefault));
        SCHECK(hipMalloc((void**)&q.d_in, sizeof(int16_t) * cf * QK_FRAME));
        SCHECK(hipMalloc((void**)&q.d_bits, cf * QK_NBITS));
        SCHECK(hipMalloc((void**)&q.d_valid, cf));
        SCHECK(hipMalloc((void**)&q.d_err, sizeof(int)));
        SCHECK(hipHostMalloc((void**)&q.h_err, sizeof(int), hipHostMallocDefault));
        SCHECK(hipEventCreateWithFlags(&q.copied, hipEventDisableTiming));
        SCHECK(hipEventCreateWithFlags(&q.received, hipEventDisableTiming));
        SCHECK(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
    }
    return QPSK_OK;
}

extern "C" qpsk_stream* qpsk_stream_create(int device, int nch, int frames, int nslot, int* err) {
    return qpsk_stream_create_mode(device, nch, frames, nslot, QPSK_MODE_REFERENCE, err);
}

extern "C" qpsk_stream* qpsk_stream_create_mode(int device, int nch, int frames, int nslot,
                                                int mode, int* err) {
    int dummy;
    if (!err) err = &dummy;
    if (nch < 1 || frames < 1 || nslot < 1 || nslot > kMaxSlots) {
        *err = QPSK_EINVAL;
        return nullptr;
    }
    qpsk_stream* s = new (std::nothrow) qpsk_stream();
    if (!s) {
        *err = QPSK_ENOMEM;
        return nullptr;
    }
    s->device = device;
    s->nch = nch;
    s->frames = frames;
    s->nslot = nslot;
    s->rx = qpsk_rx_create_mode(device, nch, mode, err);
    if (s->rx) qpsk_rx_set_owner(s->rx, s);
    int r = s->rx ? stream_alloc(s) : *err;
    if (r != QPSK_OK) {
        stream_free(s);
        delete s;
        *err = r;
        return nullptr;
    }
    *err = QPSK_OK;
    return s;
}

extern "C" void qpsk_stream_destroy(qpsk_stream* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->s_h2d);
    (void)hipStreamSynchronize(s->s_rx);
    (void)hipStreamSynchronize(s->s_d2h);
    stream_free(s);
    delete s;
}

extern "C" int16_t* qpsk_stream_acquire(qpsk_stream* s, int* err) {
    int dummy;
    if (!err) err = &dummy;
    if (!s) {
        *err = QPSK_EINVAL;
        return nullptr;
    }
    if (s->acquired != s->submitted) {   // acquired twice without a submit
        *err = QPSK_OK;
        return s->slot[s->acquired % (uint64_t)s->nslot].h_in;
    }
    // the slot's previous chunk must have been retrieved (its outputs and its
    // input buffer are the caller's until then)
    if (s->acquired - s->retrieved >= (uint64_t)s->nslot) {
        *err = QPSK_EBUSY;
        return nullptr;
    }
    *err = QPSK_OK;
    return s->slot[s->acquired++ % (uint64_t)s->nslot].h_in;
}

extern "C" int qpsk_stream_submit(qpsk_stream* s) {
    if (!s || s->submitted == s->acquired) return QPSK_EINVAL;
    Slot& q = s->slot[s->submitted % (uint64_t)s->nslot];
    const size_t cf = (size_t)s->nch * (size_t)s->frames;
    SCHECK(hipSetDevice(s->device));
    SCHECK(hipMemcpyAsync(q.d_in, q.h_in, sizeof(int16_t) * cf * QK_FRAME, hipMemcpyHostToDevice,
                          s->s_h2d));
    SCHECK(hipEventRecord(q.copied, s->s_h2d));
    SCHECK(hipStreamWaitEvent(s->s_rx, q.copied, 0));
    SCHECK(hipMemsetAsync(q.d_err, 0, sizeof(int), s->s_rx));
    const int r = qpsk_rx_launch(s->rx, q.d_in, s->frames, q.d_bits, q.d_valid, nullptr, nullptr,
                                 s->s_rx, q.d_err);
    if (r != QPSK_OK) return r;
    hipLaunchKernelGGL(err_merge_kernel, dim3(1), dim3(64), 0, s->s_rx, qpsk_rx_err_word(s->rx), q.d_err);
    SCHECK(hipGetLastError());
    SCHECK(hipEventRecord(q.received, s->s_rx));
    SCHECK(hipStreamWaitEvent(s->s_d2h, q.received, 0));
    SCHECK(hipMemcpyAsync(q.h_bits, q.d_bits, cf * QK_NBITS, hipMemcpyDeviceToHost, s->s_d2h));
    SCHECK(hipMemcpyAsync(q.h_valid, q.d_valid, cf, hipMemcpyDeviceToHost, s->s_d2h));
    SCHECK(hipMemcpyAsync(q.h_err, q.d_err, sizeof(int), hipMemcpyDeviceToHost, s->s_d2h));
    SCHECK(hipEventRecord(q.done, s->s_d2h));
    q.epoch = qpsk_rx_epoch(s->rx);
    s->submitted++;
    return QPSK_OK;
}

extern "C" int qpsk_stream_pending(const qpsk_stream* s) {
    return s ? (int)(s->submitted - s->retrieved) : 0;
}

extern "C" int qpsk_stream_retrieve(qpsk_stream* s, const uint8_t** bits, const uint8_t** valid) {
    if (!s || !bits || !valid || s->retrieved == s->submitted) return QPSK_EINVAL;
    Slot& q = s->slot[s->retrieved % (uint64_t)s->nslot];
    SCHECK(hipSetDevice(s->device));
    SCHECK(hipEventSynchronize(q.done));
    *bits = q.h_bits;
    *valid = q.h_valid;
    s->retrieved++;
    // a progress wait of this chunk's receive ran out: its bits are undefined,
    // and so are those of every later chunk of its epoch, which start from the
    // state it left (the slot is released all the same).  The epoch is the
    // chunk's own, taken at submit: a chunk submitted before a reset that ran
    // on the stalled state stays ESTALL, one submitted after it is clean.
    if (*q.h_err != 0) {
        s->stalled = true;
        s->stall_epoch = q.epoch;
        qpsk_rx_mark_stalled(s->rx, q.epoch);   // the context's state too (qpsk_rx_state_save)
    }
    return (s->stalled && q.epoch == s->stall_epoch) ? QPSK_ESTALL : QPSK_OK;
}

extern "C" qpsk_ctx* qpsk_stream_ctx(qpsk_stream* s) { return s ? s->rx : nullptr; }

// qpsk_records(): host C, qpsk_records.c
