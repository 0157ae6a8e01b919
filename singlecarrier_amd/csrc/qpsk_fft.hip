// qpsk_fft.hip -- batched GPU kiss_fft (include/qpsk_fft.h): one wave per
// transform, the points in LDS, the reference's stages (qpsk_fft_dev.h).
#include <hip/hip_runtime.h>

#include <new>
#include <stdint.h>
#include <stdlib.h>

#include "qpsk_fft.h"
#include "qpsk_fft_dev.h"
#include "qpsk_fft_tables.h"

namespace {

// in [batch][N] -> out [batch][N]; a copy through LDS first, so in may be out
__global__ void __launch_bounds__(64) fft_kernel(const qfft::cf* in, qfft::cf* out, const int* perm,
                                                 const qfft::cf* tw, int N, int inverse) {
    extern __shared__ qfft::cf buf[];
    const int lane = threadIdx.x;
    const size_t b = blockIdx.x;
    for (int pos = lane; pos < N; pos += 64) buf[pos] = in[b * N + perm[pos]];   // kf_work leaves
    qfft::lds_sync();
    qfft::stages(lane, N, buf, tw, inverse != 0);
    for (int pos = lane; pos < N; pos += 64) out[b * N + pos] = buf[pos];
}

int herr(hipError_t e) { return e == hipSuccess ? QPSK_OK : QPSK_EHIP - (int)e; }

}  // namespace

#define FCHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return herr(e_); } while (0)

struct qpsk_fft_plan {
    int device = 0, nfft = 0, inverse = 0;
    int* d_perm = nullptr;
    qfft::cf* d_tw = nullptr;
    hipStream_t stream = nullptr;
    qfft::cf* s_buf = nullptr;   // staging of the host entry point
    size_t s_cap = 0;
};

static void plan_release(qpsk_fft_plan* p) {
    (void)hipFree(p->d_perm);
    (void)hipFree(p->d_tw);
    (void)hipFree(p->s_buf);
    if (p->stream) (void)hipStreamDestroy(p->stream);
}

extern "C" qpsk_fft_plan* qpsk_fft_alloc(int device, int nfft, int inverse, int* err) {
    int dummy;
    if (!err) err = &dummy;
    if (nfft < 4 || nfft > 4096 || (nfft & (nfft - 1)) != 0) { *err = QPSK_EINVAL; return nullptr; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        *err = QPSK_ENODEV;
        return nullptr;
    }
    qpsk_fft_plan* p = new (std::nothrow) qpsk_fft_plan();
    int* perm = (int*)malloc(sizeof(int) * nfft);
    float* tw = (float*)malloc(sizeof(float) * 2 * nfft);
    if (!p || !perm || !tw) {
        delete p;
        free(perm);
        free(tw);
        *err = QPSK_ENOMEM;
        return nullptr;
    }
    p->device = device;
    p->nfft = nfft;
    p->inverse = inverse != 0;
    qpsk_fft_perm_table(nfft, perm);
    qpsk_fft_twiddle_table(nfft, p->inverse, tw);
    int r = herr(hipSetDevice(device));
    if (r == QPSK_OK) r = herr(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    if (r == QPSK_OK) r = herr(hipMalloc(&p->d_perm, sizeof(int) * nfft));
    if (r == QPSK_OK) r = herr(hipMalloc(&p->d_tw, sizeof(qfft::cf) * nfft));
    if (r == QPSK_OK) r = herr(hipMemcpy(p->d_perm, perm, sizeof(int) * nfft, hipMemcpyHostToDevice));
    if (r == QPSK_OK) r = herr(hipMemcpy(p->d_tw, tw, sizeof(qfft::cf) * nfft, hipMemcpyHostToDevice));
    free(perm);
    free(tw);
    if (r != QPSK_OK) {
        plan_release(p);
        delete p;
        *err = r;
        return nullptr;
    }
    *err = QPSK_OK;
    return p;
}

extern "C" void qpsk_fft_free(qpsk_fft_plan* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    (void)hipStreamSynchronize(p->stream);
    plan_release(p);
    delete p;
}

extern "C" int qpsk_fft_device(qpsk_fft_plan* p, const float* d_in, float* d_out, int batch,
                               void* stream) {
    if (!p || batch < 0 || (batch > 0 && (!d_in || !d_out))) return QPSK_EINVAL;
    if (batch == 0) return QPSK_OK;
    FCHECK(hipSetDevice(p->device));
    hipLaunchKernelGGL(fft_kernel, dim3(batch), dim3(64), sizeof(qfft::cf) * p->nfft,
                       (hipStream_t)stream, reinterpret_cast<const qfft::cf*>(d_in),
                       reinterpret_cast<qfft::cf*>(d_out), p->d_perm, p->d_tw, p->nfft, p->inverse);
    FCHECK(hipGetLastError());
    return QPSK_OK;
}

extern "C" int qpsk_fft(qpsk_fft_plan* p, const float* in, float* out, int batch) {
    if (!p || batch < 0 || (batch > 0 && (!in || !out))) return QPSK_EINVAL;
    if (batch == 0) return QPSK_OK;
    FCHECK(hipSetDevice(p->device));
    const size_t n = (size_t)batch * p->nfft;
    if (n > p->s_cap) {
        (void)hipFree(p->s_buf);
        p->s_buf = nullptr;
        p->s_cap = 0;
        FCHECK(hipMalloc(&p->s_buf, sizeof(qfft::cf) * n));
        p->s_cap = n;
    }
    FCHECK(hipMemcpyAsync(p->s_buf, in, sizeof(qfft::cf) * n, hipMemcpyHostToDevice, p->stream));
    int r = qpsk_fft_device(p, reinterpret_cast<const float*>(p->s_buf),
                            reinterpret_cast<float*>(p->s_buf), batch, p->stream);
    if (r != QPSK_OK) return r;
    FCHECK(hipMemcpyAsync(out, p->s_buf, sizeof(qfft::cf) * n, hipMemcpyDeviceToHost, p->stream));
    FCHECK(hipStreamSynchronize(p->stream));
    return QPSK_OK;
}
