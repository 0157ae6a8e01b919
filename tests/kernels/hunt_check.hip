// hunt_check.hip -- TEST ONLY: runs the product's MFMA correlator
// (singlecarrier_amd/csrc/qpsk_hunt.h) on given decimated frames and returns
// every lag's complex sum, so tests/test_gpu_hunt.py can compare it bit for bit
// with the reference's sequential sum (src/qpsk.c:88-96) computed on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qpsk_hunt.h"

#pragma clang fp contract(off)

__global__ void __launch_bounds__(64) hunt_check_kernel(const float2* dec, float2* out) {
    __shared__ __attribute__((aligned(16))) float TK[qhunt::kTK];
    const int lane = threadIdx.x;
    const float2* d = dec + (size_t)blockIdx.x * 256;
    float B[qhunt::kSteps];
    qhunt::bconst(lane, B);
    qhunt::store_t(lane, d, TK);
    __syncthreads();
    const qhunt::f4 acc = qhunt::correlate(lane, TK, B);
    float2* o = out + (size_t)blockIdx.x * QK_NLAG;
    o[qhunt::lag_lo(lane)] = make_float2(acc[0], acc[1]);
    o[qhunt::lag_hi(lane)] = make_float2(acc[2], acc[3]);
}

// dec: [n][256] float2 (entries 255.. unused), out: [n][128] float2 sums
extern "C" int hunt_check(const float2* dec, int n, float2* out) {
    float2 *d_dec, *d_out;
    if (hipMalloc(&d_dec, sizeof(float2) * 256 * n) != hipSuccess) return -1;
    if (hipMalloc(&d_out, sizeof(float2) * QK_NLAG * n) != hipSuccess) return -1;
    (void)hipMemcpy(d_dec, dec, sizeof(float2) * 256 * n, hipMemcpyHostToDevice);
    hunt_check_kernel<<<n, 64>>>(d_dec, d_out);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out, d_out, sizeof(float2) * QK_NLAG * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_dec);
    (void)hipFree(d_out);
    return 0;
}
