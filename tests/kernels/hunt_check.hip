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

// The product's whole hunt decision (qhunt::hunt_index: bf16 pass, exact chain
// when in doubt) on given decimated frames: out_idx[i] = max_index, out_fb[i] =
// 1 when the exact chain decided.  tests/test_gpu_hunt.py compares max_index
// with the reference's scan (src/qpsk.c:172-183) over its sequential sums.
__global__ void __launch_bounds__(64) hunt_pick_kernel(const float2* dec, int* out_idx, int* out_fb) {
    __shared__ __attribute__((aligned(16))) float TB[qhunt::kBH + qhunt::kPL];
    __shared__ __attribute__((aligned(16))) float S[qhunt::kTK > qhunt::kHBytes / 4 ? qhunt::kTK : qhunt::kHBytes / 4];
    __shared__ __attribute__((aligned(16))) float2 D[256];
    const int lane = threadIdx.x;
    qhunt::bconst_h_lds(lane, 64, TB);
    const float2* d = dec + (size_t)blockIdx.x * 256;
    for (int j = lane; j < 256; j += 64) D[j] = d[j];
    __syncthreads();
    bool fb;
    const int mi = qhunt::hunt_index(lane, D, S, TB, qhunt::wave_max_u32, fb);
    if (lane == 0) {
        out_idx[blockIdx.x] = mi;
        out_fb[blockIdx.x] = fb ? 1 : 0;
    }
}

// dec: [n][256] float2 (entry 255 unused); out_idx, out_fb: [n]
extern "C" int hunt_pick(const float2* dec, int n, int* out_idx, int* out_fb) {
    float2* d_dec;
    int *d_idx, *d_fb;
    if (hipMalloc(&d_dec, sizeof(float2) * 256 * n) != hipSuccess) return -1;
    if (hipMalloc(&d_idx, sizeof(int) * n) != hipSuccess) return -1;
    if (hipMalloc(&d_fb, sizeof(int) * n) != hipSuccess) return -1;
    (void)hipMemcpy(d_dec, dec, sizeof(float2) * 256 * n, hipMemcpyHostToDevice);
    hunt_pick_kernel<<<n, 64>>>(d_dec, d_idx, d_fb);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out_idx, d_idx, sizeof(int) * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(out_fb, d_fb, sizeof(int) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_dec);
    (void)hipFree(d_idx);
    (void)hipFree(d_fb);
    return 0;
}

// The bf16 pass alone (qhunt::store_h + correlate_h): every lag's (re, im)
// approximate sum and the window's W, so tests/test_gpu_hunt.py can measure
// |S' - S| / W on the hardware against the budget qpsk_hunt.h derives.
__global__ void __launch_bounds__(64) hunt_h_kernel(const float2* dec, float2* out, float* out_w) {
    __shared__ __attribute__((aligned(16))) float TB[qhunt::kBH + qhunt::kPL];
    __shared__ __attribute__((aligned(16))) float S[qhunt::kHBytes / 4];
    __shared__ __attribute__((aligned(16))) float2 D[256];
    const int lane = threadIdx.x;
    qhunt::bconst_h_lds(lane, 64, TB);
    const float2* d = dec + (size_t)blockIdx.x * 256;
    for (int j = lane; j < 256; j += 64) D[j] = d[j];
    __syncthreads();
    const float W = qhunt::wave_sum_f32(qhunt::store_h(lane, D, reinterpret_cast<char*>(S)));
    qhunt::lds_sync();
    const qhunt::f4 acc = qhunt::correlate_h(lane, reinterpret_cast<const char*>(S), TB);
    float2* o = out + (size_t)blockIdx.x * QK_NLAG;
    o[qhunt::lag_lo(lane)] = make_float2(acc[0], acc[1]);
    o[qhunt::lag_hi(lane)] = make_float2(acc[2], acc[3]);
    if (lane == 0) out_w[blockIdx.x] = W;
}

extern "C" int hunt_h(const float2* dec, int n, float2* out, float* out_w) {
    float2 *d_dec, *d_out;
    float* d_w;
    if (hipMalloc(&d_dec, sizeof(float2) * 256 * n) != hipSuccess) return -1;
    if (hipMalloc(&d_out, sizeof(float2) * QK_NLAG * n) != hipSuccess) return -1;
    if (hipMalloc(&d_w, sizeof(float) * n) != hipSuccess) return -1;
    (void)hipMemcpy(d_dec, dec, sizeof(float2) * 256 * n, hipMemcpyHostToDevice);
    hunt_h_kernel<<<n, 64>>>(d_dec, d_out, d_w);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out, d_out, sizeof(float2) * QK_NLAG * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(out_w, d_w, sizeof(float) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_dec);
    (void)hipFree(d_out);
    (void)hipFree(d_w);
    return 0;
}
