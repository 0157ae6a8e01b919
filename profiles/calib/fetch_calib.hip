// fetch_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shapes rx_kernel uses (known byte counts, one kernel each):
//   k_vec16   coalesced 16 B/lane loads           (the guide's x2 case)
//   k_dword   coalesced 4 B/lane loads            (front-wave input items)
//   k_rows_nt lane-per-row 8 B/step nt loads over 1344-B rows (back-wave window)
//   k_rows    the same with plain loads
//   k_store16 coalesced 16 B/lane stores
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void k_vec16(const float4* p, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i].x + p[i].w;
    if (acc == 1234.5f) *sink = acc;
}
__global__ void k_dword(const int* p, size_t n, float* sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 12345) *sink = (float)acc;
}
// rows of 168 float2; each lane walks its row 8 B per step (163 steps), like back_frame
template <bool NT>
__global__ void k_rows(const f32x2* w, int nrows, float* sink) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    const f32x2* r = w + (size_t)row * 168;
    f32x2 acc = {0.f, 0.f};
    for (int s = 1; s < 164; s++) {
        f32x2 v = NT ? __builtin_nontemporal_load(r + s) : r[s];
        acc = acc * 0.5f + v;   // dependent chain ~ a Kalman step between loads
        acc = acc * 0.5f + v;
    }
    if (acc.x == 1234.5f) *sink = acc.y;
}
__global__ void k_store16(float4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

int main() {
    const size_t bytes = 1ull << 30;
    void* buf;
    float* sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    const int nrows = 65536 * 4;   // 352 MB of rows, beyond the 256 MB Infinity Cache
    for (int rep = 0; rep < 2; rep++) {
        k_vec16<<<4096, 256>>>((const float4*)buf, bytes / 16, sink);
        k_dword<<<4096, 256>>>((const int*)buf, bytes / 4, sink);
        k_rows<true><<<nrows / 64, 64>>>((const f32x2*)buf, nrows > (int)(bytes / 1344) ? (int)(bytes / 1344) : nrows, sink);
        k_rows<false><<<nrows / 64, 64>>>((const f32x2*)buf, nrows > (int)(bytes / 1344) ? (int)(bytes / 1344) : nrows, sink);
        k_store16<<<4096, 256>>>((float4*)buf, bytes / 16);
    }
    (void)hipDeviceSynchronize();
    printf("bytes=%zu rows=%d row_bytes_read=%d\n", bytes, nrows, 163 * 8);
    return 0;
}
