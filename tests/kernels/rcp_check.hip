// rcp_check.hip -- TEST ONLY: exhaustive check of qk_rcp_rn (qpsk_rcp.h)
// against IEEE fp32 division, over a range of float bit patterns.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qpsk_rcp.h"

#pragma clang fp contract(off)

__global__ void rcp_check_kernel(uint32_t lo, uint64_t n, unsigned long long* bad,
                                 uint32_t* first) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = lo + (uint32_t)i;
        const float x = __uint_as_float(u);
        const float a = qk_rcp_rn(x), b = 1.0f / x;
        const bool same = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
        if (!same) {
            atomicAdd(bad, 1ull);
            atomicMin(first, u);
        }
    }
}

// returns 0 on success; *bad = mismatches, *first = smallest mismatching pattern
extern "C" int rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    unsigned long long* d_bad;
    uint32_t* d_first;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 4) != hipSuccess) return -1;
    (void)hipMemset(d_bad, 0, 8);
    (void)hipMemset(d_first, 0xff, 4);
    const uint64_t n = (uint64_t)hi - lo + 1;
    rcp_check_kernel<<<8192, 256>>>(lo, n, d_bad, d_first);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first, d_first, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return 0;
}
