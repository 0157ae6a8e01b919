// qpsk_rcp.h -- correctly rounded fp32 reciprocal for the Kalman gain update.
//
// kalman_calculate divides 1.0f by (a_j + ht) five times per step
// (src/kalman.c:162, 173).  The compiler's IEEE division expands to ~10
// instructions (div_scale x2, rcp, 4 fma, div_fmas, div_fixup).  For
// 2^-125 <= x <= 2^125, v_rcp_f32 followed by one FMA Newton step
//     r = rcp(x); e = fma(-x, r, 1); r = fma(e, r, r)
// returns the correctly rounded 1/x: tests/test_gpu_rcp.py checks it against
// IEEE division for EVERY positive finite float (a bit-exact statement, not a
// tolerance).  Outside that range (and for NaN) the exact division is used.
// The operands here are a_j + ht >= E = 0.1, so the fallback never runs in
// practice but keeps the function exact for all inputs.
#pragma once
#include <hip/hip_runtime.h>

// out of line: the (never taken in practice) exact path stays out of the hot
// loop's register allocation
__device__ __attribute__((noinline)) float qk_div_ieee(float x) { return 1.0f / x; }

// fast path only; callers check qk_rcp_in_range() on the operands themselves
__device__ __forceinline__ float qk_rcp_fast(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ bool qk_rcp_in_range(float lo, float hi) {
    return lo >= 0x1p-125f && hi <= 0x1p125f;   // false for NaN
}

__device__ __forceinline__ float qk_rcp_rn(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    if (__builtin_expect(!(x >= 0x1p-125f && x <= 0x1p125f), 0)) r = qk_div_ieee(x);
    return r;
}
