// qpsk_hunt.h -- the preamble hunt's 128-lag correlator on the matrix cores.
//
// Reference: correlate() src/qpsk.c:88-96 and the hunt loop :172-183.  For
// lag l < 128 the reference sums, in index order from 0,
//     S[l] = sum_{i<128} preambletable[i] * dec[l + i],   preambletable[i] = p_i + p_i j,
// with p_i = +-1 (src/qpsk.c:361-365), then takes cnormf(S[l]).  Because p_i is
// +-1 every complex product is exact up to one rounding:
//     p_i*(dr + di j)*(1 + j) = p_i * (RN(dr - di), RN(di + dr)) = p_i * T[l + i],
// so S[l] is the k-ordered chain acc = RN(acc + p_i * T) = fmaf(p_i, T, acc).
//
// gfx950's f32-input MFMA is bit-for-bit a k-ordered fmaf chain
// (cdna_hip_programming.md section 3, "FP32-input MFMA"; checked bitwise on the
// hardware by tests/test_gpu_hunt.py), so the whole correlator is a 16x16x144
// product on v_mfma_f32_16x16x4_f32 with NO change to any rounding:
//     D[m][n] = sum_{k<144} A[m][k] * B[k][n]
//     m = 2a + comp  (lag block a < 8, comp 0 = re / 1 = im),  n = b < 16,
//     lag l = 16a + b,  k = b + i,
//     A[m][k] = T_comp[16a + k],   B[k][n] = p_{k-n} if 0 <= k-n < 128 else 0.
// The k < n and k >= n + 128 terms add (+-0) to the running sum, which leaves a
// nonzero sum unchanged and a zero sum zero (sign of zero is unobservable: only
// the squares reach cnormf).  T must be finite everywhere (T * 0 must be 0):
// dec is a FIR of int16 input, |T| < 2^4.
//
// Operand layout (16x16x4 f32, cdna_hip_programming.md section 3): lane l holds
// A[l & 15][k = 4s + (l >> 4)] and B[4s + (l >> 4)][l & 15] for step s < 36; the
// result lane l holds D[4(l >> 4) + j][l & 15], j < 4, i.e. (re, im) of lag
// 32h + n (j = 0, 1) and of lag 32h + 16 + n (j = 2, 3), h = l >> 4, n = l & 15.
//
// LDS image of T ("TK"): row (kk, comp) = kk*2 + comp holds T_comp[4q + kk] at
// column q < 64, so lane l's 36 A-values for s = 0..35 are the contiguous
// columns 4a .. 4a+35 of row ((l >> 4), comp): nine 16-B reads.  Rows are
// kHuntRow floats apart (384 B = 128 mod 256) so the 16 lanes sharing a row pair
// (kk fixed) cover all 64 banks once.
#pragma once
#include <hip/hip_runtime.h>

#include "qpsk_consts.h"

namespace qhunt {

constexpr int kSteps = 36;          // K = 144 = 36 x 4
constexpr int kRow = 96;            // floats per TK row (64 used + 32 pad)
constexpr int kTK = 8 * kRow;       // floats per TK image (3 KB)

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr unsigned long long pre_mask(int half) {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i++)
        if (QK_PRE[half * 64 + i] > 0) m |= 1ull << i;
    return m;
}

// Constant B fragments of this lane for all 36 steps: p_{4s + kk - n} or 0.
__device__ __forceinline__ void bconst(int lane, float (&B)[kSteps]) {
    constexpr unsigned long long lo = pre_mask(0), hi = pre_mask(1);
    const int kk = lane >> 4, n = lane & 15;
#pragma unroll
    for (int s = 0; s < kSteps; s++) {
        const int i = 4 * s + kk - n;
        const unsigned long long m = i < 64 ? lo : hi;
        const float v = ((m >> (i & 63)) & 1ull) ? 1.0f : -1.0f;
        B[s] = (i >= 0 && i < QK_NPRE) ? v : 0.0f;
    }
}

// The B fragments as a shared LDS table (9 KB per workgroup, written once):
// BT[t][lane] = B[4t .. 4t+3] of that lane, read back as one 16-B load per 4
// steps (a kernel with no registers to spare keeps them here).
constexpr int kBT = kSteps * 64;    // floats
__device__ __forceinline__ void bconst_lds(int tid, int nthreads, float* BT) {
    for (int l = tid; l < 64; l += nthreads) {
        float B[kSteps];
        bconst(l, B);
#pragma unroll
        for (int t = 0; t < kSteps / 4; t++)
            reinterpret_cast<f4*>(BT)[t * 64 + l] = f4{B[4 * t], B[4 * t + 1], B[4 * t + 2], B[4 * t + 3]};
    }
}

// TK position of T_comp[j] (j < 256)
__device__ __forceinline__ int tk_index(int j, int comp) {
    return ((j & 3) * 2 + comp) * kRow + (j >> 2);
}

// T[j] = (RN(dr - di), RN(di + dr)) for j < 255 and T[255] = 0 (multiplied by
// B = 0 only), written into the TK image.  Lane l handles j = l + 64r.
__device__ __forceinline__ void store_t(int lane, const float2* dec, float* TK) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = lane + 64 * r;
        float tr = 0.0f, ti = 0.0f;
        if (j < 2 * QK_NLAG - 1) {
            const float2 d = dec[j];
            tr = d.x - d.y;
            ti = d.y + d.x;
        }
        TK[tk_index(j, 0)] = tr;
        TK[tk_index(j, 1)] = ti;
    }
}

// The 36-step chain.  Returns this lane's D fragment (see header comment).
__device__ __forceinline__ f4 correlate(int lane, const float* TK, const float (&B)[kSteps]) {
    const int m = lane & 15, kk = lane >> 4;
    const int a = m >> 1, comp = m & 1;
    const f4* src = reinterpret_cast<const f4*>(TK + (kk * 2 + comp) * kRow + 4 * a);
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < kSteps / 4; t++) {
        const f4 v = src[t];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, B[4 * t + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, B[4 * t + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.z, B[4 * t + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.w, B[4 * t + 3], acc, 0, 0, 0);
    }
    return acc;
}

// Same chain with B from the LDS table of bconst_lds().
__device__ __forceinline__ f4 correlate_bt(int lane, const float* TK, const float* BT) {
    const int m = lane & 15, kk = lane >> 4;
    const int a = m >> 1, comp = m & 1;
    const f4* src = reinterpret_cast<const f4*>(TK + (kk * 2 + comp) * kRow + 4 * a);
    const f4* bsrc = reinterpret_cast<const f4*>(BT) + lane;
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < kSteps / 4; t++) {
        const f4 v = src[t];
        const f4 b = bsrc[64 * t];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.z, b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.w, b.w, acc, 0, 0, 0);
    }
    return acc;
}

// lags held by this lane's fragment: (re, im) = (acc[0], acc[1]) and (acc[2], acc[3])
__device__ __forceinline__ int lag_lo(int lane) { return 32 * (lane >> 4) + (lane & 15); }
__device__ __forceinline__ int lag_hi(int lane) { return lag_lo(lane) + 16; }

}  // namespace qhunt
