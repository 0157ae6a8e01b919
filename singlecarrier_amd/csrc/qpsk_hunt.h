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

#include <utility>

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
// B = 0 only), written into the TK image.  Lane l handles j = 4l .. 4l+3, i.e.
// column l of all eight rows: the 32 lanes of a ds_write_b32 then hit 32
// distinct banks (rows are 0 mod 32 dwords apart, so j = l + 64r put four
// lanes on one bank); dec[4l .. 4l+3] arrive as two 16-B reads.
__device__ __forceinline__ void store_t(int lane, const float2* dec, float* TK) {
    const float4* d4 = reinterpret_cast<const float4*>(dec + 4 * lane);
    const float4 p = d4[0], q = d4[1];
    const float dr[4] = {p.x, p.z, q.x, q.z}, di[4] = {p.y, p.w, q.y, q.w};
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = 4 * lane + r;
        float tr = 0.0f, ti = 0.0f;
        if (j < 2 * QK_NLAG - 1) {
            tr = dr[r] - di[r];
            ti = di[r] + dr[r];
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

// ------------------------------------------------------------ VALU form
// The same k-ordered chains on the vector ALU.  An f32 MFMA occupies its
// SIMD's VALU for its whole issue time: beside a dependent
// v_mfma_f32_16x16x4_f32 chain another wave's v_pk_add_f32 stream slows from
// 5.0 to 13.0 cycles per instruction (profiles/calib/mfma_mix_r02.txt), so
// the 36 MFMAs per channel (~1,150 SIMD cycles) cost every wave on the SIMD.
// Here lane l owns lags 2l and 2l+1; step k adds p_k * T[2l+k] and
// p_k * T[2l+1+k] with one v_pk_add_f32 each ((re, im) packed; p_k = -1 is a
// negation modifier: RN(acc - T) == fmaf(-1, T, acc)).  One 16-B LDS read of
// (T[2l+k], T[2l+k+1]) (k even) serves both lags for two steps: 65 reads and
// 256 packed adds per channel.
constexpr int kTV = 256;            // float2 per T image (2 KB)

// TV[j] = T[j] = (RN(dr - di), RN(di + dr)) for j < 255, TV[255] = 0.
// Lane l handles j = l + 64r: 8-B reads and writes at 8-B lane stride.
__device__ __forceinline__ void store_tv(int lane, const float2* dec, float2* TV) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = lane + 64 * r;
        float tr = 0.0f, ti = 0.0f;
        if (j < 2 * QK_NLAG - 1) {
            const float2 d = dec[j];
            tr = d.x - d.y;
            ti = d.y + d.x;
        }
        TV[j] = make_float2(tr, ti);
    }
}

typedef float v2 __attribute__((ext_vector_type(2)));

template <bool NEG>
__device__ __forceinline__ v2 acc_add(v2 a, v2 t) {
    v2 r;
    if (NEG) asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(t));
    else asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(t));
    return r;
}

template <int K>
__device__ __forceinline__ v2 acc_step(v2 a, v2 t) {
    constexpr unsigned long long m = K < 64 ? pre_mask(0) : pre_mask(1);
    return acc_add<((m >> (K & 63)) & 1ull) == 0>(a, t);
}

template <int... I>
__device__ __forceinline__ void chain_valu(const f4* src, v2& a0, v2& a1,
                                           std::integer_sequence<int, I...>) {
    // step pair (2i, 2i+1): q = (T[2l+2i], T[2l+2i+1]), n = (T[2l+2i+2], ..)
    f4 q = src[0];
    auto pair = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const f4 n = src[i + 1];
        a0 = acc_step<2 * i>(a0, v2{q.x, q.y});
        a1 = acc_step<2 * i>(a1, v2{q.z, q.w});
        a0 = acc_step<2 * i + 1>(a0, v2{q.z, q.w});
        a1 = acc_step<2 * i + 1>(a1, v2{n.x, n.y});
        q = n;
    };
    (pair(std::integral_constant<int, I>{}), ...);
}

// Returns (re, im) of lag 2l in [0], [1] and of lag 2l+1 in [2], [3].
__device__ __forceinline__ f4 correlate_valu(int lane, const float2* TV) {
    const f4* src = reinterpret_cast<const f4*>(TV + 2 * lane);
    v2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f};
    chain_valu(src, a0, a1, std::make_integer_sequence<int, QK_NPRE / 2>{});
    return f4{a0.x, a0.y, a1.x, a1.y};
}

__device__ __forceinline__ int lag_lo_valu(int lane) { return 2 * lane; }
__device__ __forceinline__ int lag_hi_valu(int lane) { return 2 * lane + 1; }

}  // namespace qhunt
