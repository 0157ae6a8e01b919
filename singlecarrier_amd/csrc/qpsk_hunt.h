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

#ifndef QPSK_HUNT_OVERLAP
// 1: W's wave reduction after the MFMAs are issued (C3 -0.4%, 8,192 channels
// -0.8%, 16,384 +0.3%: profiles/r05_hov_ab_*.txt); 0: round 4's order (A/B knob)
#define QPSK_HUNT_OVERLAP 1
#endif

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

// ------------------------------------------------------- filtered hunt
// The hunt needs only max_index (src/qpsk.c:172-183; max_value reaches no
// output), so the exact sums are needed only when the argmax is in doubt.
// First pass: the same 16x16 product with T split into two bf16 parts,
// T = hi + lo + r (hi = RN_bf16(T), lo = RN_bf16(T - hi), |r| <= 2^-16 |T|),
// on v_mfma_f32_16x16x32_bf16 (B = p or 0 is exact in bf16): 10 MFMAs of 16
// cycles that hold the VALU for 8 each, against 36 f32 MFMAs that hold it for
// ~29 each (profiles/calib/mfma_mix_r02.txt).  Per lag and component the
// result S' is within
//     d = 2^-13 W + 2^-100,   W = sum_{j<255} |Tr_j| + |Ti_j|
// of the reference's sequential fp32 sum S: |S - sum T| <= 127u W (u = 2^-24)
// for the reference's rounding, 2^-16 W for the split, at most 2u per
// addition over the 160 terms of a chain in any order for the MFMA's fp32
// accumulation (2^-15.7 W), u |S'| for the final hi + lo add, and 2^-126 per
// term should the hardware flush bf16 denormals: 2^-14.6 W in all, 3x below d.
// Hence cnormf(S) (src/qpsk.c:75-80, three roundings) lies in
//     [L, U] = [(max(|Sr'|-d,0)^2 + max(|Si'|-d,0)^2)(1 - 2^-18),
//               ((|Sr'|+d)^2 + (|Si'|+d)^2)(1 + 2^-18)]
// (the factors also cover the roundings of computing L and U).  If exactly
// one lag l* has U >= Lmax = max L, and Lmax > 0, then cnormf(S[l*]) is the
// strict maximum and positive, so the reference's scan picks l*.  Otherwise
// (ties, near-ties, an all-zero window) the caller runs the exact chain.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
constexpr int kHSteps = 5;                     // K = 160 = 5 x 32
constexpr int kBH = kHSteps * 64 * 4;          // floats: B table, 16 B per lane and step (5 KB)
constexpr int kPL = 176;                       // floats: p_q at [q + 16], q in [-16, 160), for the exact chain
// bf16 images of T in the front's scratch (bytes): hi_r, hi_i, lo_r, lo_i, 272
// entries each (255.. zero).  An imaginary image sits 128 B (mod 256) after its
// real one: then the 16 lanes of every ds_read_b128 lane group ({0-3, 12-15,
// 20-27}, ... MI355X_MICROARCH.md LDS) read 16 distinct 16-B slots of the
// 256-B bank row (at 16 B mod 256, as first laid out, 5 of the 20 group-reads
// per image were 2-way: +40 LDS cycles per channel, SQ_LDS_BANK_CONFLICT in
// profiles/r02_v7_summary.md).
__host__ __device__ constexpr int himg(int c) { return c == 0 ? 0 : c == 1 ? 640 : c == 2 ? 1280 : 1920; }
constexpr int kHBytes = 2464;

// B tables (once per workgroup): BH[s][lane] = p_{32s + 8(l>>4) + jj - (l&15)} or
// 0, jj < 8, as bf16; PL for correlate_pl
__device__ __forceinline__ void bconst_h_lds(int tid, int nthreads, float* BH) {
    for (int x = tid; x < kHSteps * 64; x += nthreads) {
        const int s = x >> 6, l = x & 63;
        unsigned w[4];
#pragma unroll
        for (int jj = 0; jj < 8; jj += 2) {
            unsigned v = 0;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int i = 32 * s + 8 * (l >> 4) + jj + e - (l & 15);
                const unsigned b = (i >= 0 && i < QK_NPRE) ? (QK_PRE[i] > 0 ? 0x3F80u : 0xBF80u) : 0u;
                v |= b << (16 * e);
            }
            w[jj >> 1] = v;
        }
        reinterpret_cast<uint4*>(BH)[x] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    float* PL = BH + kBH;
    for (int x = tid; x < kPL; x += nthreads) {
        const int q = x - 16;
        PL[x] = (q >= 0 && q < QK_NPRE) ? (float)QK_PRE[q] : 0.0f;
    }
}

// max over the 64 lanes of a wave (DPP row shifts / row broadcasts, no LDS trips)
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false)); // row_shr:1
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false)); // row_shr:2
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xe, false)); // row_shr:4
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xc, false)); // row_shr:8
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false)); // row_bcast:15
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false)); // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// sum over the wave (DPP row shifts / broadcasts); order-free: only a bound
template <int CTRL, int RM, int BM>
__device__ __forceinline__ float dpp_f32(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, RM, BM, false));
}
__device__ __forceinline__ float wave_sum_f32(float v) {
    v = v + dpp_f32<0x111, 0xf, 0xf>(v);   // row_shr:1
    v = v + dpp_f32<0x112, 0xf, 0xf>(v);   // row_shr:2
    v = v + dpp_f32<0x114, 0xf, 0xe>(v);   // row_shr:4
    v = v + dpp_f32<0x118, 0xf, 0xc>(v);   // row_shr:8
    v = v + dpp_f32<0x142, 0xa, 0xf>(v);   // row_bcast:15
    v = v + dpp_f32<0x143, 0xc, 0xf>(v);   // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// bf16 images of T (as store_t: T[j] = (RN(dr - di), RN(di + dr)), j < 255);
// lane l writes j = 4l .. 4l+3 of each image.  Returns this lane's part of W
// (W = the wave sum of the parts, wave_sum_f32).
__device__ __forceinline__ float store_h(int lane, const float2* dec, char* H) {
    const float4* d4 = reinterpret_cast<const float4*>(dec + 4 * lane);
    const float4 p = d4[0], q = d4[1];
    const float dr[4] = {p.x, p.z, q.x, q.z}, di[4] = {p.y, p.w, q.y, q.w};
    float t[2][4];   // [comp][r]
    float w = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool in = 4 * lane + r < 2 * QK_NLAG - 1;
        t[0][r] = in ? dr[r] - di[r] : 0.0f;
        t[1][r] = in ? di[r] + dr[r] : 0.0f;
        w = w + (__builtin_fabsf(t[0][r]) + __builtin_fabsf(t[1][r]));
    }
#pragma unroll
    for (int c = 0; c < 2; c++) {
        bf2 h[2], l[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            h[e] = bf2{(__bf16)t[c][2 * e], (__bf16)t[c][2 * e + 1]};   // RN
            const float r0 = t[c][2 * e] - (float)h[e][0];               // exact
            const float r1 = t[c][2 * e + 1] - (float)h[e][1];
            l[e] = bf2{(__bf16)r0, (__bf16)r1};
        }
        uint2 hv, lv;
        __builtin_memcpy(&hv, h, 8);
        __builtin_memcpy(&lv, l, 8);
        *reinterpret_cast<uint2*>(H + himg(c) + 8 * lane) = hv;
        *reinterpret_cast<uint2*>(H + himg(2 + c) + 8 * lane) = lv;
    }
    if (lane < 2) {   // entries 256..271 (B = 0 there, but A must be finite)
#pragma unroll
        for (int c = 0; c < 4; c++)
            *reinterpret_cast<uint4*>(H + himg(c) + 512 + 16 * lane) = make_uint4(0u, 0u, 0u, 0u);
    }
    return w;
}

// The bf16 pass: this lane's D fragment (lags lag_lo / lag_hi, as correlate)
__device__ __forceinline__ f4 correlate_h(int lane, const char* H, const float* BH) {
    const int m = lane & 15, h = lane >> 4;
    const int a = m >> 1, comp = m & 1;
    const char* ahi = H + (comp ? himg(1) : himg(0)) + 32 * a + 16 * h;
    const char* alo = H + (comp ? himg(3) : himg(2)) + 32 * a + 16 * h;
    const bf8* bsrc = reinterpret_cast<const bf8*>(BH) + lane;
    f4 acc_h = {0.0f, 0.0f, 0.0f, 0.0f}, acc_l = acc_h;
#pragma unroll
    for (int s = 0; s < kHSteps; s++) {
        const bf8 b = bsrc[64 * s];
        const bf8 xh = *reinterpret_cast<const bf8*>(ahi + 64 * s);
        const bf8 xl = *reinterpret_cast<const bf8*>(alo + 64 * s);
        acc_h = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, b, acc_h, 0, 0, 0);
        acc_l = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl, b, acc_l, 0, 0, 0);
    }
    return acc_h + acc_l;
}

__device__ __forceinline__ void cn_bounds(float sr, float si, float d, float& U, float& L) {
    const float ar = __builtin_fabsf(sr), ai = __builtin_fabsf(si);
    const float ur = ar + d, ui = ai + d;
    const float lr = __builtin_fmaxf(ar - d, 0.0f), li = __builtin_fmaxf(ai - d, 0.0f);
    U = (ur * ur + ui * ui) * (1.0f + 0x1p-18f);
    L = (lr * lr + li * li) * (1.0f - 0x1p-18f);
}

// max_index from the bf16 pass when it is certain (see above), else -1.
// `W` is store_h's bound sum; wave_max is the caller's u32 wave max.
template <typename WaveMax>
__device__ __forceinline__ int pick_h(int lane, f4 s, float W, WaveMax wave_max) {
    const float d = W * 0x1p-13f + 0x1p-100f;
    float U0, L0, U1, L1;
    cn_bounds(s[0], s[1], d, U0, L0);
    cn_bounds(s[2], s[3], d, U1, L1);
    // L >= 0: its bits order as unsigned; NaN cannot occur (T is finite)
    const unsigned lm = wave_max(max(__float_as_uint(L0), __float_as_uint(L1)));
    if (lm == 0u) return -1;
    const float Lm = __uint_as_float(lm);
    const unsigned long long b0 = __ballot(U0 >= Lm), b1 = __ballot(U1 >= Lm);
    if (__popcll(b0) + __popcll(b1) != 1) return -1;
    return b0 ? lag_lo(__ffsll((long long)b0) - 1) : lag_hi(__ffsll((long long)b1) - 1);
}

// The exact chain (correlate) with B from the PL line: step s of lane l uses
// p_{4s + (l>>4) - (l&15)} = PL[16 + 4s + (l>>4) - (l&15)].
__device__ __forceinline__ f4 correlate_pl(int lane, const float* TK, const float* PL) {
    const int m = lane & 15, kk = lane >> 4;
    const int a = m >> 1, comp = m & 1;
    const f4* src = reinterpret_cast<const f4*>(TK + (kk * 2 + comp) * kRow + 4 * a);
    const float* bl = PL + 16 + kk - m;   // m == n == lane & 15
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < kSteps / 4; t++) {
        const f4 v = src[t];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, bl[16 * t + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, bl[16 * t + 4], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.z, bl[16 * t + 8], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.w, bl[16 * t + 12], acc, 0, 0, 0);
    }
    return acc;
}

// the writes of one wave's lanes visible to its other lanes' reads (LDS)
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The reference's scan (src/qpsk.c:172-183) over exact sums: the first lag
// whose cnormf (src/qpsk.c:75-80) is > the running max, which starts at 0.
// Values are >= 0 or NaN (never selected): as non-negative float bits they
// order as unsigned; take the wave max, then the lowest lag holding it; a
// maximum of 0 leaves max_index at 0.  Lane order is lag order within each of
// the two fragments (LO / HI map a lane to its lags).
template <typename WaveMax, typename LO, typename HI>
__device__ __forceinline__ int argmax_exact(f4 acc, WaveMax wave_max, LO lag_of_lo, HI lag_of_hi) {
    const float r0 = acc[0], i0 = acc[1], r1 = acc[2], i1 = acc[3];
    const float c0 = r0 * r0 + i0 * i0;
    const float c1 = r1 * r1 + i1 * i1;
    const unsigned k0 = c0 > 0.0f ? __float_as_uint(c0) : 0u;
    const unsigned k1 = c1 > 0.0f ? __float_as_uint(c1) : 0u;
    const unsigned km = wave_max(max(k0, k1));
    if (km == 0u) return 0;
    const unsigned long long m0 = __ballot(k0 == km), m1 = __ballot(k1 == km);
    const int i0x = m0 ? lag_of_lo(__ffsll((long long)m0) - 1) : 1 << 20;
    const int i1x = m1 ? lag_of_hi(__ffsll((long long)m1) - 1) : 1 << 20;
    return min(i0x, i1x);
}

// max_index of dec's 128 lags on the matrix cores: the bf16 pass, and the
// exact chain when it cannot decide (fb = true).  S: the wave's scratch (LDS,
// >= max(kHBytes, 4 kTK) bytes, 16-B aligned); TB: bconst_h_lds's tables.
template <typename WaveMax>
__device__ __forceinline__ int hunt_index(int lane, const float2* dec, float* S, const float* TB,
                                          WaveMax wave_max, bool& fb) {
    char* H = reinterpret_cast<char*>(S);
    const float w = store_h(lane, dec, H);
    fb = false;
#if QPSK_HUNT_OVERLAP
    // the MFMAs first, W's DPP reduction in their shadow (neither waits for
    // the other; the all-zero test only needs W before the pick)
    lds_sync();
    const f4 acc = correlate_h(lane, H, TB);
    const float W = wave_sum_f32(w);
    if (W == 0.0f) return 0;
    const int pick = pick_h(lane, acc, W, wave_max);
#else
    const float W = wave_sum_f32(w);
    // an all-zero window (W sums non-negative terms: 0 only if every T is):
    // every sum is 0, so no lag exceeds the initial max and max_index stays 0
    if (W == 0.0f) return 0;
    lds_sync();
    const int pick = pick_h(lane, correlate_h(lane, H, TB), W, wave_max);
#endif
    fb = pick < 0;
    if (!fb) return pick;
    lds_sync();   // the exact image overwrites H
    store_t(lane, dec, S);
    lds_sync();
    return argmax_exact(correlate_pl(lane, S, TB + kBH), wave_max, lag_lo, lag_hi);
}

}  // namespace qhunt
