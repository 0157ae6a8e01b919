// qpsk_fft_dev.h -- the reference's kiss_fft (src/fft.c) on one wavefront.
//
// A power-of-two transform of N points (4 <= N <= 4096) held in LDS, computed
// by the 64 lanes of one wave with the reference's factorization and
// butterflies, so the result is bit-identical to fft() (src/fft.c:133):
//   kf_factor (src/fft.c:433-459): radix-4 stages, then one radix-2 stage when
//     log2 N is odd (it is the innermost factor);
//   kf_work (src/fft.c:388-431): the recursion's leaf copies are an input
//     permutation (built on the host, qfft::build_perm), and its recombination
//     order is innermost stage first, every butterfly of a stage independent;
//   kf_bfly4 / kf_bfly2 (src/fft.c:190-255): the exact operation sequence,
//     with gcc -O2's reading of the C99 complex expressions: a complex
//     product is (ac - bd, ad + bc) and `x + y * I` is (x + y * 0.0f, y)
//     (the y * 0.0f decides the sign of a zero real part).
// No contraction (-ffp-contract=off and the pragma), so every product and sum
// is rounded once, as on the host.  Twiddles come from the host
// (qfft::twiddles, fft_alloc's formula, src/fft.c:67-74).
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

namespace qfft {

struct cf {
    float r, i;
};

__device__ __forceinline__ cf mul(cf a, cf b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ cf add(cf a, cf b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cf sub(cf a, cf b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cf mk(float x, float y) { return {x + y * 0.0f, y}; }   // x + y * I

__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// kf_bfly4 (src/fft.c:213-255) for one k: F = Fout of the butterfly group
__device__ __forceinline__ void bfly4(cf* F, int m, int k, int fs, const cf* tw, bool inverse) {
    cf* f = F + k;
    const cf s0 = mul(f[m], tw[k * fs]);
    const cf s1 = mul(f[2 * m], tw[2 * k * fs]);
    const cf s2 = mul(f[3 * m], tw[3 * k * fs]);
    const cf a = f[0];
    const cf s5 = sub(a, s1);
    const cf a1 = add(a, s1);
    const cf s3 = add(s0, s2);
    const cf s4 = sub(s0, s2);
    f[2 * m] = sub(a1, s3);
    f[0] = add(a1, s3);
    if (inverse) {
        f[m] = mk(s5.r - s4.i, s5.i + s4.r);
        f[3 * m] = mk(s5.r + s4.i, s5.i - s4.r);
    } else {
        f[m] = mk(s5.r + s4.i, s5.i - s4.r);
        f[3 * m] = mk(s5.r - s4.i, s5.i + s4.r);
    }
}

// kf_bfly2 (src/fft.c:190-211) for one k
__device__ __forceinline__ void bfly2(cf* F, int m, int k, int fs, const cf* tw) {
    const cf t = mul(F[m + k], tw[k * fs]);
    const cf a = F[k];
    F[m + k] = sub(a, t);
    F[k] = add(a, t);
}

// The stages of an N-point transform on buf (already in kf_work's leaf
// order), innermost first; caller synchronises the wave before and after.
// Stage s (0 = outermost): radix p_s, m_s = N / (p_0 .. p_s), fstride =
// p_0 .. p_{s-1}.  Butterfly b of a stage: group b / m, index k = b % m.
__device__ __forceinline__ void stages(int lane, int N, cf* buf, const cf* tw, bool inverse) {
    const int lg = 31 - __builtin_clz(N);
    const int n4 = lg / 2;                 // radix-4 stages (outermost)
    const bool r2 = (lg & 1) != 0;         // one radix-2 stage, innermost
    if (r2) {                              // p = 2, m = 1, fstride = N / 2
        for (int b = lane; b < N / 2; b += 64) bfly2(buf + 2 * b, 1, 0, N / 2, tw);
        lds_sync();
    }
    for (int s = n4 - 1; s >= 0; s--) {
        const int fs = 1 << (2 * s);       // 4^s
        const int m = N / (fs * 4);
        for (int b = lane; b < N / 4; b += 64) {
            const int g = b / m, k = b - g * m;
            bfly4(buf + g * 4 * m, m, k, fs, tw, inverse);
        }
        lds_sync();
    }
}

}  // namespace qfft
