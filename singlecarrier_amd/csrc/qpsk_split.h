// qpsk_split.h -- the lane map of the 4x2 kernel's split FIR (qpsk_rx.hip
// fir_split; DESIGN.md "Round 6", item 1).  Plain constexpr C++ shared by the
// kernel (its __constant__ table) and the host-side property test
// (tests/kernels/split_tab_dump.hip, tests/test_split_tab.py).
//
// M is the front's LDS sample buffer (float2); F_{n+1}[j] reads M[kSplitM1 + j
// + s], s < 49.  ds_read_b64 serves lanes 0-31 and 32-63 apart, float2 f in
// bank pair f mod 32.  Pass 1's lanes 0..62 read M[15 l + rt + s]; lane 63
// takes F[j1], F[j1+5], F[j1+10] with its base in the pair lanes 32..62 leave
// free; pass 2 computes the other 64 of F[0..66], lane l the entry j[r][l].
#pragma once

#include <stdint.h>

constexpr int kSplitM1 = 1240;   // qpsk_rx.hip kM1: where F_{n+1}'s samples start in M

// the residue (mod 32) of lane 63's pass-1 base, as a j offset from kSplitM1
__host__ __device__ constexpr int split_r(int rt) { return (15 * 63 + rt - kSplitM1) & 31; }
// lane 63's first output F[j1]: j1 = r or r + 32, j1 + 10 <= 66
__host__ __device__ constexpr int split_j1(int r) { return r <= 24 ? r + 32 : r; }

struct SplitTab {
    uint8_t j[32][64];   // [r][lane]: pass 2's output F[j]
};
// lanes 32..63: j = 35..66 with each of pass 1's j in that range replaced by
// j - 32 (the same bank pair, so one j per pair); lanes 0..31: the rest of
// [0, 66] in ascending order
constexpr SplitTab make_split_tab() {
    SplitTab t{};
    for (int r = 0; r < 32; r++) {
        const int j1 = split_j1(r);
        bool used[67] = {};
        used[j1] = used[j1 + 5] = used[j1 + 10] = true;
        for (int i = 0; i < 32; i++) {
            const int v = 35 + i;
            const int j = (v == j1 || v == j1 + 5 || v == j1 + 10) ? v - 32 : v;
            t.j[r][32 + i] = (uint8_t)j;
            used[j] = true;
        }
        int l = 0;
        for (int v = 0; v < 67; v++)
            if (!used[v]) t.j[r][l++] = (uint8_t)v;
    }
    return t;
}
