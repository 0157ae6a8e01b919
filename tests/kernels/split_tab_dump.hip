// Test-only host program: prints the split FIR's lane map (qpsk_split.h) as
// the kernel's __constant__ table holds it -- 32 lines of 64 pass-2 entries --
// then rt, split_r(rt), split_j1 for rt in [0, 256).  Read by
// tests/test_split_tab.py; no device code, no GPU.
#include <cstdio>

#include "qpsk_split.h"

int main() {
    constexpr SplitTab t = make_split_tab();
    for (int r = 0; r < 32; r++) {
        for (int l = 0; l < 64; l++) std::printf("%d%c", t.j[r][l], l == 63 ? '\n' : ' ');
    }
    for (int rt = 0; rt < 256; rt++) std::printf("%d %d %d\n", rt, split_r(rt), split_j1(split_r(rt)));
    return 0;
}
