"""The 4x2 kernel's split-FIR lane map (singlecarrier_amd/csrc/qpsk_split.h),
checked on the host for every rx_timing the receiver can hold (3..255,
/root/reference/src/qpsk.c:53, 219): it computes each of F[0..66] exactly once
(pass 1's lane 63 the triple F[j1], F[j1+5], F[j1+10], pass 2 the other 64),
pass 1 is free of LDS bank conflicts, and pass 2 keeps one 2-way lane group
at most (DESIGN.md "Round 6", item 1).  Bank model: ds_read_b64 serves lanes
0-31 and 32-63 apart, float2 f in bank pair f mod 32 (MI355X_MICROARCH.md LDS).
The table is what the kernel's __constant__ kSplitTab is built from; the GPU
parity tests (test_split_fir_window_boundary: all 32 residues) show the
outputs exact."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KM1 = 1240


@pytest.fixture(scope="module")
def dump(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("split") / "split_tab_dump")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                        "-I", os.path.join(ROOT, "singlecarrier_amd", "csrc"),
                        os.path.join(ROOT, "tests", "kernels", "split_tab_dump.hip"), "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("hipcc unavailable: " + r.stderr[-500:])
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    tab = np.array([[int(v) for v in out[r].split()] for r in range(32)])
    rts = {int(a): (int(b), int(c)) for a, b, c in (line.split() for line in out[32:32 + 256])}
    return tab, rts


def _groups(addr):
    """max number of distinct addresses in one bank pair, per 32-lane group"""
    worst = []
    for g in (addr[:32], addr[32:]):
        pairs = {}
        for a in g:
            if a is not None:
                pairs.setdefault(a % 32, set()).add(a)
        worst.append(max(len(v) for v in pairs.values()))
    return worst


def test_every_rx_timing(dump):
    tab, rts = dump
    for rt in range(3, 256):
        r, j1 = rts[rt]
        assert r == (15 * 63 + rt - KM1) % 32 and j1 in (r, r + 32) and j1 + 10 <= 66
        j = tab[r]
        triple = {j1, j1 + 5, j1 + 10}
        assert len(set(j)) == 64 and not (set(j) & triple)
        assert set(j) | triple == set(range(67))               # F[0..66], each once
        pass1 = [15 * l + rt for l in range(63)] + [KM1 + j1]
        assert _groups(pass1) == [1, 1], rt                    # conflict-free
        w = _groups([KM1 + int(x) for x in j])
        assert w[1] == 1 and w[0] <= 2, (rt, w)                # one 2-way group at most


def test_lanes_32_to_63_are_35_to_66_with_the_triple_folded_down(dump):
    tab, _ = dump
    for r in range(32):
        j1 = r + 32 if r <= 24 else r
        hi = [v - 32 if v in (j1, j1 + 5, j1 + 10) else v for v in range(35, 67)]
        assert list(tab[r, 32:]) == hi
        assert list(tab[r, :32]) == sorted(tab[r, :32])        # the rest, ascending
