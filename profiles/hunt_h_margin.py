"""Observed error of the bf16 hunt pass against the reference's fp32 sums,
relative to W (the budget qpsk_hunt.h derives is 2^-14.6 W; the kernel's
decision uses d = 2^-13 W).  Stress windows of tests/test_gpu_hunt.py.

    python profiles/hunt_h_margin.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_hunt as t  # noqa: E402

rng = np.random.default_rng(20261017)
kinds = {"typical": t._frames(rng, 1024, 1.0, False), "preamble": t._frames(rng, 1024, 3.0, True),
         "near-ties": t._near_ties(rng, 512), "low amplitude": t._frames(rng, 1024, 1e-3, True)}
c = t._cases(rng, 256)
for i, nm in enumerate(["gaussian", "wide exponents", "cancellation", "subnormal", "sparse"]):
    kinds[nm] = c[256 * i:256 * (i + 1)]
for nm, dec in kinds.items():
    n = dec.shape[0]
    buf = np.zeros((n, 256, 2), np.float32)
    buf[:, :255, 0] = dec.real
    buf[:, :255, 1] = dec.imag
    out = np.zeros((n, 128, 2), np.float32)
    w = np.zeros(n, np.float32)
    assert t._lib().hunt_h(buf.ctypes.data, n, out.ctypes.data, w.ctypes.data) == 0
    re, im = t.ref_sums(dec)
    err = np.maximum(np.abs(out[..., 0].astype(np.float64) - re), np.abs(out[..., 1].astype(np.float64) - im))
    r = err.max(axis=1) / np.maximum(w.astype(np.float64), 1e-300)
    print(f"{nm:15s} max |S'-S|/W = 2^{np.log2(max(r.max(), 1e-300)):.1f}   median 2^{np.log2(max(np.median(r), 1e-300)):.1f}")
