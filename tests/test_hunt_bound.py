"""Host check of the filtered hunt's decision rule (singlecarrier_amd/csrc/
qpsk_hunt.h pick_h): for sums S' anywhere within the stated error budget of
the reference's fp32 sums S, whenever the rule commits to a lag it is the
reference's max_index (src/qpsk.c:172-183).  The budget used here is the
derivation's own total (2^-14.6 W), below the kernel's d = 2^-13 W; the
rule's arithmetic (bounds, the 1 +- 2^-18 factors, the unsigned-bits max) is
replayed in float32 as the kernel does it."""
import numpy as np

import oracle


def ref_sums_index(dec):
    p = oracle.preamble().astype(np.float32)
    dr, di = dec.real.astype(np.float32), dec.imag.astype(np.float32)
    tr, ti = (dr - di).astype(np.float32), (di + dr).astype(np.float32)
    n = dec.shape[0]
    re = np.zeros((n, 128), np.float32)
    im = np.zeros((n, 128), np.float32)
    for i in range(128):
        re = (re + p[i] * tr[:, i:i + 128]).astype(np.float32)
        im = (im + p[i] * ti[:, i:i + 128]).astype(np.float32)
    c = (re * re + im * im).astype(np.float32)
    best = np.zeros(n, np.float32)
    idx = np.zeros(n, np.int64)
    for lag in range(128):
        up = c[:, lag] > best
        best = np.where(up, c[:, lag], best)
        idx = np.where(up, lag, idx)
    w = (np.abs(tr) + np.abs(ti)).sum(axis=1, dtype=np.float64).astype(np.float32)
    return re, im, idx, w


def pick(sr, si, w):
    """pick_h in float32: -1 when undecided."""
    f32 = np.float32
    d = (w * f32(2.0 ** -13) + f32(2.0 ** -100)).astype(f32)[:, None]
    ar, ai = np.abs(sr), np.abs(si)
    ur, ui = (ar + d).astype(f32), (ai + d).astype(f32)
    lr = np.maximum((ar - d).astype(f32), f32(0))
    li = np.maximum((ai - d).astype(f32), f32(0))
    U = ((ur * ur).astype(f32) + (ui * ui).astype(f32)).astype(f32) * f32(1 + 2.0 ** -18)
    L = ((lr * lr).astype(f32) + (li * li).astype(f32)).astype(f32) * f32(1 - 2.0 ** -18)
    lm = L.max(axis=1)
    cand = U >= lm[:, None]
    ok = (lm > 0) & (cand.sum(axis=1) == 1)
    return np.where(ok, np.argmax(cand, axis=1), -1)


def _windows(rng, n):
    p = oracle.preamble().astype(np.float32)
    sym = (rng.choice([-1, 1], (n, 255)) + 1j * rng.choice([-1, 1], (n, 255))) * 0.7
    pre = rng.random(n) < 0.4
    off = rng.integers(0, 128, n)
    for k in np.flatnonzero(pre):
        sym[k, off[k]:off[k] + 128] = p * (1 + 1j) * 0.7
    amp = 2.0 ** rng.uniform(-12, 3, n)[:, None]
    noise = rng.uniform(0, 0.5, n)[:, None]
    dec = amp * (sym + noise * (rng.standard_normal((n, 255)) + 1j * rng.standard_normal((n, 255))))
    # near-ties: a second copy of the window's strongest structure
    tie = rng.random(n) < 0.2
    dec[tie, 127:] = dec[tie, :128] * (1 + rng.choice([-1, 1], tie.sum())[:, None] * 10.0 ** rng.uniform(-8, -3, tie.sum())[:, None])
    return dec.astype(np.complex64)


def test_decision_rule_never_contradicts_the_reference():
    rng = np.random.default_rng(11)
    n = 3000
    dec = _windows(rng, n)
    re, im, idx, w = ref_sums_index(dec)
    budget = (w * np.float32(2.0 ** -14.6))[:, None]
    decided = 0
    for trial in range(4):
        # worst-case-shaped errors: uniform in the budget, and at its edges
        if trial < 2:
            er = rng.uniform(-1, 1, re.shape) * budget
            ei = rng.uniform(-1, 1, im.shape) * budget
        else:
            er = rng.choice([-1.0, 1.0], re.shape) * budget
            ei = rng.choice([-1.0, 1.0], im.shape) * budget
        sr = (re + er).astype(np.float32)
        si = (im + ei).astype(np.float32)
        got = pick(sr, si, w)
        m = got >= 0
        decided += m.sum()
        assert (got[m] == idx[m]).all(), np.flatnonzero(m & (got != idx))[:5]
    assert decided > 0.8 * 4 * n     # the rule decides most windows
