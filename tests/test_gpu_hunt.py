"""The preamble hunt's correlator on the matrix cores (singlecarrier_amd/csrc/
qpsk_hunt.h) is bit-identical to the reference's sequential complex sum
(correlate(), src/qpsk.c:88-96): for every lag, the (re, im) sums of 128
+-1 x T terms in index order.  This pins the hardware property the kernel relies
on -- v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain -- on inputs built to
expose any other summation order, wider accumulator or flushed denormal."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kernels")


def _lib():
    path = os.path.join(HERE, "libhunt_check.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", HERE], check=True)
    lib = C.CDLL(path)
    lib.hunt_check.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.hunt_pick.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.hunt_h.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    return lib


def ref_sums(dec):
    """src/qpsk.c:88-96 in fp32: sum_i (p_i + p_i j) * dec[l + i], i ascending.
    dec: complex64 [n][255] -> complex sums [n][128] as float32 (re, im)."""
    dr, di = dec.real.astype(np.float32), dec.imag.astype(np.float32)
    p = oracle.preamble().astype(np.float32)
    n = dec.shape[0]
    re = np.zeros((n, 128), np.float32)
    im = np.zeros((n, 128), np.float32)
    for i in range(128):
        a, b = dr[:, i:i + 128], di[:, i:i + 128]
        # (p + pj)(a + bj) = (p*a - p*b, p*b + p*a), each product exact
        re = re + (p[i] * a - p[i] * b)
        im = im + (p[i] * b + p[i] * a)
    return re, im


def _cases(rng, n):
    kinds = []
    g = rng.standard_normal((n, 255 * 2)).astype(np.float32)
    kinds.append(g)                                                      # typical
    e = rng.uniform(-40, 4, (n, 510))
    kinds.append((rng.choice([-1, 1], (n, 510)) * 2.0 ** e
                  * rng.uniform(1, 2, (n, 510))).astype(np.float32))     # wide exponents
    c = rng.standard_normal((n, 510)).astype(np.float32)
    c[:, ::7] *= np.float32(2.0 ** 12)                                   # cancellation
    c[:, 3::11] *= np.float32(2.0 ** -12)
    kinds.append(c)
    d = (rng.standard_normal((n, 510)) * 1e-39).astype(np.float32)       # subnormals
    kinds.append(d)
    z = rng.standard_normal((n, 510)).astype(np.float32)
    z[rng.random((n, 510)) < 0.7] = 0.0                                  # sparse / zeros
    kinds.append(z)
    x = np.concatenate(kinds)
    return (x[:, 0::2] + 1j * x[:, 1::2]).astype(np.complex64)


def test_mfma_correlator_bit_exact():
    rng = np.random.default_rng(20261015)
    dec = _cases(rng, 2048)
    n = dec.shape[0]
    buf = np.zeros((n, 256, 2), np.float32)
    buf[:, :255, 0] = dec.real
    buf[:, :255, 1] = dec.imag
    out = np.zeros((n, 128, 2), np.float32)
    assert _lib().hunt_check(buf.ctypes.data, n, out.ctypes.data) == 0
    re, im = ref_sums(dec)
    bad_re = out[..., 0].view(np.uint32) != re.view(np.uint32)
    bad_im = out[..., 1].view(np.uint32) != im.view(np.uint32)
    # +-0 may differ in sign (only squares are used); everything else bitwise
    bad_re &= ~((out[..., 0] == 0) & (re == 0))
    bad_im &= ~((out[..., 1] == 0) & (im == 0))
    assert not bad_re.any() and not bad_im.any(), (
        f"{int(bad_re.sum())} re / {int(bad_im.sum())} im sums differ, "
        f"first case {np.argwhere(bad_re | bad_im)[0]}")


def ref_index(dec):
    """The reference's hunt (src/qpsk.c:172-183): the first lag whose cnormf
    (src/qpsk.c:75-80, fp32, no fusion) is > the running max from 0."""
    re, im = ref_sums(dec)
    c = (re * re + im * im).astype(np.float32)
    best = np.zeros(c.shape[0], np.float32)
    idx = np.zeros(c.shape[0], np.int64)
    for lag in range(128):
        up = c[:, lag] > best
        best = np.where(up, c[:, lag], best)
        idx = np.where(up, lag, idx)
    return idx


def _pick(dec):
    n = dec.shape[0]
    buf = np.zeros((n, 256, 2), np.float32)
    buf[:, :255, 0] = dec.real
    buf[:, :255, 1] = dec.imag
    idx = np.zeros(n, np.int32)
    fb = np.zeros(n, np.int32)
    assert _lib().hunt_pick(buf.ctypes.data, n, idx.ctypes.data, fb.ctypes.data) == 0
    return idx, fb


def _frames(rng, n, amp, preamble):
    """QPSK-like decimated windows: random symbols plus ISI-like jitter, with
    the preamble (p_i (1 + j)) at a random lag when `preamble`."""
    p = oracle.preamble().astype(np.float32)
    sym = (rng.choice([-1, 1], (n, 255)) + 1j * rng.choice([-1, 1], (n, 255))) * 0.7
    if preamble:
        off = rng.integers(0, 128, n)
        for k in range(n):
            sym[k, off[k]:off[k] + 128] = p * (1 + 1j) * 0.7
    sym = sym + 0.05 * (rng.standard_normal((n, 255)) + 1j * rng.standard_normal((n, 255)))
    return (amp * sym).astype(np.complex64)


def _near_ties(rng, n):
    """Two preamble copies, at lags 0 and 127, whose amplitudes differ by a
    relative eps from 0 to 1e-3: max_index flips between them around eps = 0,
    and the bf16 pass must hand every case it cannot separate to the exact
    chain."""
    p = oracle.preamble().astype(np.float32)
    eps = np.concatenate([[0.0], np.geomspace(1e-9, 1e-3, n // 2 - 1)])
    eps = np.concatenate([eps, -eps])[:n]
    dec = np.zeros((n, 255), np.complex64)
    a = rng.uniform(0.3, 2.0, n)
    for k in range(n):
        dec[k, :128] += (p * (1 + 1j) * a[k]).astype(np.complex64)
        dec[k, 127:255] += (p * (1 + 1j) * a[k] * (1 + eps[k])).astype(np.complex64)
    dec += (1e-3 * (rng.standard_normal((n, 255)) + 1j * rng.standard_normal((n, 255)))).astype(np.complex64)
    return dec.astype(np.complex64)


def test_filtered_hunt_index_matches_reference():
    """qhunt::hunt_index (the product's hunt: bf16 hi/lo pass with an error
    bound, exact chain when in doubt) picks the reference's max_index on
    typical frames at several amplitudes, exact ties (constant and all-zero
    windows), constructed near-ties and the wide-exponent / cancellation /
    subnormal / sparse cases; both paths are exercised."""
    rng = np.random.default_rng(20261016)
    parts = [_frames(rng, 512, a, pre) for a in (1.0, 1e-3, 4.0) for pre in (False, True)]
    parts.append(_near_ties(rng, 512))
    parts.append(_cases(rng, 256))
    const = np.full((4, 255), 0.37 - 0.11j, np.complex64)
    const[1] = 0.0
    const[2] = 1e-30 + 0j
    const[3, 200:] = 0.0                 # a truncated constant: no tie
    parts.append(const)
    dec = np.concatenate(parts)
    idx, fb = _pick(dec)
    ref = ref_index(dec)
    bad = np.flatnonzero(idx != ref)
    assert bad.size == 0, f"{bad.size} of {len(dec)} differ, first {bad[:5]}: {idx[bad[:5]]} vs {ref[bad[:5]]}"
    # both paths ran: the bf16 pass decided most typical frames, the exact
    # chain every tie (constant and zero windows) and the closest near-ties
    n_typ = 6 * 512
    assert fb[:n_typ].mean() < 0.05
    assert fb[-4] == 1 and fb[-2] == 1   # constant (all lags tie), underflowing window
    assert fb[-3] == 0                   # all-zero window: max_index 0 without the chain
    assert fb[n_typ:n_typ + 512].sum() > 0 and fb[n_typ:n_typ + 512].mean() < 1.0


def test_bf16_pass_within_its_error_budget():
    """The hardware side of the filtered hunt's proof: on the stress windows
    the bf16 hi/lo pass (v_mfma_f32_16x16x32_bf16) lands within 2^-14.6 W of
    the reference's sequential fp32 sums (plus 2^-110 for flushed denormals),
    the budget qpsk_hunt.h derives and then covers 3x over (d = 2^-13 W +
    2^-100); W as the kernel computes it bounds the exact sum of |Tr| + |Ti|."""
    rng = np.random.default_rng(20261017)
    dec = np.concatenate([_frames(rng, 512, 1.0, False), _frames(rng, 512, 3.0, True),
                          _near_ties(rng, 256), _cases(rng, 256)])
    n = dec.shape[0]
    buf = np.zeros((n, 256, 2), np.float32)
    buf[:, :255, 0] = dec.real
    buf[:, :255, 1] = dec.imag
    out = np.zeros((n, 128, 2), np.float32)
    w = np.zeros(n, np.float32)
    assert _lib().hunt_h(buf.ctypes.data, n, out.ctypes.data, w.ctypes.data) == 0
    re, im = ref_sums(dec)
    dr, di = dec.real.astype(np.float32), dec.imag.astype(np.float32)
    w_exact = (np.abs(dr - di).astype(np.float64) + np.abs(di + dr)).sum(axis=1)
    assert (w.astype(np.float64) >= w_exact * (1 - 2.0 ** -16)).all()
    err = np.maximum(np.abs(out[..., 0].astype(np.float64) - re), np.abs(out[..., 1].astype(np.float64) - im))
    # relative budget, plus the absolute allowance for denormal flushing
    # (the subnormal windows: <= 2^-126 per term; the kernel's d adds 2^-100)
    bound = 2.0 ** -14.6 * w_exact + 2.0 ** -110
    excess = err.max(axis=1) / bound
    assert excess.max() <= 1.0, (excess.max(), int(excess.argmax()))
