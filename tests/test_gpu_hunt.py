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
