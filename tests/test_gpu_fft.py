"""The reference's kiss_fft on the GPU (include/qpsk_fft.h), run with -m gpu.

Expected values come from the oracle restatement oracle.cpu_fft (qc_fft),
which tests/test_oracle.py pins bit for bit to the reference's own compiled
src/fft.c.  Every comparison is on the bits (signed zeros included).
"""
import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu

SIZES = [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096]


def _cases(n, batch, seed):
    rng = np.random.default_rng(seed)
    x = np.empty((batch, n), np.complex64)
    x[:] = rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))
    x[0] = rng.integers(-3, 4, n) + 1j * rng.integers(-3, 4, n)
    x[1].view(np.float32)[:] = rng.choice([-0.0, 0.0, 1.0, -1.0], 2 * n)
    x[2] = rng.standard_normal(n) * 1e4
    x[3] = 0
    return x


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("inverse", [False, True])
def test_fft_bit_exact(n, inverse):
    x = _cases(n, 9, n + inverse)
    plan = sc.FftPlan(n, inverse)
    got = plan(x)
    np.testing.assert_array_equal(got.view(np.uint32), oracle.cpu_fft(x, inverse).view(np.uint32))
    plan.close()


def test_fft_large_batch_in_place_on_device():
    import torch
    n, batch = 256, 4096
    x = _cases(n, batch, 7)
    plan = sc.FftPlan(n)
    d = torch.from_numpy(x.view(np.float32)).cuda()
    plan.run_device(d, d)          # in place
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.complex64)
    ref = oracle.cpu_fft(x)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
