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


# ------------------------------------------------- the FFT-correlation hunt variant
# QPSK_MODE_FFT_HUNT (flag): the receiver's hunt correlates through kiss_fft.
# Expected values: the oracle restatement's same mode (its hunt pinned to the
# reference's own fft() in tests/test_oracle.py).  Exact, soft symbols included.
MODES = [sc.MODE_FFT_HUNT, sc.MODE_DEC752 | sc.MODE_FFT_HUNT]


def _vs_oracle(x, mode):
    rx = sc.Receiver(x.shape[0], mode=mode)
    assert rx.mode == mode
    out = rx.demod(x, trace=True, soft=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=mode)
    np.testing.assert_array_equal(out["trace"][..., 0], tr["max_index"])
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_array_equal(out["bits"], bits)
    np.testing.assert_array_equal(out["trace"][..., 3], tr["rx_timing"])
    vm = valid.astype(bool)
    np.testing.assert_array_equal(out["soft"][vm], tr["soft"][vm])
    rx.close()
    return out


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("nch,ebn0", [(1, 1000.0), (130, 4.0), (2048, 1000.0), (1024, 1.0)])
def test_fft_hunt_receiver(mode, nch, ebn0):
    _vs_oracle(oracle.synth(900 + nch, nch, 12, ebn0), mode)


@pytest.mark.parametrize("mode", MODES)
def test_fft_hunt_edge_inputs(mode):
    rng = np.random.default_rng(8)
    x = np.stack([
        np.zeros((8, 1880), np.int16),
        np.full((8, 1880), -32768, np.int16),
        np.tile(np.array([32767, -32768], np.int16), (8, 940)),
        rng.integers(-32768, 32768, (8, 1880)).astype(np.int16),
    ])
    _vs_oracle(x, mode)


@pytest.mark.parametrize("shape", ["4x2", "2x4d", "1x8"])
def test_fft_hunt_every_shape(shape, monkeypatch):
    monkeypatch.setenv("QPSK_SHAPE", shape)
    _vs_oracle(oracle.synth(66, 300, 10, 3.0), sc.MODE_FFT_HUNT)


def test_fft_hunt_sample_file(golden_dir):
    """preamble_qpsk_8k.raw through the FFT-hunt variant: same hunt decisions
    as the direct correlator there, so the reference's output file results."""
    import hashlib
    import json
    import os
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    frames = sc.read_raw(os.path.join(golden_dir, "preamble_qpsk_8k.raw"))
    out = _vs_oracle(frames[None], sc.MODE_FFT_HUNT)
    assert hashlib.md5(sc.records(out["bits"][0], out["valid"][0])).hexdigest() == exp["output_md5"]


def test_fft_hunt_full_size():
    nch, nf = 65536, 32
    x = oracle.synth(3, nch, nf)
    rx = sc.Receiver(nch, mode=sc.MODE_FFT_HUNT)
    out = rx.demod(x, trace=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=sc.MODE_FFT_HUNT)
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_array_equal(out["bits"], bits)
    np.testing.assert_array_equal(out["trace"][..., 0], tr["max_index"])
