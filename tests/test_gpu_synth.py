"""GPU synthesis of the benchmark input (qpsk_synth_device, singlecarrier_amd/
csrc/qpsk_synth_dev.hip) against the host generator qpsk_synth_batch(), whose
transmitter reproduces the reference's qpsk_tx_frame (src/qpsk.c:278-322)
bit for bit (tests/test_abi.py, tests/golden/tx_golden.npz).  The device
formulation is parallel over (channel, TX block) instead of stateful, so this
is a parity test of that reformulation: noiseless output must be identical,
sample for sample."""
import ctypes as C

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("seed,nch,nf,c0", [(3, 300, 5, 0), (1, 64, 40, 0), (7, 130, 9, 4000),
                                            (11, 1, 2, 123456)])
def test_noiseless_identical_to_host(seed, nch, nf, c0):
    d = sc.synth_device(seed, nch, nf, c0=c0).cpu().numpy()
    h = sc.synth(seed, nch, nf, c0=c0)
    assert d.shape == h.shape
    bad = d != h
    assert not bad.any(), f"{int(bad.sum())} samples differ, first at {np.argwhere(bad)[0]}"


@pytest.mark.parametrize("ebn0", [0.0, 4.0, 9.0])
def test_awgn_matches_host(ebn0):
    """Same counter-based Box-Muller; the double log/cos come from the device
    libm, so equality is checked, not assumed: every sample identical."""
    d = sc.synth_device(5, 128, 6, ebn0).cpu().numpy()
    h = sc.synth(5, 128, 6, ebn0)
    ndiff = int((d != h).sum())
    assert ndiff == 0, f"{ndiff} of {d.size} noisy samples differ (max |diff| " \
                       f"{int(np.abs(d.astype(int) - h).max())})"


def test_odd_lengths_and_tail():
    """nsamples that end inside a packet, in a gap and before the first sample."""
    for ns in (1, 700, 2783 + 1900, 3 * 2783 - 5):
        out = torch.empty((40, ns), dtype=torch.int16, device="cuda")
        assert sc.lib().qpsk_synth_device(9, 0, 40, 1000.0, out.data_ptr(), ns, None) == 0
        torch.cuda.synchronize()
        h = np.empty((40, ns), np.int16)
        sc.lib().qpsk_synth_batch(9, 0, 40, 1000.0, h.ctypes.data, ns, 4)
        assert (out.cpu().numpy() == h).all(), ns


def test_rx_on_device_synthesised_input():
    """The receive path fed straight from the device generator (no host copy of
    the input), checked against the oracle on the same samples."""
    nch, nf = 200, 12
    x = sc.synth_device(42, nch, nf, 6.0)
    bits = torch.empty((nch, nf, 62), dtype=torch.uint8, device="cuda")
    valid = torch.empty((nch, nf), dtype=torch.uint8, device="cuda")
    rx = sc.Receiver(nch)
    rx.demod_device(x, bits, valid)
    torch.cuda.synchronize()
    eb, ev, _ = oracle.cpu_rx(x.cpu().numpy())
    assert (valid.cpu().numpy() == ev).all() and (bits.cpu().numpy() == eb).all()
    assert ev.any()
    rx.close()
