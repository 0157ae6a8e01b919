"""CPU-side checks of the product library: it builds, loads, and exports every
function the public headers declare; host-only surface functions behave like
the reference.  No GPU compute here."""
import os
import re

import numpy as np
import pytest

import singlecarrier_amd as sc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\(", src):
            if m.group(1).startswith(("qpsk_", "cnormf")):
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(sc.LIB_PATH):
        sc.build()
    L = sc.lib()
    declared = _declared()
    assert {"qpsk_rx_frame", "qpsk_tx_frame", "qpsk_mod", "qpsk_demod", "cnormf",
            "qpsk_rx_create", "qpsk_rx_batch", "qpsk_rx_batch_device"} <= declared
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert set(sc.SYMBOLS) >= declared


def test_state_snapshot_size():
    """qpsk_rx_state_size (host only): a 64-byte header plus, per channel, the
    two-frame sample history (2 x 1880 int16), the next frame's equalizer
    window (168 float2), its preamble position and rx_timing."""
    L = sc.lib()
    assert L.qpsk_rx_state_size(0) == 0
    per = 2 * 1880 * 2 + 168 * 8 + 4 + 4
    assert L.qpsk_rx_state_size(1) == 64 + per
    assert L.qpsk_rx_state_size(65536) == 64 + 65536 * per


def test_code_object_targets_gfx950():
    data = open(sc.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_surface_host_functions():
    assert sc.cnormf(3 + 4j) == 25.0
    assert sc.qpsk_mod([0, 0], 0) == 1 + 1j
    assert sc.qpsk_mod([1, 0], 0) == 1 - 1j    # bits[index] = Q
    assert sc.qpsk_mod([0, 1], 0) == -1 + 1j   # bits[index+1] = I
    assert sc.qpsk_demod(-1 - 1j) == [1, 1]
    assert sc.qpsk_demod(1 - 1j) == [1, 0]


def _tx_golden_frames(golden_dir):
    g = np.load(os.path.join(golden_dir, "tx_golden.npz"))
    syms = np.split(g["symbols"], np.cumsum(g["lengths"])[:-1])
    return list(zip(syms, g["preamble"])), g["samples"]


def test_tx_frame_matches_reference(golden_dir):
    """Host qpsk_tx_frame (src/qpsk.c:278-322) == the reference TX golden."""
    frames, expect = _tx_golden_frames(golden_dir)
    sc.qpsk_tx_init()
    got = np.concatenate([sc.qpsk_tx_frame(s, bool(p)) for s, p in frames])
    np.testing.assert_array_equal(got, expect)


def test_oracle_tx_matches_reference(golden_dir):
    import oracle
    frames, expect = _tx_golden_frames(golden_dir)
    np.testing.assert_array_equal(np.concatenate(oracle.cpu_tx(frames)), expect)


def test_no_gpu_is_a_loud_error():
    """Without a GPU the receiver must raise, never fall back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(sc.QpskError):
        sc.Receiver(4)


def test_product_synth_matches_goldens(golden_dir):
    """The product's input generator reproduces the golden inputs (same spec as
    the oracle's restatement, pinned by sha256)."""
    import hashlib
    for name in ("synth_s1_clean", "synth_s4_eb0"):
        g = np.load(os.path.join(golden_dir, name + ".npz"))
        x = sc.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
        assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])


def test_c_driver_links_against_the_library():
    """examples/qpsk_rx_raw.c: the reference RX loop relinked to libqpsk_hip.so."""
    import subprocess
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(os.path.join(ROOT, "examples", "qpsk_rx_raw"))


def test_record_writer_reproduces_reference_output_file(golden_dir):
    """qpsk_records (include/qpsk_stream.h, host code): the reference driver's
    496-byte records (src/qpsk.c:455-457) from the golden per-frame outputs of
    preamble_qpsk_8k.raw give the reference output file (md5 b56a4d36...)."""
    import hashlib
    import json
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    nf = exp["frames"]
    bits = np.zeros((nf, 62), np.uint8)
    valid = np.zeros(nf, np.uint8)
    for n, b in exp["valid_bits"].items():
        valid[int(n)] = 1
        bits[int(n)] = [int(ch) for ch in b]
    recs = sc.records(bits, valid)
    assert len(recs) == exp["output_bytes"] == 496 * int(valid.sum())
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"]
    assert sc.records(bits, np.zeros(nf, np.uint8)) == b""


def test_create_mode_rejects_unknown_modes():
    """qpsk_rx_create_mode validates its arguments before touching a device."""
    import ctypes as C
    L = sc.lib()
    for mode, nch in ((4, 4), (-1, 4), (sc.MODE_DEC752, 0)):
        err = C.c_int(0)
        assert not L.qpsk_rx_create_mode(0, nch, mode, C.byref(err))
        assert err.value == -1   # QPSK_EINVAL
    assert L.qpsk_rx_mode(None) == -1


def test_fft_host_twiddles_match_the_reference_formula():
    """The product's twiddle table (qpsk_fft_host.c) has the bits of the
    reference's fft_alloc (src/fft.c:67-74), via the oracle restatement (itself
    pinned to the compiled reference in tests/test_oracle.py)."""
    import oracle
    for n in (4, 8, 64, 256, 512, 4096):
        for inv in (False, True):
            np.testing.assert_array_equal(sc.fft_twiddle_table(n, inv).view(np.uint32),
                                          oracle.fft_twiddles(n, inv).view(np.uint32))


def test_fft_alloc_rejects_unsupported_sizes():
    import ctypes as C
    for n in (0, 2, 3, 12, 100, 8192):
        err = C.c_int(0)
        assert not sc.lib().qpsk_fft_alloc(0, n, 0, C.byref(err))
        assert err.value == -1


def test_state_load_rejects_short_or_foreign_buffers():
    """Receiver.state_load checks a snapshot's length and magic before reading
    its header (a short or foreign buffer is QPSK_EINVAL, not a numpy error);
    no context is touched, so no GPU is needed."""
    rx = sc.Receiver.__new__(sc.Receiver)
    rx._h = None
    for snap in (b"", b"QPSKSTA1", b"XPSKSTA1" + bytes(120)):
        with pytest.raises(sc.QpskError) as ei:
            rx.state_load(snap)
        assert ei.value.code == sc.QPSK_EINVAL
