"""The dec752 receiver mode on the MI355X path (run with -m gpu).

QPSK_MODE_DEC752 is the "intended semantics" variant of SURVEY.md 8f rank 3:
decimated_frame with the 752 entries its decimation loop writes
(src/qpsk.c:157-162) instead of the reference build's overflow into
input_frame.  It is NOT reference parity; its expected values come from
oracle/_ref/libqpsk_ref752.so (the unmodified reference sources linked with the
array padded, oracle/ref/dec752.ld) through the golden fixtures, and from the
oracle restatement's dec752 mode, pinned to that build by tests/test_oracle.py.
Every comparison is exact, soft symbols included.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu

D752 = ["synth_d752_s1_clean", "synth_d752_s2_eb4"]


def _vs_oracle(x, **kw):
    rx = sc.Receiver(x.shape[0], mode=sc.MODE_DEC752)
    assert rx.mode == sc.MODE_DEC752
    out = rx.demod(x, trace=True, soft=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_array_equal(out["bits"], bits)
    t = out["trace"]
    np.testing.assert_array_equal(t[..., 0], tr["max_index"])
    np.testing.assert_array_equal(t[..., 1], tr["matches"])
    np.testing.assert_array_equal(t[..., 3], tr["rx_timing"])
    vm = valid.astype(bool)
    np.testing.assert_array_equal(out["soft"][vm], tr["soft"][vm])
    assert not out["soft"][~vm].any()
    rx.close()
    return out


def test_sample_file_md5(golden_dir):
    exp = json.load(open(os.path.join(golden_dir, "sample_expected_dec752.json")))
    frames = sc.read_raw(os.path.join(golden_dir, "preamble_qpsk_8k.raw"))
    rx = sc.Receiver(1, mode=sc.MODE_DEC752)
    out = rx.demod(frames[None], trace=True, soft=True)
    recs = sc.records(out["bits"][0], out["valid"][0])
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"] == "b4bbd42413bbc25518b7c1c0ebe64fc1"
    for n, t in enumerate(exp["trace"]):
        assert list(out["trace"][0, n]) == [t["max_index"], t["matches"], t["valid"], t["rx_timing"]]
    for n, s in exp["soft"].items():
        np.testing.assert_array_equal(out["soft"][0, int(n)], np.array(s, np.float32))


@pytest.mark.parametrize("name", D752)
def test_synth_goldens(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    x = oracle.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])
    rx = sc.Receiver(x.shape[0], mode=sc.MODE_DEC752)
    out = rx.demod(x, trace=True, soft=True)
    np.testing.assert_array_equal(np.packbits(out["bits"], axis=-1), g["bits"])
    np.testing.assert_array_equal(out["valid"], g["valid"])
    np.testing.assert_array_equal(out["trace"][..., 0], g["max_index"])
    np.testing.assert_array_equal(out["trace"][..., 1], g["matches"])
    np.testing.assert_array_equal(out["trace"][..., 3], g["rx_timing"])
    np.testing.assert_array_equal(out["soft"], g["soft"])


@pytest.mark.parametrize("nch,ebn0", [(1, 1000.0), (65, 5.0), (2048, 1000.0), (1024, 2.0)])
def test_vs_oracle(nch, ebn0):
    x = oracle.synth(700 + nch, nch, 14, ebn0)
    _vs_oracle(x)


def test_edge_inputs():
    rng = np.random.default_rng(6)
    x = np.stack([
        np.zeros((8, 1880), np.int16),
        np.full((8, 1880), 32767, np.int16),
        np.full((8, 1880), -32768, np.int16),
        np.tile(np.array([32767, -32768], np.int16), (8, 940)),
        rng.integers(-32768, 32768, (8, 1880)).astype(np.int16),
        rng.integers(-3, 4, (8, 1880)).astype(np.int16),
    ])
    _vs_oracle(x)


@pytest.mark.parametrize("shape", ["4x2", "2x4d", "1x8"])
def test_every_workgroup_shape(shape, monkeypatch):
    monkeypatch.setenv("QPSK_SHAPE", shape)
    x = oracle.synth(62, 300, 12, 5.0)
    _vs_oracle(x)


@pytest.mark.parametrize("shift", [6, 11])
def test_low_amplitude_streams(shift):
    """The filtered hunt's near and exact ties (see test_gpu_parity.py) under
    the dec752 semantics."""
    x = (oracle.synth(41 + shift, 192, 12, 8.0).astype(np.int32) >> shift).astype(np.int16)
    _vs_oracle(x)


def test_streaming_split_equals_one_call():
    """The carried sample history is longer in this mode (x_{n-1}[0..1703]):
    feeding 16 frames as 1+4+2+9 == one call."""
    x = oracle.synth(10, 130, 16, 6.0)
    whole = sc.Receiver(130, mode=sc.MODE_DEC752).demod(x, trace=True, soft=True)
    rx = sc.Receiver(130, mode=sc.MODE_DEC752)
    parts = [rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True)
             for a, b in ((0, 1), (1, 5), (5, 7), (7, 16))]
    for k in ("bits", "valid", "trace", "soft"):
        np.testing.assert_array_equal(np.concatenate([p[k] for p in parts], axis=1), whole[k])


def test_modes_are_independent_contexts():
    """A reference-mode and a dec752 context side by side on one device."""
    x = oracle.synth(12, 96, 10, 5.0)
    r0 = sc.Receiver(96)
    r1 = sc.Receiver(96, mode=sc.MODE_DEC752)
    o1 = r1.demod(x)
    o0 = r0.demod(x)
    np.testing.assert_array_equal(o0["bits"], oracle.cpu_rx(x)[0])
    np.testing.assert_array_equal(o1["bits"], oracle.cpu_rx(x, mode=oracle.MODE_DEC752)[0])
    assert (o0["valid"] != o1["valid"]).any()


def test_full_size_c3():
    """65536 channels x 32 frames in dec752 mode: bits, valid flags and the
    rx_timing trace equal the oracle's for every channel."""
    nch, nf = 65536, 32
    x = oracle.synth(3, nch, nf)
    rx = sc.Receiver(nch, mode=sc.MODE_DEC752)
    out = rx.demod(x, trace=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_array_equal(out["bits"], bits)
    np.testing.assert_array_equal(out["trace"][..., 3], tr["rx_timing"])
    np.testing.assert_array_equal(out["trace"][..., 0], tr["max_index"])


def test_c_driver_mode_flag(golden_dir, tmp_path):
    """examples/qpsk_rx_raw.c -b -m 1: the dec752 receiver from C gives the
    padded reference build's output file for the sample capture."""
    import subprocess
    exe = os.path.abspath(os.path.join(golden_dir, "..", "..", "examples", "qpsk_rx_raw"))
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True)
    raw = os.path.join(golden_dir, "preamble_qpsk_8k.raw")
    subprocess.run([exe, "-b", "-m", "1", raw, "-o", str(tmp_path / "d")], check=True)
    exp = json.load(open(os.path.join(golden_dir, "sample_expected_dec752.json")))
    assert hashlib.md5((tmp_path / "d0.bin").read_bytes()).hexdigest() == exp["output_md5"]
