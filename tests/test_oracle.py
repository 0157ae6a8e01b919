"""Pin the oracle (clean-room restatement oracle/cpu_ref.c) to the reference.

Goldens in tests/golden/ were produced by the UNMODIFIED reference
(tests/golden/make_golden.py).  Where oracle/_ref is present the restatement is
also diffed live against the reference on fresh random channels.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle

SYNTH = ["synth_s1_clean", "synth_s2_eb8", "synth_s3_eb4", "synth_s4_eb0"]


def _sample(golden_dir):
    raw = np.fromfile(os.path.join(golden_dir, "preamble_qpsk_8k.raw"), np.int16)
    nf = raw.size // oracle.FRAME
    return raw[: nf * oracle.FRAME].reshape(1, nf, oracle.FRAME)


def test_sample_file_md5(golden_dir):
    """C1: the reference's capture through the restatement = reference output
    (src/qpsk.c:436-458 record format, md5 b56a4d36...)."""
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    raw = open(os.path.join(golden_dir, "preamble_qpsk_8k.raw"), "rb").read()
    assert hashlib.md5(raw).hexdigest() == exp["input_md5"] == "1175fea4332f8e742524d49641e32c62"
    x = _sample(golden_dir)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    recs = b"".join(np.concatenate([bits[0, n], np.zeros(434, np.uint8)]).tobytes()
                    for n in range(x.shape[1]) if valid[0, n])
    assert len(recs) == exp["output_bytes"] == 1984
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"] == "b56a4d3609d0312934aaef69903c5298"
    for n, t in enumerate(exp["trace"]):
        for k in ("max_index", "matches", "valid", "rx_timing"):
            assert int(tr[0, n][k]) == t[k], (n, k)
    st = np.load(os.path.join(golden_dir, "sample_stages.npz"))
    vm = st["valid"].astype(bool)
    np.testing.assert_array_equal(tr[0]["soft"][vm], st["soft"][vm])


@pytest.mark.parametrize("ebn0", [1000.0, 8.0, 3.0, 0.0])
def test_window_observable_range(ebn0):
    """The equalizer and the data symbols read only dec[mi .. mi + 162]
    (src/qpsk.c:188, 204-215: 128 training steps and 31 data steps, 5 taps):
    with every other entry of the frame's dec set to NaN after the hunt
    (qc_poison_unobservable) the restatement's outputs, soft symbols included,
    do not change.  This is what lets the GPU's split FIR compute dec[255..289]
    only when mi >= 93 ("the split FIR")."""
    import ctypes
    flag = ctypes.c_int.in_dll(oracle.cpu_lib(), "qc_poison_unobservable")
    rng = np.random.default_rng(9)
    x = oracle.synth(91, 96, 10, ebn0)
    x[0] = 0                                          # silence
    x[1, 3:5] = 32767                                 # saturated frames
    x[2] = rng.integers(-32768, 32768, x[2].shape)    # full-scale noise
    b1, v1, t1 = oracle.cpu_rx(x, trace=True)
    flag.value = 1
    try:
        b2, v2, t2 = oracle.cpu_rx(x, trace=True)
    finally:
        flag.value = 0
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(t1.view(np.uint8), t2.view(np.uint8))   # incl. soft, bitwise
    mi = t1["max_index"][v1.astype(bool)]
    assert v1.sum() > 0 and (ebn0 < 5 or (mi >= 93).any())


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build not present")
def test_window_observable_range_in_the_reference(golden_dir):
    """The split FIR's premise, pinned on the unmodified reference itself
    (oracle/_ref, the -Wl,--wrap=train_eq tap): with decimated_frame[0..289]
    set to NaN outside [mi, mi + 162] before each frame's equalizer
    (/root/reference/src/qpsk.c:186-215, after the hunt), the reference's
    outputs -- valid flags, bits, max_index, matches, rx_timing, and the soft
    symbols of valid frames, bitwise -- do not change on the sample file and
    seeded noiseless / AWGN sets; with one entry fewer at either end
    ([mi + 1, mi + 162] or [mi, mi + 161]) they do.  (Invalid frames' data_eq
    runs at rx_timing, src/qpsk.c:225-229, and its soft symbols are no output:
    they are compared on valid frames only.)"""
    rng = np.random.default_rng(19)
    sets = [_sample(golden_dir)]
    for seed, eb in ((92, 1000.0), (93, 8.0), (94, 3.0), (95, 0.0)):
        sets.append(oracle.synth(seed, 24, 10, eb))
    sets[-1][0] = 0                                          # silence
    sets[-1][1, 3:5] = 32767                                 # saturated frames
    sets[-1][2] = rng.integers(-32768, 32768, sets[-1][2].shape)   # full-scale noise

    def outputs(r):
        bits, valid, tr = r
        vm = valid.astype(bool)
        return (valid, bits, tr["max_index"], tr["matches"], tr["rx_timing"],
                tr["soft"][vm].view(np.uint32))

    nvalid = nhigh = 0
    narrower = {(1, 162): 0, (0, 161): 0}
    for x in sets:
        base = outputs(oracle.ref_rx(x, trace=True))
        for a, b in zip(base, outputs(oracle.ref_rx_poisoned(x, 0, 162))):
            np.testing.assert_array_equal(a, b)
        for lohi in narrower:
            got = outputs(oracle.ref_rx_poisoned(x, *lohi))
            narrower[lohi] += sum(not np.array_equal(a, b) for a, b in zip(base, got))
        vm = base[0].astype(bool)
        nvalid += int(vm.sum())
        nhigh += int((base[2][vm] >= 93).sum())
    assert nvalid > 50 and nhigh > 5           # windows reaching past dec[254] ran
    assert all(v > 0 for v in narrower.values()), narrower


def test_mixer_table_kat(golden_dir):
    """P[t] = R^(t+1) (src/qpsk.c:139) and the (-1)^n frame alternation."""
    kat = np.load(os.path.join(golden_dir, "kat.npz"))
    p = oracle.mixer_table()
    np.testing.assert_array_equal(p, kat["mixer_frame0"])
    np.testing.assert_array_equal(-p, kat["mixer_frame1"])
    assert p[0].view(np.uint32).tolist() == [0x3F26423A, 0xBF42A9F7]
    assert (p == 0).sum() == 93


def test_keystream_kat(golden_dir):
    """Descrambler keystream: frame n uses bits [62n, 62n+62) (src/scramble.c)."""
    kat = np.load(os.path.join(golden_dir, "kat.npz"))
    ks = oracle.keystream(kat["keystream"].size)
    np.testing.assert_array_equal(ks, kat["keystream"])
    assert "".join(map(str, ks[:62])) == \
        "00000011111101100000100000110100001100001011100010100011100100"
    full = oracle.keystream(2 * 32767)
    np.testing.assert_array_equal(full[:32767], full[32767:])  # maximal-length LFSR


@pytest.mark.parametrize("name", SYNTH)
def test_synth_goldens(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    x = oracle.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    np.testing.assert_array_equal(np.packbits(bits, axis=-1), g["bits"])
    np.testing.assert_array_equal(valid, g["valid"])
    for k in ("max_index", "matches", "rx_timing"):
        np.testing.assert_array_equal(tr[k], g[k])
    vm = valid.astype(bool)
    np.testing.assert_array_equal(tr["soft"][vm], g["soft"][vm])


def test_edge_inputs_vs_reference():
    """Saturated, alternating and all-zero frames: restatement == reference."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(5)
    x = np.stack([
        np.zeros((6, oracle.FRAME), np.int16),
        np.full((6, oracle.FRAME), 32767, np.int16),
        np.full((6, oracle.FRAME), -32768, np.int16),
        np.tile(np.array([32767, -32768], np.int16), (6, oracle.FRAME // 2)),
        rng.integers(-32768, 32768, (6, oracle.FRAME)).astype(np.int16),
        rng.integers(-3, 4, (6, oracle.FRAME)).astype(np.int16),
    ])
    b1, v1, t1 = oracle.cpu_rx(x, trace=True)
    b2, v2, t2 = oracle.ref_rx(x, trace=True)
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(b1, b2)
    for k in ("max_index", "matches", "rx_timing"):
        np.testing.assert_array_equal(t1[k], t2[k])


@pytest.mark.parametrize("ebn0", [1000.0, 6.0, 2.0])
def test_random_channels_vs_reference(ebn0):
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    x = oracle.synth(1234 + int(ebn0), 48, 20, ebn0, c0=1000)
    b1, v1, t1 = oracle.cpu_rx(x, trace=True)
    b2, v2, t2 = oracle.ref_rx(x, trace=True)
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(b1, b2)
    for k in ("max_index", "matches", "rx_timing"):
        np.testing.assert_array_equal(t1[k], t2[k])
    vm = v2.astype(bool)
    np.testing.assert_array_equal(t1["soft"][vm], t2["soft"][vm])


# ---------------------------------------------------------------- dec752 mode
# "Intended semantics" (SURVEY.md 8f rank 3): decimated_frame with the 752
# entries its loop writes (src/qpsk.c:157-162).  NOT reference parity.  Pinned
# by oracle/_ref/libqpsk_ref752.so -- the unmodified reference sources linked
# so that the array owns indices 562..751 (oracle/ref/dec752.ld) -- whose
# sample-file output md5 b4bbd424... is also the one SURVEY.md 8f records.
D752 = ["synth_d752_s1_clean", "synth_d752_s2_eb4"]


def test_dec752_sample_file_md5(golden_dir):
    exp = json.load(open(os.path.join(golden_dir, "sample_expected_dec752.json")))
    x = _sample(golden_dir)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    recs = b"".join(np.concatenate([bits[0, n], np.zeros(434, np.uint8)]).tobytes()
                    for n in range(x.shape[1]) if valid[0, n])
    assert len(recs) == exp["output_bytes"] == 1488
    md5 = hashlib.md5(recs).hexdigest()
    assert md5 == exp["output_md5"] == "b4bbd42413bbc25518b7c1c0ebe64fc1"
    assert md5.startswith("b4bbd424")
    for n, t in enumerate(exp["trace"]):
        for k in ("max_index", "matches", "valid", "rx_timing"):
            assert int(tr[0, n][k]) == t[k], (n, k)
    for n, s in exp["soft"].items():
        np.testing.assert_array_equal(tr[0, int(n)]["soft"], np.array(s, np.float32))


@pytest.mark.parametrize("name", D752)
def test_dec752_synth_goldens(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    assert int(g["mode"]) == oracle.MODE_DEC752
    x = oracle.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    np.testing.assert_array_equal(np.packbits(bits, axis=-1), g["bits"])
    np.testing.assert_array_equal(valid, g["valid"])
    for k in ("max_index", "matches", "rx_timing"):
        np.testing.assert_array_equal(tr[k], g[k])
    vm = valid.astype(bool)
    np.testing.assert_array_equal(tr["soft"][vm], g["soft"][vm])


def test_dec752_differs_from_reference(golden_dir):
    """The mode is a different receiver: same input, different decisions."""
    x = _sample(golden_dir)
    _, _, t0 = oracle.cpu_rx(x, trace=True)
    _, _, t1 = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    assert (t0["max_index"] != t1["max_index"]).any()


@pytest.mark.parametrize("ebn0", [1000.0, 3.0])
def test_dec752_random_channels_vs_padded_reference(ebn0):
    if not oracle.ref_available(oracle.MODE_DEC752):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(9)
    x = np.concatenate([
        oracle.synth(4321 + int(ebn0), 40, 20, ebn0, c0=500),
        np.zeros((1, 20, oracle.FRAME), np.int16),
        np.full((1, 20, oracle.FRAME), -32768, np.int16),
        rng.integers(-32768, 32768, (2, 20, oracle.FRAME)).astype(np.int16),
    ])
    b1, v1, t1 = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_DEC752)
    b2, v2, t2 = oracle.ref_rx(x, trace=True, mode=oracle.MODE_DEC752)
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(b1, b2)
    for k in ("max_index", "matches", "rx_timing"):
        np.testing.assert_array_equal(t1[k], t2[k])
    vm = v2.astype(bool)
    np.testing.assert_array_equal(t1["soft"][vm], t2["soft"][vm])


# ---------------------------------------------------------------- kiss_fft
# The reference's FFT (src/fft.c; nothing in the reference calls it) restated in
# oracle/cpu_ref.c (qc_fft), diffed bit for bit against the compiled reference:
# every radix (4, 2, 3, 5, generic), forward and inverse, signed zeros.
FFT_SIZES = [1, 2, 3, 4, 5, 6, 7, 8, 12, 15, 16, 25, 60, 64, 100, 128, 243, 256, 343, 512,
             1000, 1024, 4096]


@pytest.mark.parametrize("n", FFT_SIZES)
def test_fft_restatement_vs_reference(n):
    if not oracle.ref_fft_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(n)
    cases = [
        (rng.standard_normal(n) + 1j * rng.standard_normal(n)),
        rng.integers(-3, 4, n) + 1j * rng.integers(-3, 4, n),
        rng.standard_normal(n) * 1e4,
    ]
    z = np.zeros(n, np.complex64)
    z.view(np.float32)[:] = rng.choice([-0.0, 0.0, 1.0, -1.0], 2 * n)
    cases.append(z)
    for x in cases:
        x = np.asarray(x, np.complex64)
        for inv in (False, True):
            np.testing.assert_array_equal(oracle.cpu_fft(x, inv).view(np.uint32),
                                          oracle.ref_fft(x, inv).view(np.uint32))


def test_fft_restatement_is_a_dft():
    x = (np.random.default_rng(3).standard_normal(256) * (1 + 1j)).astype(np.complex64)
    np.testing.assert_allclose(oracle.cpu_fft(x), np.fft.fft(x), atol=1e-4)
    np.testing.assert_allclose(oracle.cpu_fft(x, True), np.fft.ifft(x) * 256, atol=1e-4)


# ------------------------------------------------------- FFT-correlation hunt
# The QC_MODE_FFT_HUNT receiver variant replaces the hunt's direct sums by a
# kiss_fft correlation.  The reference never calls its FFT, so no reference
# build of this receiver exists; its hunt is pinned by composing the
# reference's OWN fft() (oracle/_ref/libkissfft_ref.so) in numpy float32.
PRE = np.array(json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                           "fft_hunt_preamble.json"))), np.float32)


def _hunt_with_reference_fft(dec):
    c = np.zeros(256, np.complex64)
    c.real[:128], c.imag[:128] = PRE, -PRE            # conj(preambletable[i])
    C = oracle.ref_fft(c)
    q_r, q_i = C.real, -C.imag                         # Q = conj(C)
    X = oracle.ref_fft(np.asarray(dec, np.complex64)[:256])
    y = np.empty(256, np.complex64)                    # (ac - bd, ad + bc) in float32
    y.real = X.real * q_r - X.imag * q_i
    y.imag = X.real * q_i + X.imag * q_r
    S = oracle.ref_fft(y, True)[:128]
    v = S.real * S.real + S.imag * S.imag              # cnormf, src/qpsk.c:75-80
    best, mi = np.float32(0), 0
    for l in range(128):                               # src/qpsk.c:172-183
        if v[l] > best:
            best, mi = v[l], l
    return mi, q_r + 1j * q_i


def test_fft_hunt_vs_reference_fft():
    if not oracle.ref_fft_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(11)
    for t in range(60):
        dec = (rng.standard_normal(290) + 1j * rng.standard_normal(290)).astype(np.complex64)
        if t % 3 == 0:   # a preamble at a random lag under noise
            lag = int(rng.integers(0, 128))
            dec[lag:lag + 128] += 3 * (PRE + 1j * PRE)
        if t == 1:
            dec[:] = 0
        mi, q = _hunt_with_reference_fft(dec)
        assert oracle.fft_hunt(dec) == mi, t
    np.testing.assert_array_equal(oracle.fft_hunt_spectrum().view(np.uint32),
                                  q.astype(np.complex64).view(np.uint32))


def test_fft_hunt_mode_runs_and_is_the_direct_receiver_here():
    """On the golden channels the FFT hunt picks the same lags as the direct
    correlator (its rounding differs, its argmax does not), so the variant's
    outputs equal the reference's there."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "synth_s3_eb4.npz"))
    x = oracle.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=oracle.MODE_FFT_HUNT)
    np.testing.assert_array_equal(tr["max_index"], g["max_index"])
    np.testing.assert_array_equal(np.packbits(bits, axis=-1), g["bits"])


def test_decimated_frame_kat(golden_dir):
    """Stage KAT: the restatement's decimated_frame[0..289] after
    every call on the sample capture equals the reference's own buffer
    (tests/golden/sample_stages.npz, from oracle/_ref), bit for bit.  This
    pins the mixer, the RRC FIR and the model-A decimation separately from
    the decisions."""
    st = np.load(os.path.join(golden_dir, "sample_stages.npz"))
    dec = oracle.cpu_stages(_sample(golden_dir)[0])
    np.testing.assert_array_equal(dec.view(np.uint32), st["dec"].view(np.uint32))


def test_decimated_frame_dec752_vs_padded_reference():
    if not oracle.ref_available(oracle.MODE_DEC752):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    x = oracle.synth(77, 1, 12, 4.0)[0]
    ref_dec = oracle.ref_stages(x, mode=oracle.MODE_DEC752)[0]
    dec = oracle.cpu_stages(x, mode=oracle.MODE_DEC752)
    np.testing.assert_array_equal(dec.view(np.uint32), ref_dec.view(np.uint32))
