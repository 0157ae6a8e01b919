"""Parity of the MI355X receive path with the reference (run with -m gpu).

Every comparison is exact: bits, valid flags, max_index/matches/rx_timing
traces and the soft I/Q symbols of valid frames are compared bit for bit
(the north_star's 1e-5 RMS soft-symbol tolerance is therefore
met with zero error).  Expected values come from the golden fixtures made by
the unmodified reference (tests/golden/make_golden.py) and, at larger sizes,
from the oracle restatement (oracle/cpu_ref.c), itself pinned to the reference
by tests/test_oracle.py.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu

SYNTH = ["synth_s1_clean", "synth_s2_eb8", "synth_s3_eb4", "synth_s4_eb0"]


def _sample(golden_dir):
    return sc.read_raw(os.path.join(golden_dir, "preamble_qpsk_8k.raw"))


def _assert_same(out, bits, valid, tr):
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_array_equal(out["bits"], bits)
    if tr is not None and "trace" in out:
        t = out["trace"]
        np.testing.assert_array_equal(t[..., 0], tr["max_index"])
        np.testing.assert_array_equal(t[..., 1], tr["matches"])
        np.testing.assert_array_equal(t[..., 2], tr["valid"])
        np.testing.assert_array_equal(t[..., 3], tr["rx_timing"])
    if tr is not None and "soft" in out:
        vm = valid.astype(bool)
        np.testing.assert_array_equal(out["soft"][vm], tr["soft"][vm])
        assert not out["soft"][~vm].any()


def _vs_oracle(x, **kw):
    rx = sc.Receiver(x.shape[0])
    out = rx.demod(x, trace=True, soft=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    _assert_same(out, bits, valid, tr)
    rx.close()
    return out


def test_sample_file_md5(golden_dir):
    """C1 config: preamble_qpsk_8k.raw -> reference output file md5."""
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    frames = _sample(golden_dir)
    rx = sc.Receiver(1)
    out = rx.demod(frames[None], trace=True, soft=True)
    recs = sc.records(out["bits"][0], out["valid"][0])
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"] == "b56a4d3609d0312934aaef69903c5298"
    for n, t in enumerate(exp["trace"]):
        assert list(out["trace"][0, n]) == [t["max_index"], t["matches"], t["valid"], t["rx_timing"]]
    st = np.load(os.path.join(golden_dir, "sample_stages.npz"))
    vm = st["valid"].astype(bool)
    np.testing.assert_array_equal(out["soft"][0][vm], st["soft"][vm])


def test_reference_surface_rx_frame(golden_dir):
    """qpsk_rx_frame() drop-in (headers/qpsk_internal.h:83) frame by frame."""
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    sc.qpsk_rx_init()
    recs = b""
    for fr in _sample(golden_dir):
        v, b = sc.qpsk_rx_frame(fr)
        if v:
            recs += np.concatenate([b, np.zeros(434, np.uint8)]).tobytes()
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"]


@pytest.mark.parametrize("name", SYNTH)
def test_synth_goldens(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    x = oracle.synth(int(g["seed"]), int(g["nch"]), int(g["nframes"]), float(g["ebn0_db"]))
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["input_sha256"])
    rx = sc.Receiver(x.shape[0])
    out = rx.demod(x, trace=True, soft=True)
    np.testing.assert_array_equal(np.packbits(out["bits"], axis=-1), g["bits"])
    np.testing.assert_array_equal(out["valid"], g["valid"])
    np.testing.assert_array_equal(out["trace"][..., 0], g["max_index"])
    np.testing.assert_array_equal(out["trace"][..., 1], g["matches"])
    np.testing.assert_array_equal(out["trace"][..., 3], g["rx_timing"])
    np.testing.assert_array_equal(out["soft"], g["soft"])


def test_c2_4096_channels():
    """C2 config: 4096 synthetic channels x 16 frames, bit-exact."""
    x = oracle.synth(1, 4096, 16)
    out = _vs_oracle(x)
    assert 0.2 < out["valid"].mean() < 0.7


@pytest.mark.parametrize("nch", [1, 2, 63, 65, 130])
def test_ragged_channel_counts(nch):
    x = oracle.synth(77 + nch, nch, 12, 5.0)
    _vs_oracle(x)


def test_edge_inputs():
    rng = np.random.default_rng(5)
    x = np.stack([
        np.zeros((8, 1880), np.int16),
        np.full((8, 1880), 32767, np.int16),
        np.full((8, 1880), -32768, np.int16),
        np.tile(np.array([32767, -32768], np.int16), (8, 940)),
        rng.integers(-32768, 32768, (8, 1880)).astype(np.int16),
        rng.integers(-3, 4, (8, 1880)).astype(np.int16),
    ])
    _vs_oracle(x)


@pytest.mark.parametrize("shape", [None, "4x2", "2x4d"])
@pytest.mark.parametrize("shift", [4, 8, 11])
def test_low_amplitude_streams(shift, shape, monkeypatch):
    """Synthetic streams scaled down by 2^shift (quantised to a few int16
    levels at 11): correlations that tie exactly or nearly, which the
    filtered hunt hands to the exact chain (qpsk_hunt.h hunt_index); on the
    default (dual-chain, quad) shape for this batch and forced 4x2 / 2x4d."""
    if shape:
        monkeypatch.setenv("QPSK_SHAPE", shape)
    x = (oracle.synth(31 + shift, 256, 12, 8.0).astype(np.int32) >> shift).astype(np.int16)
    _vs_oracle(x)


def test_streaming_split_equals_one_call():
    """State (rx_timing, carried symbols, sample history, frame counter) persists
    across calls: feeding 16 frames as 5+1+1+9 == one 16-frame call."""
    x = oracle.synth(9, 192, 16, 6.0)
    rx1 = sc.Receiver(192)
    whole = rx1.demod(x, trace=True, soft=True)
    rx2 = sc.Receiver(192)
    parts = [rx2.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True)
             for a, b in ((0, 5), (5, 6), (6, 7), (7, 16))]
    assert rx2.frames == 16
    for k in ("bits", "valid", "trace", "soft"):
        np.testing.assert_array_equal(np.concatenate([p[k] for p in parts], axis=1), whole[k])
    rx2.reset()
    again = rx2.demod(x, trace=True, soft=True)
    np.testing.assert_array_equal(again["bits"], whole["bits"])


def test_independent_contexts():
    xa = oracle.synth(21, 70, 8)
    xb = oracle.synth(22, 70, 8, 4.0)
    ra, rb = sc.Receiver(70), sc.Receiver(70)
    oa1 = ra.demod(xa[:, :4])
    ob = rb.demod(xb)
    oa2 = ra.demod(np.ascontiguousarray(xa[:, 4:]))
    bits, valid, _ = oracle.cpu_rx(xa)
    np.testing.assert_array_equal(np.concatenate([oa1["bits"], oa2["bits"]], 1), bits)
    np.testing.assert_array_equal(ob["bits"], oracle.cpu_rx(xb)[0])


def test_device_api_torch():
    import torch
    x = oracle.synth(31, 256, 10, 7.0)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    rx = sc.Receiver(256)
    dx = torch.from_numpy(x).cuda()
    db = torch.zeros((256, 10, 62), dtype=torch.uint8, device="cuda")
    dv = torch.zeros((256, 10), dtype=torch.uint8, device="cuda")
    dt = torch.zeros((256, 10, 4), dtype=torch.int32, device="cuda")
    ds = torch.zeros((256, 10, 31, 2), dtype=torch.float32, device="cuda")
    rx.demod_device(dx, db, dv, dt, ds)
    torch.cuda.synchronize()
    _assert_same({"bits": db.cpu().numpy(), "valid": dv.cpu().numpy(),
                  "trace": dt.cpu().numpy(), "soft": ds.cpu().numpy()}, bits, valid, tr)


@pytest.mark.parametrize("ebn0", [0.0, 3.0, 6.0, 10.0])
def test_awgn_sweep_points(ebn0):
    """C5 config points (reduced channel count): zero disagreement vs reference."""
    x = oracle.synth(500 + int(ebn0), 1024, 16, ebn0)
    _vs_oracle(x)


def test_full_size_c3():
    """C3 config at full size (65536 channels x 32 frames): every channel's
    bits, valid flags, trace (max_index, matches, rx_timing) and the soft
    symbols of every valid frame equal the oracle's, bit for bit."""
    nch, nf = 65536, 32
    x = oracle.synth(3, nch, nf)
    rx = sc.Receiver(nch)
    out = rx.demod(x, trace=True, soft=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    _assert_same(out, bits, valid, tr)


@pytest.mark.parametrize("ebn0", [0.0, 5.0, 10.0])
def test_c5_awgn_full_channel_count(ebn0):
    """C5 (BASELINE configs[4]) on the default kernel at its stated channel
    count: 65,536 AWGN channels x 16 frames; bits, valid flags and the trace
    equal the oracle's (the validity decision of src/qpsk.c:196 under noise)."""
    nch, nf = 65536, 16
    x = oracle.synth(3, nch, nf, ebn0)
    rx = sc.Receiver(nch)
    out = rx.demod(x, trace=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    _assert_same(out, bits, valid, tr)
    assert 0 < valid.sum() < valid.size


def test_c_driver_single_and_batch(golden_dir, tmp_path):
    """The C driver (examples/qpsk_rx_raw.c) reproduces the reference's output
    file: frame-by-frame through qpsk_rx_frame(), and as one channel of a
    batched qpsk_rx_batch() call next to synthetic channels."""
    import subprocess
    exe = os.path.join(os.path.dirname(golden_dir), "..", "examples", "qpsk_rx_raw")
    exe = os.path.abspath(exe)
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True)
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    raw = os.path.join(golden_dir, "preamble_qpsk_8k.raw")
    out = tmp_path / "single.bin"
    subprocess.run([exe, raw, str(out)], check=True)
    assert hashlib.md5(out.read_bytes()).hexdigest() == exp["output_md5"]
    # batch: the sample file plus two synthetic 14-frame channels
    paths = [raw]
    syn = oracle.synth(99, 2, 14, 6.0)
    for i in range(2):
        p = tmp_path / f"syn{i}.raw"
        syn[i].tofile(p)
        paths.append(str(p))
    subprocess.run([exe, "-b", *paths, "-o", str(tmp_path / "ch")], check=True)
    assert hashlib.md5((tmp_path / "ch0.bin").read_bytes()).hexdigest() == exp["output_md5"]
    bits, valid, _ = oracle.cpu_rx(syn)
    for i in range(2):
        assert (tmp_path / f"ch{i + 1}.bin").read_bytes() == sc.records(bits[i], valid[i])


@pytest.mark.parametrize("shape", ["4x2", "2x4d", "1x8"])
def test_every_workgroup_shape(shape, monkeypatch):
    """rx_kernel<G, FP> (groups per workgroup x front waves per group) is chosen
    by batch size (pick_shape); QPSK_SHAPE forces each one on the same ragged
    batch."""
    monkeypatch.setenv("QPSK_SHAPE", shape)
    x = oracle.synth(61, 300, 12, 5.0)
    _vs_oracle(x)


def test_split_fir_window_boundary(monkeypatch):
    """The 4x2 kernel's split FIR computes dec[255..289] (F_{n+1}[67..101])
    only after the hunt and only when mi >= 93, where the window's observable
    part (dec[mi .. mi+162]) reaches them.  On a forced 4x2 batch every output
    must be exact, and the batch must hold valid frames on both sides of the
    boundary, the data symbols of the mi >= 93 ones read from the late pass."""
    monkeypatch.setenv("QPSK_SHAPE", "4x2")
    x = oracle.synth(71, 512, 8, 8.0)
    out = _vs_oracle(x)
    mi = out["trace"][..., 0][out["valid"].astype(bool)]
    assert (mi >= 93).sum() > 20 and ((mi < 93) & (mi >= 80)).sum() > 5, np.bincount(mi)
    # pass 1's lane 63 and pass 2's lane map follow rx_timing mod 32 (the LDS
    # bank pair lanes 32..62 leave free, qpsk_rx.hip split_r): every residue ran
    rt_in = np.concatenate([np.full((x.shape[0], 1), 3), out["trace"][:, :-1, 3]], axis=1)
    assert len(np.unique((rt_in - 295) & 31)) == 32


@pytest.mark.parametrize("width", ["16", "32", "64"])
def test_dual_chain_group_widths(width, monkeypatch):
    """One group per workgroup runs the dual-chain kernel (back waves for the
    even and the odd frames, LDS progress counters); QPSK_WIDTH forces its
    group width (channels per workgroup) on one ragged batch, and with it the
    back layout: a quad of lanes per channel at W = 16 / 32 (back_frame_quad,
    W / 16 back waves per frame chain), a lane per channel at W = 64 (which
    also moves 2 channels between the front waves, pick_shape's split)."""
    monkeypatch.setenv("QPSK_WIDTH", width)
    x = oracle.synth(64, 333, 15, 4.0)
    _vs_oracle(x)


@pytest.mark.parametrize("shape,width", [("4x2", None), ("2x4d", None), ("1x8", "64"),
                                         ("1x8", "32"), ("1x8", "16")])
def test_head_prepass(shape, width, monkeypatch):
    """SURVEY.md 8f rank 4, the frame-parallel FIR-head pre-pass
    (QPSK_HEADPASS=1): head_kernel computes every channel-frame's
    rx_timing-independent F_{n+1}[0..101] ahead of the frame loop and the
    fronts copy it instead of filtering.  Every shape, a ragged AWGN batch
    with silent and saturated channels, every output exact."""
    monkeypatch.setenv("QPSK_HEADPASS", "1")
    monkeypatch.setenv("QPSK_SHAPE", shape)
    if width:
        monkeypatch.setenv("QPSK_WIDTH", width)
    x = oracle.synth(95, 300, 11, 5.0)
    x[7] = 0
    x[8] = 32767
    _vs_oracle(x)


def test_head_prepass_across_call_splits(monkeypatch):
    """The pre-pass reads frame n-1's tail from the carried history for a
    call's first frame: calls of 1, 1, 4, 1 and the remaining frames."""
    monkeypatch.setenv("QPSK_HEADPASS", "1")
    nch, nf = 260, 12
    x = oracle.synth(96, nch, nf, 4.0)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    rx = sc.Receiver(nch)
    parts, a = [], 0
    for b in (1, 2, 6, 7, nf):
        parts.append(rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True))
        a = b
    out = {k: np.concatenate([p[k] for p in parts], axis=1) for k in ("bits", "valid", "trace", "soft")}
    _assert_same(out, bits, valid, tr)


@pytest.mark.parametrize("nch", [8192, 16384])
def test_head_prepass_c4_shards(nch, monkeypatch):
    """The pre-pass at the C4 N = 8 and N = 4 shard sizes (x 32 frames, AWGN)."""
    monkeypatch.setenv("QPSK_HEADPASS", "1")
    x = oracle.synth(97, nch, 32, 6.0)
    _vs_oracle(x)


@pytest.mark.parametrize("width", [None, "32"])
@pytest.mark.parametrize("ebn0", [1000.0, 6.0, 0.0])
def test_quad_back_edges_and_noise(ebn0, width, monkeypatch):
    """The quad-per-channel back (160 channels: W = 16, or W = 32 forced) on
    saturated, zero and constant channels next to noisy ones (sign-of-zero and
    padding paths of back_frame_quad), every output exact."""
    if width:
        monkeypatch.setenv("QPSK_WIDTH", width)
    x = oracle.synth(71, 160, 9, ebn0)
    x[3] = 0
    x[17] = 32767
    x[18] = -32768
    x[40, 2:5] = 0
    x[77, :, ::2] = 12345
    _vs_oracle(x)


@pytest.mark.parametrize("width", [None, "32"])
def test_quad_back_exact_division(width, monkeypatch):
    """QPSK_FORCE_EXACT on the quad back (100 channels: W = 16, or W = 32
    forced: two back waves per frame chain): the IEEE-division retrain path."""
    monkeypatch.setenv("QPSK_FORCE_EXACT", "1")
    if width:
        monkeypatch.setenv("QPSK_WIDTH", width)
    x = oracle.synth(72, 100, 8, 4.0)
    _vs_oracle(x)


@pytest.mark.parametrize("ngpu,c0", [(2, 32768), (4, 16384), (8, 57344)])
def test_c4_shards_at_size(ngpu, c0):
    """C4 (BASELINE configs[3]): the shard rank g of `bench.py --gpus N`
    demodulates, at its stated size -- 65,536 / N channels x 32 frames, AWGN --
    with the shape pick_shape selects for it (N = 2: 2x4 dual-chain, lane
    backs; N = 4: 1x8 dual W = 64, lane backs, split 2; N = 8: 1x8 dual W = 32,
    quad backs).  The shard's channels are the batch's channels
    [c0, c0 + 65536 / N) (oracle.synth's channel offset): ranks 1, 1 and 7
    of the three splits.  Every output, soft symbols included, equals the
    oracle's (the loop being split is src/qpsk.c:436-458)."""
    nch = 65536 // ngpu
    x = oracle.synth(81, nch, 32, 6.0, c0=c0)
    _vs_oracle(x)



def test_progress_wait_timeout_is_an_error(monkeypatch):
    """A dual-chain progress wait that runs past its bound must surface as
    QPSK_ESTALL, never as silently different bits (src/qpsk.c:447: every
    frame's result is defined).  QPSK_DEBUG_STALL adds one wait that cannot end
    (short bound) to the first back wave of workgroup 0; the call reports the
    error, and a new context without the knob is clean."""
    x = oracle.synth(66, 96, 6, 4.0)
    monkeypatch.setenv("QPSK_DEBUG_STALL", "1")
    rx = sc.Receiver(96)   # 96 channels: a dual-chain shape
    with pytest.raises(sc.QpskError) as ei:
        rx.demod(x)
    assert ei.value.code == sc.QPSK_ESTALL
    rx.close()
    monkeypatch.delenv("QPSK_DEBUG_STALL")
    _vs_oracle(x)


def test_progress_wait_timeout_is_an_error_tiny_call(monkeypatch):
    """The same for a host call of <= 64 channel-frames (8 channels x 4 frames),
    which runs on the pinned staging block and gets the error word from
    rx_data_kernel (no separate launch): the stall still comes back as
    QPSK_ESTALL, and the word is cleared by being taken."""
    x = oracle.synth(67, 8, 4, 4.0)
    monkeypatch.setenv("QPSK_DEBUG_STALL", "1")
    rx = sc.Receiver(8)
    with pytest.raises(sc.QpskError) as ei:
        rx.demod(x)
    assert ei.value.code == sc.QPSK_ESTALL
    assert sc.lib().qpsk_rx_sync(rx._h) == 0   # taken by the call
    rx.close()
    monkeypatch.delenv("QPSK_DEBUG_STALL")
    _vs_oracle(x)


@pytest.mark.parametrize("nch", [8, 96, 33000])
def test_mis_shaped_launch_is_an_error(nch, monkeypatch):
    """rx_kernel's roles are fixed per instantiation; a launch with a block
    that does not hold them (QPSK_DEBUG_BLOCK: one wave short) would leave
    every progress wait to run to its bound.  The kernel refuses it at once:
    the call reports QPSK_ESTALL (tiny host call, dual-chain and 4x2 shapes),
    and a new context without the knob is exact."""
    x = oracle.synth(68, nch, 2, 4.0)
    monkeypatch.setenv("QPSK_DEBUG_BLOCK", "1")
    rx = sc.Receiver(nch)
    with pytest.raises(sc.QpskError) as ei:
        rx.demod(x)
    assert ei.value.code == sc.QPSK_ESTALL
    rx.close()
    monkeypatch.delenv("QPSK_DEBUG_BLOCK")
    if nch <= 96:
        _vs_oracle(x)


def test_exact_division_fallback(monkeypatch):
    """The Kalman step's fast reciprocal has an exact-division fallback that
    recomputes a whole frame (rx_kernel) or job (rx_data_kernel) when an
    operand leaves the fast path's range; QPSK_FORCE_EXACT takes it for every
    frame, and the outputs must not change."""
    monkeypatch.setenv("QPSK_FORCE_EXACT", "1")
    x = oracle.synth(63, 200, 10, 4.0)
    _vs_oracle(x)


def test_long_stream_crosses_the_keystream_period():
    """The descrambler's keystream repeats every 32,767 bits = 1,057 frames of 62
    bits minus 1 (src/scramble.c: 15-bit LFSR); the GPU indexes it by the
    global frame counter.  1,100 frames fed in uneven calls == the oracle."""
    nch, nf = 48, 1100
    x = oracle.synth(123, nch, nf, 1000.0)
    bits, valid, _ = oracle.cpu_rx(x)
    rx = sc.Receiver(nch)
    outs, a = [], 0
    for b in (300, 1, 499, 300):
        outs.append(rx.demod(np.ascontiguousarray(x[:, a:a + b])))
        a += b
    assert rx.frames == nf
    np.testing.assert_array_equal(np.concatenate([o["valid"] for o in outs], 1), valid)
    np.testing.assert_array_equal(np.concatenate([o["bits"] for o in outs], 1), bits)
    assert valid[:, 1057:].any()


def test_per_call_job_limit():
    """The data-job queue is addressed with 32-bit byte offsets: a call of
    nch * nframes >= 2^28 channel-frames (1 TB of input) is refused with
    QPSK_EINVAL before any device work (include/qpsk_batch.h)."""
    import ctypes as C
    rx = sc.Receiver(65536)
    L = sc.lib()
    fake = C.c_void_p(1 << 20)   # 16-B aligned, never dereferenced
    r = L.qpsk_rx_batch_device(rx._h, fake, 4096, fake, fake, None, None, None)
    assert r == -1
    # the context is still usable
    x = oracle.synth(76, 65536, 1, 1000.0)
    np.testing.assert_array_equal(rx.demod(x)["bits"], oracle.cpu_rx(x)[0])


@pytest.mark.parametrize("seed", range(6))
def test_random_batches_and_splits(seed):
    """Seeded random shapes: channel count (ragged groups, every shape the
    batch size selects), frame count, Eb/N0 and how the frames are split over
    calls; everything (bits, flags, trace, soft) equals the oracle."""
    rng = np.random.default_rng(900 + seed)
    nch = int(rng.choice([1, 17, 64, 200, 777, 3000, 16500, 40000]))
    nf = int(rng.integers(2, 12))
    ebn0 = float(rng.choice([1000.0, 8.0, 4.0, 1.0]))
    x = oracle.synth(1000 + seed, nch, nf, ebn0)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    cuts = sorted(set(int(c) for c in rng.integers(1, nf, size=2)))
    rx = sc.Receiver(nch)
    parts, a = [], 0
    for b in cuts + [nf]:
        parts.append(rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True))
        a = b
    out = {k: np.concatenate([p[k] for p in parts], axis=1) for k in ("bits", "valid", "trace", "soft")}
    _assert_same(out, bits, valid, tr)


@pytest.mark.parametrize("nch", [100, 333, 8192])
def test_quad_backs_across_call_splits(nch):
    """Quad-back batches (<= 32 channels per CU) fed as calls of 1, 1, 4, 1 and
    the remaining frames: the dual-chain state (both chains' rx_timing and
    preamble positions, the frame parity of the windows) crosses every call
    boundary, and every output equals the oracle."""
    nf = 13 if nch < 1000 else 9
    x = oracle.synth(140 + nch, nch, nf, 5.0 if nch != 333 else 1000.0)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    rx = sc.Receiver(nch)
    parts, a = [], 0
    for b in (1, 2, 6, 7, nf):
        parts.append(rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True))
        a = b
    out = {k: np.concatenate([p[k] for p in parts], axis=1) for k in ("bits", "valid", "trace", "soft")}
    _assert_same(out, bits, valid, tr)


def _gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.parametrize("mode", [sc.MODE_REFERENCE, sc.MODE_DEC752, sc.MODE_DEC752 | sc.MODE_FFT_HUNT])
def test_state_snapshot_resumes_exactly(mode):
    """Checkpoint / resume (qpsk_rx_state_save / _load): 7 frames
    on context A, a snapshot, loaded into a fresh context B (the second GPU
    when there is one), 9 more frames there == one 16-frame call, bit for
    bit, soft symbols included; and == the oracle (the statics being carried
    are src/qpsk.c:34-53 and src/scramble.c:41-42).  In every receiver mode
    (dec752's front reads a longer history)."""
    nch, nf, cut = 300, 16, 7
    x = oracle.synth(150, nch, nf, 5.0)
    whole = sc.Receiver(nch, mode=mode).demod(x, trace=True, soft=True)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=mode)
    _assert_same(whole, bits, valid, tr)
    a = sc.Receiver(nch, mode=mode)
    first = a.demod(np.ascontiguousarray(x[:, :cut]), trace=True, soft=True)
    snap = a.state_save()
    assert len(snap) == sc.lib().qpsk_rx_state_size(nch)
    a.close()
    b = sc.Receiver(nch, device=1 if _gpus() > 1 else 0, mode=mode)
    b.state_load(snap)
    assert b.frames == cut
    rest = b.demod(np.ascontiguousarray(x[:, cut:]), trace=True, soft=True)
    for k in ("bits", "valid", "trace", "soft"):
        np.testing.assert_array_equal(np.concatenate([first[k], rest[k]], axis=1), whole[k])


def test_state_snapshot_moves_a_channel_range_between_shapes():
    """Channels [5000, 5128) of a 20,000-channel context (the 2x4 dual-chain
    shape, lane backs) continue on a 128-channel context (1x8, quad backs):
    the snapshot is the per-channel state, independent of the kernel shape.
    Also: a context that has received frames takes only a snapshot of its own
    frame index, and a snapshot of another receiver mode is refused."""
    nch, nf, cut, c0, n = 20000, 10, 6, 5000, 128
    x = oracle.synth(151, nch, nf, 3.0)
    whole = sc.Receiver(nch).demod(x, trace=True, soft=True)
    a = sc.Receiver(nch)
    a.demod(np.ascontiguousarray(x[:, :cut]))
    snap = a.state_save(c0, n)
    b = sc.Receiver(n)
    b.state_load(snap)
    rest = b.demod(np.ascontiguousarray(x[c0:c0 + n, cut:]), trace=True, soft=True)
    for k in ("bits", "valid", "trace", "soft"):
        np.testing.assert_array_equal(rest[k], whole[k][c0:c0 + n, cut:])
    # b is now at frame nf != the snapshot's cut: refused
    with pytest.raises(sc.QpskError) as ei:
        b.state_load(snap)
    assert ei.value.code == sc.QPSK_EINVAL
    d = sc.Receiver(n, mode=sc.MODE_DEC752)
    with pytest.raises(sc.QpskError) as ei:
        d.state_load(snap)
    assert ei.value.code == sc.QPSK_EINVAL
    bad = bytearray(snap)
    bad[0] ^= 1
    with pytest.raises(sc.QpskError):
        sc.Receiver(n).state_load(bytes(bad))
