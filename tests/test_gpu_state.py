"""Checkpoint / resume guards (qpsk_rx_state_save / _load; run with -m gpu).

The reference keeps the receiver's per-channel state in statics
(/root/reference/src/qpsk.c:34-53) and the descrambler register, a function
of the frame index, in src/scramble.c:41-42.  A snapshot carries one
channel range's state and the context's frame index.  These tests pin what
the round-5 review found unguarded:
- a channel range loaded into a fresh context at frame G != 0 moves the
  context's (shared) frame index; its other channels would restart from reset
  state at keystream offset 62 G, which no reference run produces, so the
  context refuses to receive until every channel has been loaded;
- a snapshot is a function of the channels' state alone (the window slots no
  output reads are zeroed), whatever the context's size or kernel shape;
- a stalled context (QPSK_ESTALL: state undefined) refuses to export;
- a snapshot crosses processes: saved to a file by one, loaded by another.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("bits", "valid", "trace", "soft")


def _cat(parts):
    return {k: np.concatenate([p[k] for p in parts], axis=1) for k in KEYS}


def _raises(code, fn, *a):
    with pytest.raises(sc.QpskError) as ei:
        fn(*a)
    assert ei.value.code == code


def test_partial_load_into_fresh_context_waits_for_every_channel():
    nch, nf, cut = 200, 10, 6
    x = oracle.synth(160, nch, nf, 6.0)
    whole = sc.Receiver(nch).demod(x, trace=True, soft=True)
    a = sc.Receiver(nch)
    a.demod(np.ascontiguousarray(x[:, :cut]))
    s1, s2 = a.state_save(0, 120), a.state_save(120, 80)
    b = sc.Receiver(nch)
    b.state_load(s1, 0)
    assert b.frames == cut
    rest = np.ascontiguousarray(x[:, cut:])
    _raises(sc.QPSK_EINVAL, b.demod, rest)        # channels 120..199 not loaded yet
    _raises(sc.QPSK_EINVAL, b.state_save, 0, 120)
    b.state_load(s1, 0)                           # again: still 80 to go
    _raises(sc.QPSK_EINVAL, b.demod, rest)
    b.state_load(s2, 120)
    out = b.demod(rest, trace=True, soft=True)
    for k in KEYS:
        np.testing.assert_array_equal(out[k], whole[k][:, cut:])
    # a reset abandons the assembly: frame 0, every channel in reset state
    c = sc.Receiver(nch)
    c.state_load(s2, 120)
    c.reset()
    assert c.frames == 0
    o = c.demod(x, trace=True, soft=True)
    for k in KEYS:
        np.testing.assert_array_equal(o[k], whole[k])
    # a frame-0 snapshot moves no frame index: a partial load needs no others
    z = sc.Receiver(nch).state_save(0, 50)
    d = sc.Receiver(nch)
    d.state_load(z, 10)
    o = d.demod(x, trace=True, soft=True)
    for k in KEYS:
        np.testing.assert_array_equal(o[k], whole[k])


@pytest.mark.parametrize("shape", [None, "4x2"])
def test_snapshot_is_a_function_of_the_channel_state(shape, monkeypatch):
    """Channels 200..299 in a 300-channel context and alone in a 100-channel
    one reach the same state by different kernel schedules (the fronts' dec
    buffers hold other channels' entries past what the window uses; 4x2: the
    split FIR leaves dec[255..289] for mi < 93): the snapshots are equal byte
    for byte, and equal again when taken twice."""
    if shape:
        monkeypatch.setenv("QPSK_SHAPE", shape)
    nf = 9
    x = oracle.synth(161, 300, nf, 8.0)
    a, b = sc.Receiver(300), sc.Receiver(100)
    a.demod(x)
    b.demod(np.ascontiguousarray(x[200:]))
    sa, sb = a.state_save(200, 100), b.state_save(0, 100)
    off = 64 + 100 * (2 * 1880 * 2 + 168 * 8)        # header, history, windows: then mi
    mi = np.frombuffer(sa[off:off + 400], np.int32)
    assert (mi < 93).any() and (mi >= 124).any()   # both sides of every stale range
    assert sa == sb
    assert a.state_save(200, 100) == sa


def test_stalled_context_refuses_to_export(monkeypatch):
    """QPSK_DEBUG_STALL=first: the context's first call stalls (QPSK_ESTALL);
    its state is undefined and state_save refuses with QPSK_ESTALL until a
    reset.  A stall not yet taken by qpsk_rx_sync (device call) is seen too,
    without taking it: the sync still reports it."""
    import torch
    x = oracle.synth(162, 96, 6, 4.0)
    monkeypatch.setenv("QPSK_DEBUG_STALL", "first")
    rx = sc.Receiver(96)                           # 96 channels: a dual-chain shape
    _raises(sc.QPSK_ESTALL, rx.demod, x)
    _raises(sc.QPSK_ESTALL, rx.state_save)
    rx.reset()
    rx.demod(x)                                    # the knob stalls the first launch only
    assert len(rx.state_save()) == sc.lib().qpsk_rx_state_size(96)
    rx.close()
    dv = sc.Receiver(96)
    dx = torch.from_numpy(x).cuda()
    db = torch.zeros((96, 6, 62), dtype=torch.uint8, device="cuda")
    dvl = torch.zeros((96, 6), dtype=torch.uint8, device="cuda")
    dv.demod_device(dx, db, dvl)
    _raises(sc.QPSK_ESTALL, dv.state_save)         # peeked in the error word
    _raises(sc.QPSK_ESTALL, dv.sync)               # still there for the sync
    _raises(sc.QPSK_ESTALL, dv.state_save)
    monkeypatch.delenv("QPSK_DEBUG_STALL")


_CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    sys.path.insert(0, {root!r})
    import singlecarrier_amd as sc
    step, d = sys.argv[1], sys.argv[2]
    x = np.load(d + "/x.npy")
    nch, cut = x.shape[0], int(sys.argv[3])
    rx = sc.Receiver(nch)
    if step == "save":
        out = rx.demod(np.ascontiguousarray(x[:, :cut]), trace=True, soft=True)
        open(d + "/snap.bin", "wb").write(rx.state_save())
    else:
        rx.state_load(open(d + "/snap.bin", "rb").read())
        assert rx.frames == cut
        out = rx.demod(np.ascontiguousarray(x[:, cut:]), trace=True, soft=True)
    np.savez(d + "/" + step + ".npz", **out)
""")


def test_snapshot_crosses_processes(tmp_path):
    """One process demodulates 5 frames and writes its snapshot to a file; a
    second process reads it and demodulates the other 7: together they equal
    one 12-frame call in this process, bit for bit."""
    nch, nf, cut = 260, 12, 5
    x = oracle.synth(163, nch, nf, 5.0)
    np.save(tmp_path / "x.npy", x)
    script = tmp_path / "child.py"
    script.write_text(_CHILD.format(root=ROOT))
    for step in ("save", "load"):
        r = subprocess.run([sys.executable, str(script), step, str(tmp_path), str(cut)],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
    whole = sc.Receiver(nch).demod(x, trace=True, soft=True)
    parts = [dict(np.load(tmp_path / f"{s}.npz")) for s in ("save", "load")]
    got = _cat(parts)
    for k in KEYS:
        np.testing.assert_array_equal(got[k], whole[k])
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    np.testing.assert_array_equal(got["bits"], bits)
    np.testing.assert_array_equal(got["valid"], valid)
