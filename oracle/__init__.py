"""TEST INFRASTRUCTURE ONLY -- the oracle.

ctypes bindings for
  * ``oracle/libqpsk_cpu.so``  -- clean-room C restatement of the reference RX
    path (``oracle/cpu_ref.c``), plus the TX restatement used for synthesis;
  * ``oracle/_ref/libqpsk_ref.so`` -- the UNMODIFIED reference sources compiled
    from /root/reference by ``oracle/Makefile`` (present in the build container
    and shipped prebuilt to the GPU box; never required).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
import this package, and only as the checker / baseline -- the product path
(``singlecarrier_amd``) never touches it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FRAME = 1880
NBITS = 62
NDSYM = 31

TRACE_DTYPE = np.dtype([("max_index", "<i4"), ("matches", "<i4"), ("valid", "<i4"),
                        ("rx_timing", "<i4"), ("soft", "<f4", (31, 2))])
REF_TRACE_DTYPE = np.dtype([("max_index", "<i4"), ("matches", "<i4"), ("valid", "<i4"),
                            ("rx_timing", "<i4"), ("soft", "<f4", (31, 2)),
                            ("raw_dibit", "u1", (31,)), ("pad", "u1", (1,))])
assert TRACE_DTYPE.itemsize == 264 and REF_TRACE_DTYPE.itemsize == 296

_cpu = None
_ref = None


def build(ref: bool = True) -> None:
    """Compile the restatement (always) and the reference harness (when the
    reference tree is present).  Building the checker is not using it."""
    subprocess.run(["make", "-s", "-C", HERE, "cpu"], check=True)
    if ref and os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def cpu_lib():
    global _cpu
    if _cpu is None:
        path = os.path.join(HERE, "libqpsk_cpu.so")
        if not os.path.exists(path):
            build(ref=False)
        lib = C.CDLL(path)
        lib.qc_rx_batch.restype = C.c_long
        lib.qc_rx_batch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_int]
        lib.qc_rx_batch_mode.restype = C.c_long
        lib.qc_rx_batch_mode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_int, C.c_int]
        lib.qc_synth_batch.restype = None
        lib.qc_synth_batch.argtypes = [C.c_uint64, C.c_uint32, C.c_int, C.c_double,
                                       C.c_void_p, C.c_long, C.c_int]
        lib.qc_mixer_table.argtypes = [C.c_void_p]
        lib.qc_fft.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.qc_fft_twiddles.argtypes = [C.c_int, C.c_int, C.c_void_p]
        lib.qc_rx_stages.restype = C.c_long
        lib.qc_rx_stages.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        lib.qc_fft_hunt.restype = C.c_int
        lib.qc_fft_hunt.argtypes = [C.c_void_p]
        lib.qc_fft_hunt_spectrum.argtypes = [C.c_void_p]
        lib.qc_keystream.argtypes = [C.c_void_p, C.c_int]
        _cpu = lib
    return _cpu


# receiver semantics (cpu_ref.h QC_MODE_*; singlecarrier_amd.MODE_*)
MODE_REF = 0      # the reference as built (gcc -O2, "model A" overflow)
MODE_DEC752 = 1   # decimated_frame[752] ("intended semantics", NOT reference parity)
MODE_FFT_HUNT = 2  # flag: the preamble hunt correlates through kiss_fft (src/fft.c)
_REF_LIBS = {MODE_REF: "libqpsk_ref.so", MODE_DEC752: "libqpsk_ref752.so"}   # no FFT-hunt build:
# the reference never calls its FFT; that variant is pinned per component


def ref_available(mode: int = MODE_REF) -> bool:
    return mode in _REF_LIBS and os.path.exists(os.path.join(HERE, "_ref", _REF_LIBS[mode]))


def ref_lib(mode: int = MODE_REF):
    """The reference build for `mode`: libqpsk_ref.so, or libqpsk_ref752.so (the
    same unmodified sources with decimated_frame followed by owned padding,
    oracle/ref/dec752.ld)."""
    global _ref
    if _ref is None:
        _ref = {}
    if mode not in _ref:
        lib = C.CDLL(os.path.join(HERE, "_ref", _REF_LIBS[mode]))
        lib.ref_rx_stream.restype = C.c_int
        lib.ref_rx_stream.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.ref_rx_batch.restype = C.c_int
        lib.ref_rx_batch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.ref_layout_gap.restype = C.c_long
        lib.ref_log_set.argtypes = [C.c_void_p, C.c_size_t]
        lib.ref_poison_set.argtypes = [C.c_int, C.c_int, C.c_int]
        _ref[mode] = lib
    return _ref[mode]


def _frames(x):
    x = np.ascontiguousarray(x, dtype=np.int16)
    if x.ndim == 2:
        x = x[None]
    assert x.ndim == 3 and x.shape[2] == FRAME
    return x


def cpu_rx(x, threads: int = 0, trace: bool = False, mode: int = MODE_REF):
    """Restatement over x [nch][nframes][1880] (or [nframes][1880]).
    Returns bits [nch][nframes][62] u8, valid [nch][nframes] u8, trace|None."""
    x = _frames(x)
    nch, nf, _ = x.shape
    bits = np.zeros((nch, nf, NBITS), np.uint8)
    valid = np.zeros((nch, nf), np.uint8)
    tr = np.zeros((nch, nf), TRACE_DTYPE) if trace else None
    threads = threads or min(16, os.cpu_count() or 1)
    cpu_lib().qc_rx_batch_mode(_p(x), nch, nf, _p(bits), _p(valid), _p(tr), threads, mode)
    return bits, valid, tr


def ref_rx(x, trace: bool = False, log: bool = False, mode: int = MODE_REF):
    """The unmodified reference, one channel at a time (single thread)."""
    x = _frames(x)
    nch, nf, _ = x.shape
    lib = ref_lib(mode)
    bits = np.zeros((nch, nf, NBITS), np.uint8)
    valid = np.zeros((nch, nf), np.uint8)
    tr = np.zeros((nch, nf), REF_TRACE_DTYPE) if trace else None
    buf = C.create_string_buffer(1 << 20) if log else None
    if log:
        lib.ref_log_set(buf, len(buf))
    for c in range(nch):
        r = lib.ref_rx_stream(_p(x[c]), nf, _p(bits[c]), _p(valid[c]),
                              _p(tr[c]) if trace else None)
        if r < 0:
            raise RuntimeError("reference static layout is not the expected one")
    if log:
        lib.ref_log_set(None, 0)
    return (bits, valid, tr, buf.value.decode()) if log else (bits, valid, tr)


def ref_rx_poisoned(x, lo: int, hi: int, mode: int = MODE_REF):
    """ref_rx with the observability probe on: before each frame's equalizer
    the reference's decimated_frame[0..289] outside [mi + lo, mi + hi] is NaN
    (oracle/ref/ref_trace.c ref_poison_set)."""
    lib = ref_lib(mode)
    lib.ref_poison_set(1, lo, hi)
    try:
        return ref_rx(x, trace=True, mode=mode)
    finally:
        lib.ref_poison_set(0, 0, 0)


def ref_stages(x, mode: int = MODE_REF):
    """One channel through the reference, frame by frame, returning the
    reference's own buffers after each call: dec [nf][290][2] (decimated_frame
    [0..289]) and mixed [nf][1880][2] (input_frame[1880..3759])."""
    x = _frames(x)[0]
    nf = x.shape[0]
    lib = ref_lib(mode)
    lib.ref_rx_reset.restype = C.c_int
    lib.ref_rx_frame.restype = C.c_int
    lib.ref_rx_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.ref_peek_dec.argtypes = [C.c_void_p]
    lib.ref_peek_mixed.argtypes = [C.c_void_p]
    if lib.ref_rx_reset() != 0:
        raise RuntimeError("reference static layout is not the expected one")
    dec = np.zeros((nf, 290, 2), np.float32)
    mixed = np.zeros((nf, FRAME, 2), np.float32)
    bits = np.zeros((nf, NBITS), np.uint8)
    valid = np.zeros(nf, np.uint8)
    for n in range(nf):
        valid[n] = lib.ref_rx_frame(_p(x[n]), _p(bits[n]), None)
        lib.ref_peek_dec(_p(dec[n]))
        lib.ref_peek_mixed(_p(mixed[n]))
    return dec, mixed, bits, valid


def _tx_packets(init, frame, symbols):
    outs = []
    init()
    for sym, pre in symbols:
        s = np.ascontiguousarray(np.asarray(sym, np.complex64)).view(np.float32)
        out = np.zeros(5 * (s.size // 2), np.int16)
        n = frame(_p(out), _p(s), s.size // 2, int(pre))
        outs.append(out[:n])
    return outs


def cpu_tx(symbols):
    """TX restatement: symbols = [(complex array, is_preamble), ...] -> [int16 arrays]."""
    lib = cpu_lib()
    lib.qc_tx_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    st = C.create_string_buffer(49 * 8 + 8)
    return _tx_packets(lambda: lib.qc_tx_init(st),
                       lambda o, s, n, p: lib.qc_tx_frame(st, o, s, n, p), symbols)


def ref_tx(symbols):
    """The unmodified reference transmitter qpsk_tx_frame (src/qpsk.c:278)."""
    lib = ref_lib()
    lib.ref_tx_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    return _tx_packets(lib.ref_tx_reset, lib.ref_tx_frame, symbols)


def synth(seed: int, nch: int, nframes: int, ebn0_db: float = 1000.0, c0: int = 0,
          threads: int = 0) -> np.ndarray:
    """Synthetic channel streams [nch][nframes][1880] int16."""
    out = np.empty((nch, nframes, FRAME), np.int16)
    threads = threads or min(16, os.cpu_count() or 1)
    cpu_lib().qc_synth_batch(seed, c0, nch, float(ebn0_db), _p(out), nframes * FRAME, threads)
    return out


def mixer_table() -> np.ndarray:
    p = np.zeros((FRAME, 2), np.float32)
    cpu_lib().qc_mixer_table(_p(p))
    return p


def keystream(n: int) -> np.ndarray:
    ks = np.zeros(n, np.uint8)
    cpu_lib().qc_keystream(_p(ks), n)
    return ks


def preamble() -> np.ndarray:
    """The PN preamble p_i = +-1 (src/constants.c:25-42), read from the
    restatement's own table in cpu_ref.c (k_pre)."""
    import re
    src = open(os.path.join(HERE, "cpu_ref.c")).read()
    body = src[src.index("k_pre[QC_PRE] = {"):]
    body = body[body.index("{") + 1:body.index("}")]
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(vals) == 128 and set(vals) == {-1, 1}
    return np.asarray(vals, np.int8)


# ------------------------------------------------------------------- kiss_fft
def cpu_fft(x, inverse: bool = False) -> np.ndarray:
    """Restatement of the reference's fft() (src/fft.c) on a complex64 vector
    (or [batch][nfft])."""
    x = np.ascontiguousarray(x, dtype=np.complex64)
    out = np.empty_like(x)
    flat, fo = x.reshape(-1, x.shape[-1]), out.reshape(-1, x.shape[-1])
    for b in range(flat.shape[0]):
        r = cpu_lib().qc_fft(flat.shape[1], int(inverse), _p(flat[b]), _p(fo[b]))
        assert r == 0
    return out


def fft_twiddles(nfft: int, inverse: bool = False) -> np.ndarray:
    tw = np.empty(nfft, np.complex64)
    cpu_lib().qc_fft_twiddles(nfft, int(inverse), _p(tw))
    return tw


def ref_fft_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libkissfft_ref.so"))


_kfr = None


def ref_fft(x, inverse: bool = False) -> np.ndarray:
    """The reference's own kiss_fft (oracle/_ref/libkissfft_ref.so)."""
    global _kfr
    if _kfr is None:
        _kfr = C.CDLL(os.path.join(HERE, "_ref", "libkissfft_ref.so"))
        _kfr.ref_fft.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    x = np.ascontiguousarray(x, dtype=np.complex64)
    out = np.empty_like(x)
    flat, fo = x.reshape(-1, x.shape[-1]), out.reshape(-1, x.shape[-1])
    for b in range(flat.shape[0]):
        assert _kfr.ref_fft(flat.shape[1], int(inverse), _p(flat[b]), _p(fo[b])) == 0
    return out


def fft_hunt(dec) -> int:
    """qc_fft_hunt: max_index of the FFT-correlation hunt over dec[0..255]."""
    d = np.ascontiguousarray(np.asarray(dec, np.complex64)[:256])
    return int(cpu_lib().qc_fft_hunt(_p(d)))


def fft_hunt_spectrum() -> np.ndarray:
    q = np.empty(256, np.complex64)
    cpu_lib().qc_fft_hunt_spectrum(_p(q))
    return q


def cpu_stages(x, mode: int = MODE_REF) -> np.ndarray:
    """decimated_frame[0..289] after each call, one channel x [nframes][1880]."""
    x = np.ascontiguousarray(x, dtype=np.int16).reshape(-1, FRAME)
    dec = np.zeros((x.shape[0], 290, 2), np.float32)
    cpu_lib().qc_rx_stages(_p(x), x.shape[0], mode, _p(dec))
    return dec
