"""singlecarrier_amd -- MI355X receive path of the SingleCarrier QPSK modem.

Python mirror of the C-ABI in ``include/qpsk_internal.h`` (the reference's
``headers/qpsk_internal.h:79-84`` surface) and ``include/qpsk_batch.h`` (the
batched, multi-channel receiver), over ``singlecarrier_amd/libqpsk_hip.so``.

There is no CPU fallback: if the HIP library is missing or no GPU is present,
the receive functions raise.  (The CPU restatement in ``oracle/`` is test
infrastructure, never called from here.)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# QPSK_LIB overrides the library path (A/B experiments with variant builds only)
LIB_PATH = os.environ.get("QPSK_LIB") or os.path.join(HERE, "libqpsk_hip.so")

FRAME_SIZE = 1880        # headers/qpsk_internal.h:45
DATA_SYMBOLS = 31        # headers/qpsk_internal.h:37
PREAMBLE_LENGTH = 128    # headers/qpsk_internal.h:50
BITS_PER_FRAME = 496     # headers/qpsk_internal.h:48 (record size of the RX driver)
NBITS = 62               # bits written per valid frame (src/qpsk.c:206-215)
CYCLES = 5

_lib = None


class _CF(C.Structure):
    _fields_ = [("re", C.c_float), ("im", C.c_float)]


class QpskError(RuntimeError):
    """A negative QPSK_E* code from the library (``.code``)."""
    code = 0


# error codes (include/qpsk_batch.h, qpsk_stream.h)
QPSK_EINVAL, QPSK_ENOMEM, QPSK_ENODEV, QPSK_EBUSY, QPSK_ESTALL = -1, -2, -3, -4, -5


def build(verbose: bool = False) -> str:
    """Compile libqpsk_hip.so for gfx950 (hipcc cross-compiles without a GPU)."""
    out = subprocess.run(["make", "-C", os.path.join(HERE, "csrc")], capture_output=True,
                         text=True)
    if out.returncode != 0:
        raise QpskError("build failed:\n" + out.stdout[-4000:] + out.stderr[-4000:])
    if verbose:
        print(out.stdout)
    return LIB_PATH


# the receive kernels' sources and build rules, in the order the Makefile's KSRC
# hashes them (csrc/Makefile: qpsk_kernel_hash())
KERNEL_SOURCES = ("qpsk_rx.hip", "qpsk_hunt.h", "qpsk_rcp.h", "qpsk_consts.h", "qpsk_fft_dev.h",
                  "qpsk_fft_tables.h", "qpsk_rx_internal.h", "qpsk_split.h", "Makefile")


def kernel_source_hash(csrc: str = None) -> str:
    """The hash the Makefile compiles into the library (KERNEL_SOURCES, the
    C-ABI headers they include, the compile flags and the compiler's version),
    for the sources in `csrc` (default: this package's csrc/).  The Makefile is
    the one definition: this asks it (make khash)."""
    csrc = csrc or os.path.join(HERE, "csrc")
    inc = os.path.join(os.path.dirname(HERE), "include")
    out = subprocess.run(["make", "-s", "--no-print-directory", "-C", csrc, "khash", f"INCDIR={inc}"],
                         capture_output=True, text=True)
    if out.returncode != 0:
        raise QpskError("make khash failed:\n" + out.stderr[-2000:])
    return out.stdout.strip()


def kernel_hash() -> str:
    """qpsk_kernel_hash() of the loaded library (no GPU needed)."""
    return lib().qpsk_kernel_hash().decode()


def lib():
    """Load the HIP library (fails loudly when it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QpskError(f"{LIB_PATH} not built: run singlecarrier_amd.build() "
                            "or make -C singlecarrier_amd/csrc")
        try:  # share torch's HIP runtime when torch is in use (same soname)
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        vp, i32, u64 = C.c_void_p, C.c_int, C.c_uint64
        L.qpsk_rx_create.restype = vp
        L.qpsk_rx_create.argtypes = [i32, i32, C.POINTER(C.c_int)]
        L.qpsk_rx_create_mode.restype = vp
        L.qpsk_rx_create_mode.argtypes = [i32, i32, i32, C.POINTER(C.c_int)]
        L.qpsk_rx_mode.argtypes = [vp]
        L.qpsk_rx_destroy.argtypes = [vp]
        L.qpsk_rx_reset.argtypes = [vp]
        L.qpsk_rx_channels.argtypes = [vp]
        L.qpsk_rx_frames.restype = u64
        L.qpsk_rx_frames.argtypes = [vp]
        L.qpsk_rx_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.qpsk_rx_batch_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
        L.qpsk_strerror.restype = C.c_char_p
        L.qpsk_strerror.argtypes = [i32]
        L.qpsk_kernel_hash.restype = C.c_char_p
        L.qpsk_kernel_hash.argtypes = []
        L.qpsk_rx_frame.argtypes = [vp, vp]
        L.qpsk_tx_frame.argtypes = [vp, vp, i32, C.c_bool]
        L.qpsk_surface_error.restype = i32
        L.qpsk_rx_timing_enable.argtypes = [vp, i32]
        L.qpsk_rx_sync.argtypes = [vp]
        L.qpsk_rx_timing_collect.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.qpsk_rx_timing_split.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                           C.POINTER(C.c_int)]
        L.qpsk_synth_batch.restype = None
        L.qpsk_synth_batch.argtypes = [u64, C.c_uint32, i32, C.c_double, vp, C.c_long, i32]
        L.qpsk_synth_device.argtypes = [u64, C.c_uint32, i32, C.c_double, vp, C.c_long, vp]
        L.qpsk_tx_phase_table.restype = None
        L.qpsk_tx_phase_table.argtypes = [vp, C.c_long]
        L.qpsk_stream_create.restype = vp
        L.qpsk_stream_create.argtypes = [i32, i32, i32, i32, C.POINTER(C.c_int)]
        L.qpsk_stream_create_mode.restype = vp
        L.qpsk_stream_create_mode.argtypes = [i32, i32, i32, i32, i32, C.POINTER(C.c_int)]
        L.qpsk_stream_destroy.argtypes = [vp]
        L.qpsk_stream_acquire.restype = vp
        L.qpsk_stream_acquire.argtypes = [vp, C.POINTER(C.c_int)]
        L.qpsk_stream_submit.argtypes = [vp]
        L.qpsk_stream_pending.argtypes = [vp]
        L.qpsk_stream_retrieve.argtypes = [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.qpsk_stream_ctx.restype = vp
        L.qpsk_stream_ctx.argtypes = [vp]
        L.qpsk_records.restype = C.c_size_t
        L.qpsk_records.argtypes = [vp, vp, i32, vp]
        L.qpsk_fft_alloc.restype = vp
        L.qpsk_fft_alloc.argtypes = [i32, i32, i32, C.POINTER(C.c_int)]
        L.qpsk_fft_free.argtypes = [vp]
        L.qpsk_fft_device.argtypes = [vp, vp, vp, i32, vp]
        L.qpsk_fft.argtypes = [vp, vp, vp, i32]
        L.qpsk_fft_twiddle_table.restype = None
        L.qpsk_fft_twiddle_table.argtypes = [i32, i32, vp]
        L.qpsk_fft_perm_table.argtypes = [i32, vp]
        L.qpsk_rx_state_size.restype = C.c_size_t
        L.qpsk_rx_state_size.argtypes = [i32]
        L.qpsk_rx_state_save.argtypes = [vp, i32, i32, vp, C.c_size_t]
        L.qpsk_rx_state_load.argtypes = [vp, i32, i32, vp, C.c_size_t]
        L.cnormf.restype = C.c_float
        L.cnormf.argtypes = [_CF]   # _Complex float == {float, float} in one SSE reg (SysV)
        _lib = L
    return _lib


SYMBOLS = ["qpsk_rx_create", "qpsk_rx_create_mode", "qpsk_rx_mode", "qpsk_rx_destroy", "qpsk_rx_reset", "qpsk_rx_channels",
           "qpsk_rx_frames", "qpsk_rx_batch", "qpsk_rx_batch_device", "qpsk_rx_sync", "qpsk_strerror",
           "qpsk_kernel_hash",
           "cnormf", "qpsk_mod", "qpsk_demod", "qpsk_rx_frame", "qpsk_tx_frame",
           "qpsk_rx_init", "qpsk_tx_init", "qpsk_surface_error", "qpsk_tx_state_init",
           "qpsk_tx_frame_state", "qpsk_synth_batch", "qpsk_rx_timing_enable",
           "qpsk_rx_timing_collect", "qpsk_rx_timing_split", "qpsk_synth_device",
           "qpsk_tx_phase_table", "qpsk_stream_create", "qpsk_stream_create_mode", "qpsk_stream_destroy",
           "qpsk_stream_acquire", "qpsk_stream_submit", "qpsk_stream_pending",
           "qpsk_stream_retrieve", "qpsk_stream_ctx", "qpsk_records", "qpsk_fft_alloc",
           "qpsk_fft_free", "qpsk_fft_device", "qpsk_fft", "qpsk_rx_state_size",
           "qpsk_rx_state_save", "qpsk_rx_state_load"]


def _check(rc: int) -> None:
    if rc != 0:
        e = QpskError(f"qpsk error {rc}: {lib().qpsk_strerror(rc).decode()}")
        e.code = rc
        raise e


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor (device memory)


# receiver semantics (include/qpsk_batch.h QPSK_MODE_*)
MODE_REFERENCE = 0   # bit-identical to the reference as built
MODE_DEC752 = 1      # decimated_frame[752] ("intended semantics"), NOT reference parity
MODE_FFT_HUNT = 2    # flag: preamble hunt through the reference's kiss_fft (src/fft.c)


class Receiver:
    """A batch of ``nch`` independent receivers on one GPU (``qpsk_ctx``).

    Each channel behaves like the reference receiver fed that channel's stream
    from a fresh start (src/qpsk.c:427-458); state persists across calls.
    ``mode`` selects the receiver semantics (MODE_REFERENCE or MODE_DEC752).
    """

    def __init__(self, nch: int, device: int = 0, mode: int = MODE_REFERENCE):
        err = C.c_int(0)
        self._h = lib().qpsk_rx_create_mode(device, nch, mode, C.byref(err))
        if not self._h:
            _check(err.value or -3)
        self.nch = nch
        self.device = device
        self.mode = int(lib().qpsk_rx_mode(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().qpsk_rx_destroy(self._h)
            self._h = None

    __del__ = close

    def reset(self) -> None:
        _check(lib().qpsk_rx_reset(self._h))

    @property
    def frames(self) -> int:
        return int(lib().qpsk_rx_frames(self._h))

    def state_save(self, c0: int = 0, n: int | None = None) -> bytes:
        """Snapshot of channels [c0, c0 + n) (qpsk_rx_state_save): the carried
        per-channel state and the frame index, as bytes."""
        n = self.nch - c0 if n is None else n
        buf = np.zeros(int(lib().qpsk_rx_state_size(n)), np.uint8)
        _check(lib().qpsk_rx_state_save(self._h, c0, n, _ptr(buf), buf.size))
        return buf.tobytes()

    def state_load(self, snap: bytes, c0: int = 0, n: int | None = None) -> None:
        """Load a snapshot of n channels into channels [c0, c0 + n)
        (qpsk_rx_state_load)."""
        buf = np.frombuffer(snap, np.uint8)
        if len(snap) < 64 or bytes(snap[:8]) != b"QPSKSTA1":   # StateHdr: 64 bytes, magic first
            _check(QPSK_EINVAL)
        if n is None:
            n = int(np.frombuffer(snap[20:24], np.int32)[0])   # StateHdr.n
        _check(lib().qpsk_rx_state_load(self._h, c0, n, _ptr(buf), buf.size))

    def timing(self, on: bool = True) -> None:
        """Enable per-call step-kernel span events (see qpsk_rx_timing_collect)."""
        _check(lib().qpsk_rx_timing_enable(self._h, int(on)))

    def collect_timing(self):
        """(summed kernel span in ms, frames) since the last collect."""
        ms, n = C.c_float(0), C.c_int(0)
        _check(lib().qpsk_rx_timing_collect(self._h, C.byref(ms), C.byref(n)))
        return float(ms.value), int(n.value)

    def collect_timing_split(self):
        """(rx_kernel ms, rx_data_kernel ms, frames) since the last collect."""
        a, b, n = C.c_float(0), C.c_float(0), C.c_int(0)
        _check(lib().qpsk_rx_timing_split(self._h, C.byref(a), C.byref(b), C.byref(n)))
        return float(a.value), float(b.value), int(n.value)

    def demod(self, x, trace: bool = False, soft: bool = False):
        """Host arrays: x int16 [nch][nframes][1880] -> dict of numpy arrays
        bits [nch][nframes][62], valid [nch][nframes] (+ trace [..][4], soft [..][31][2])."""
        x = np.ascontiguousarray(x, dtype=np.int16)
        if x.ndim != 3 or x.shape[0] != self.nch or x.shape[2] != FRAME_SIZE:
            raise ValueError(f"expected int16 [{self.nch}][nframes][{FRAME_SIZE}], got {x.shape}")
        nf = x.shape[1]
        out = {"bits": np.zeros((self.nch, nf, NBITS), np.uint8),
               "valid": np.zeros((self.nch, nf), np.uint8)}
        if trace:
            out["trace"] = np.zeros((self.nch, nf, 4), np.int32)
        if soft:
            out["soft"] = np.zeros((self.nch, nf, DATA_SYMBOLS, 2), np.float32)
        _check(lib().qpsk_rx_batch(self._h, _ptr(x), nf, _ptr(out["bits"]), _ptr(out["valid"]),
                                   _ptr(out.get("trace")), _ptr(out.get("soft"))))
        return out

    def sync(self) -> None:
        """Wait for the latest demod_device call; raise QpskError (QPSK_ESTALL)
        if any call since the previous check failed on the device."""
        _check(lib().qpsk_rx_sync(self._h))

    def demod_device(self, x, bits, valid, trace=None, soft=None, stream=None) -> None:
        """Device tensors (torch, on this device): enqueue on ``stream``
        (default: torch's current stream) and return without synchronising."""
        import torch
        if x.dtype != torch.int16 or x.dim() != 3 or x.shape[0] != self.nch \
                or x.shape[2] != FRAME_SIZE or not x.is_contiguous() or not x.is_cuda:
            raise ValueError("x must be a contiguous cuda int16 [nch][nframes][1880] tensor")
        nf = x.shape[1]
        for name, t, shape in (("bits", bits, (self.nch, nf, NBITS)),
                               ("valid", valid, (self.nch, nf)),
                               ("trace", trace, (self.nch, nf, 4)),
                               ("soft", soft, (self.nch, nf, DATA_SYMBOLS, 2))):
            if t is not None and (tuple(t.shape) != shape or not t.is_contiguous() or not t.is_cuda):
                raise ValueError(f"{name} must be a contiguous cuda tensor of shape {shape}")
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        _check(lib().qpsk_rx_batch_device(self._h, _ptr(x), nf, _ptr(bits), _ptr(valid),
                                          _ptr(trace), _ptr(soft), C.c_void_p(stream.cuda_stream)))


# --- the reference's single-channel surface (headers/qpsk_internal.h:79-84) ---

class Stream:
    """Streaming ingest over pinned chunk slots (include/qpsk_stream.h): fill
    ``acquire()`` in place, ``submit()``, later ``retrieve()`` the oldest chunk.
    Every channel's state carries across chunks."""

    def __init__(self, nch: int, frames: int, nslot: int = 3, device: int = 0,
                 mode: int = MODE_REFERENCE):
        err = C.c_int(0)
        self._h = lib().qpsk_stream_create_mode(device, nch, frames, nslot, mode, C.byref(err))
        if not self._h:
            _check(err.value or -3)
        self.nch, self.frames, self.nslot = nch, frames, nslot

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().qpsk_stream_destroy(self._h)
            self._h = None

    __del__ = close

    def acquire(self) -> np.ndarray:
        """The next chunk's pinned input buffer as int16 [nch][frames][1880]."""
        err = C.c_int(0)
        p = lib().qpsk_stream_acquire(self._h, C.byref(err))
        if not p:
            _check(err.value or -1)
        n = self.nch * self.frames * FRAME_SIZE
        buf = (C.c_int16 * n).from_address(p)
        return np.frombuffer(buf, np.int16).reshape(self.nch, self.frames, FRAME_SIZE)

    def submit(self) -> None:
        _check(lib().qpsk_stream_submit(self._h))

    @property
    def pending(self) -> int:
        return int(lib().qpsk_stream_pending(self._h))

    def retrieve(self, copy: bool = True):
        """(bits [nch][frames][62], valid [nch][frames]) of the oldest chunk."""
        b, v = C.c_void_p(), C.c_void_p()
        _check(lib().qpsk_stream_retrieve(self._h, C.byref(b), C.byref(v)))
        cf = self.nch * self.frames
        bits = np.frombuffer((C.c_uint8 * (cf * NBITS)).from_address(b.value), np.uint8)
        valid = np.frombuffer((C.c_uint8 * cf).from_address(v.value), np.uint8)
        bits = bits.reshape(self.nch, self.frames, NBITS)
        valid = valid.reshape(self.nch, self.frames)
        return (bits.copy(), valid.copy()) if copy else (bits, valid)


def cnormf(val: complex) -> float:
    """|val|^2 as the reference computes it (src/qpsk.c:75-80)."""
    return float(lib().cnormf(_CF(val.real, val.imag)))


def qpsk_mod(bits, index: int) -> complex:
    """Gray map: I = bits[index+1], Q = bits[index] (src/qpsk.c:251-256)."""
    i = -1.0 if bits[index + 1] == 1 else 1.0
    q = -1.0 if bits[index] == 1 else 1.0
    return complex(i, q)


def qpsk_demod(symbol: complex) -> list:
    """[Q, I] hard decisions, bits[1] = Re<0, bits[0] = Im<0 (src/qpsk.c:268-271)."""
    return [int(np.float32(symbol.imag) < 0), int(np.float32(symbol.real) < 0)]


def qpsk_rx_init() -> None:
    lib().qpsk_rx_init()
    _check(lib().qpsk_surface_error())


def qpsk_rx_frame(frame, bits=None):
    """One 1880-sample frame through the one-channel GPU receiver (src/qpsk.c:133).
    Returns 1 and fills bits[0..61] on a valid frame, else 0."""
    fr = np.ascontiguousarray(frame, dtype=np.int16)
    if fr.shape != (FRAME_SIZE,):
        raise ValueError("frame must be 1880 int16 samples")
    b = np.zeros(NBITS, np.uint8)
    v = lib().qpsk_rx_frame(_ptr(fr), _ptr(b))
    _check(lib().qpsk_surface_error())
    if v and bits is not None:
        bits[:NBITS] = b
    return v, b


def qpsk_tx_init() -> None:
    lib().qpsk_tx_init()


def qpsk_tx_frame(symbols, preamble: bool) -> np.ndarray:
    """Host TX of the reference (src/qpsk.c:278-322): len(symbols) complex
    symbols -> 5*len int16 samples."""
    s = np.ascontiguousarray(np.asarray(symbols, np.complex64))
    out = np.zeros(s.size * CYCLES, np.int16)
    n = lib().qpsk_tx_frame(_ptr(out), _ptr(s), s.size, bool(preamble))
    return out[:n]


def synth(seed: int, nch: int, nframes: int, ebn0_db: float = 1000.0, c0: int = 0,
          threads: int = 0) -> np.ndarray:
    """Synthetic channel streams int16 [nch][nframes][1880] (include/qpsk_synth.h)."""
    out = np.empty((nch, nframes, FRAME_SIZE), np.int16)
    threads = threads or min(16, os.cpu_count() or 1)
    lib().qpsk_synth_batch(seed, c0, nch, float(ebn0_db), _ptr(out), nframes * FRAME_SIZE,
                           threads)
    return out


def synth_device(seed: int, nch: int, nframes: int, ebn0_db: float = 1000.0, c0: int = 0,
                 device: int | None = None, out=None):
    """The same streams as synth(), generated on the GPU: a torch int16 tensor
    [nch][nframes][1880] on `device` (qpsk_synth_device)."""
    import torch
    if out is None:
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        out = torch.empty((nch, nframes, FRAME_SIZE), dtype=torch.int16, device=dev)
    with torch.cuda.device(out.device):
        stream = torch.cuda.current_stream().cuda_stream
        _check(lib().qpsk_synth_device(seed, c0, nch, float(ebn0_db), out.data_ptr(),
                                       nframes * FRAME_SIZE, stream))
    return out


def tx_phase_table(ntx: int) -> np.ndarray:
    """Carrier phase of the first ntx transmitted samples, float32 [ntx][2]."""
    out = np.empty((ntx, 2), np.float32)
    lib().qpsk_tx_phase_table(_ptr(out), ntx)
    return out


def read_raw(path: str) -> np.ndarray:
    """A reference .raw capture as frames [nframes][1880]; the short tail is
    dropped like the reference driver (src/qpsk.c:442-445)."""
    raw = np.fromfile(path, np.int16)
    nf = raw.size // FRAME_SIZE
    return raw[: nf * FRAME_SIZE].reshape(nf, FRAME_SIZE)


def records(bits: np.ndarray, valid: np.ndarray) -> bytes:
    """The reference driver's output file (src/qpsk.c:455-457): one 496-byte
    record per valid frame, bits in bytes 0..61, the rest zero (qpsk_records,
    host code)."""
    bits = np.ascontiguousarray(bits, np.uint8)
    valid = np.ascontiguousarray(valid, np.uint8)
    nf = valid.shape[0]
    out = np.empty(max(nf, 1) * BITS_PER_FRAME, np.uint8)
    n = lib().qpsk_records(_ptr(bits), _ptr(valid), nf, _ptr(out))
    return out[:n].tobytes()


class FftPlan:
    """The reference's kiss_fft on the GPU (include/qpsk_fft.h): fft_alloc(nfft,
    inverse) + batched fft(), bit-identical to src/fft.c.  nfft: a power of two
    in [4, 4096]."""

    def __init__(self, nfft: int, inverse: bool = False, device: int = 0):
        err = C.c_int(0)
        self._h = lib().qpsk_fft_alloc(device, nfft, int(inverse), C.byref(err))
        if not self._h:
            _check(err.value or -3)
        self.nfft, self.inverse, self.device = nfft, bool(inverse), device

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().qpsk_fft_free(self._h)
            self._h = None

    __del__ = close

    def __call__(self, x) -> np.ndarray:
        """complex64 [..., nfft] host array -> its transform (host)."""
        x = np.ascontiguousarray(x, dtype=np.complex64)
        if x.shape[-1] != self.nfft:
            raise ValueError(f"last axis must be {self.nfft}")
        out = np.empty_like(x)
        _check(lib().qpsk_fft(self._h, _ptr(x), _ptr(out), x.size // self.nfft))
        return out

    def run_device(self, x, out=None, stream=None):
        """torch complex64 (or float32 [..., nfft, 2]) cuda tensors; enqueued."""
        import torch
        if out is None:
            out = torch.empty_like(x)
        n = x.numel() // (self.nfft * (1 if x.is_complex() else 2))
        s = stream if stream is not None else torch.cuda.current_stream(x.device)
        _check(lib().qpsk_fft_device(self._h, x.data_ptr(), out.data_ptr(), n, s.cuda_stream))
        return out


def fft_twiddle_table(nfft: int, inverse: bool = False) -> np.ndarray:
    """The product's host twiddle table (qpsk_fft_host.c), for tests."""
    tw = np.empty(nfft, np.complex64)
    lib().qpsk_fft_twiddle_table(nfft, int(inverse), _ptr(tw))
    return tw
