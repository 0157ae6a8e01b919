"""Contexts driven from several host threads at once (run with -m gpu).

SURVEY.md 8b asks the C-ABI to be thread-safe across contexts.  The reference
receiver is not reentrant (file-scope statics, /root/reference/src/qpsk.c:34-53),
so this is a property of the build alone and is shown here: four host threads
each create their own context at the same moment (behind a barrier: the
receiver's constant tables are built once, under C++11 static initialisation)
and demodulate a different seeded batch -- different channel counts, so
different kernel shapes, and one dec752 context -- over several calls.  Every
output must equal the oracle's for that batch, bit for bit.

The same from C with pthreads: tests/callers/threads_caller.c.  Threads use
device t % N when N > 1 GPUs are visible, else all share device 0.
"""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (seed, channels, frames, Eb/N0, mode): quad backs at W = 16 (<= 4,096) and
# W = 32 (4,097..8,192), lane backs at W = 64 (8,193..16,384)
JOBS = [(81, 300, 9, 6.0, sc.MODE_REFERENCE),
        (82, 130, 9, 1000.0, sc.MODE_DEC752),
        (83, 4500, 6, 8.0, sc.MODE_REFERENCE),
        (84, 9000, 6, 4.0, sc.MODE_REFERENCE)]


def _devices():
    import torch
    return max(1, torch.cuda.device_count())


def _inputs():
    return [oracle.synth(s, n, f, e) for s, n, f, e, _ in JOBS]


def test_contexts_from_four_host_threads():
    sc.lib()                        # load the library before the threads start
    ndev = _devices()
    xs = _inputs()
    start = threading.Barrier(len(JOBS))
    outs, errs = [None] * len(JOBS), [None] * len(JOBS)

    def work(t):
        try:
            x = xs[t]
            start.wait()
            rx = sc.Receiver(x.shape[0], device=t % ndev, mode=JOBS[t][4])
            nf = x.shape[1]
            parts = []
            for a, b in ((0, 2), (2, 3), (3, nf)):
                parts.append(rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True))
            assert rx.frames == nf
            rx.close()
            outs[t] = {k: np.concatenate([p[k] for p in parts], axis=1) for k in parts[0]}
        except BaseException as e:   # re-raised in the main thread
            errs[t] = e

    th = [threading.Thread(target=work, args=(t,)) for t in range(len(JOBS))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for t in range(len(JOBS)):
        if errs[t] is not None:
            raise errs[t]
        assert outs[t] is not None, f"thread {t} did not finish"
    for t, x in enumerate(xs):
        bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=JOBS[t][4])
        o = outs[t]
        np.testing.assert_array_equal(o["valid"], valid, err_msg=f"thread {t}")
        np.testing.assert_array_equal(o["bits"], bits, err_msg=f"thread {t}")
        np.testing.assert_array_equal(o["trace"][..., 0], tr["max_index"])
        np.testing.assert_array_equal(o["trace"][..., 3], tr["rx_timing"])
        vm = valid.astype(bool)
        np.testing.assert_array_equal(o["soft"][vm], tr["soft"][vm])
        assert 0 < valid.sum() < valid.size


def test_contexts_from_four_pthreads(tmp_path):
    """tests/callers/threads_caller.c: the same from C, one pthread per context."""
    exe = str(tmp_path / "threads_caller")
    libdir = os.path.dirname(sc.LIB_PATH)
    r = subprocess.run(["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "callers", "threads_caller.c"), "-o", exe,
                        sc.LIB_PATH, f"-Wl,-rpath,{libdir}", "-lpthread"],   # QPSK_LIB: any file name
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    xs = _inputs()
    args = [exe, str(_devices())]
    for t, (x, job) in enumerate(zip(xs, JOBS)):
        x.tofile(tmp_path / f"in{t}.raw")
        args += [str(tmp_path / f"in{t}.raw"), str(x.shape[0]), str(x.shape[1]), str(job[4]),
                 str(tmp_path / f"out{t}.bin")]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for t, x in enumerate(xs):
        bits, valid, _ = oracle.cpu_rx(x, mode=JOBS[t][4])
        got = np.fromfile(tmp_path / f"out{t}.bin", np.uint8)
        nb = bits.size
        np.testing.assert_array_equal(got[:nb].reshape(bits.shape), bits, err_msg=f"thread {t}")
        np.testing.assert_array_equal(got[nb:].reshape(valid.shape), valid, err_msg=f"thread {t}")


def test_streams_from_three_host_threads():
    """qpsk_stream objects (each owning its context, pinned slots and three HIP
    streams) fed from three host threads at once: every chunk sequence equals
    the oracle over the concatenated frames."""
    sc.lib()
    ndev = _devices()
    jobs = [(91, 150, 4, 5, 7.0, 3), (92, 700, 2, 6, 3.0, 2), (93, 4200, 3, 4, 9.0, 3)]
    xs = [oracle.synth(s, n, f * k, e) for s, n, f, k, e, _ in jobs]
    start = threading.Barrier(len(jobs))
    outs, errs = [None] * len(jobs), [None] * len(jobs)

    def work(t):
        try:
            _, nch, fpc, nchunk, _, nslot = jobs[t]
            x = xs[t]
            start.wait()
            st = sc.Stream(nch, fpc, nslot=nslot, device=t % ndev)
            gb, gv = [], []
            for k in range(nchunk):
                st.acquire()[...] = x[:, k * fpc:(k + 1) * fpc]
                st.submit()
                if st.pending == nslot:
                    b, v = st.retrieve()
                    gb.append(b)
                    gv.append(v)
            while st.pending:
                b, v = st.retrieve()
                gb.append(b)
                gv.append(v)
            st.close()
            outs[t] = (np.concatenate(gb, axis=1), np.concatenate(gv, axis=1))
        except BaseException as e:
            errs[t] = e

    th = [threading.Thread(target=work, args=(t,)) for t in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for t in range(len(jobs)):
        if errs[t] is not None:
            raise errs[t]
        bits, valid, _ = oracle.cpu_rx(xs[t])
        np.testing.assert_array_equal(outs[t][1], valid, err_msg=f"thread {t}")
        np.testing.assert_array_equal(outs[t][0], bits, err_msg=f"thread {t}")
        assert valid.any()


def test_pthreads_under_threadsanitizer(tmp_path):
    """The same four-pthread run with the library's host code and the caller
    built with ThreadSanitizer (tests/callers/Makefile `tsan`, ROCm clang; the
    device code is the product's): no data race is reported, and the outputs
    still equal the oracle's.  Prebuilt in the build container (skipped when
    absent)."""
    exe = os.path.join(ROOT, "tests", "callers", "build", "threads_caller_tsan")
    if not os.path.exists(exe):
        pytest.skip("make -C tests/callers tsan")
    xs = _inputs()
    args = [exe, str(_devices())]
    for t, (x, job) in enumerate(zip(xs, JOBS)):
        x.tofile(tmp_path / f"in{t}.raw")
        args += [str(tmp_path / f"in{t}.raw"), str(x.shape[0]), str(x.shape[1]), str(job[4]),
                 str(tmp_path / f"out{t}.bin")]
    supp = os.path.join(ROOT, "tests", "callers", "tsan.supp")   # the uninstrumented ROCm runtime
    env = dict(os.environ, TSAN_OPTIONS=f"halt_on_error=1:exitcode=66:report_signal_unsafe=0:suppressions={supp}")
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, r.stderr[-3000:]
    for t, x in enumerate(xs):
        bits, valid, _ = oracle.cpu_rx(x, mode=JOBS[t][4])
        got = np.fromfile(tmp_path / f"out{t}.bin", np.uint8)
        np.testing.assert_array_equal(got[:bits.size].reshape(bits.shape), bits, err_msg=f"thread {t}")
        np.testing.assert_array_equal(got[bits.size:].reshape(valid.shape), valid, err_msg=f"thread {t}")
