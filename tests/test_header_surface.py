"""The drop-in header (include/qpsk_internal.h) against a caller of the
reference's header surface (Missing #2).

tests/callers/ref_caller.c includes only qpsk_internal.h and uses the
reference header's macros, RXState, C99 `complex float` and cmplx() as the
reference driver does (src/qpsk.c:346-461).  It must compile unchanged against
the repo header and link libqpsk_hip.so; every macro must have the reference
header's value and type (/root/reference/headers/qpsk_internal.h:23-75, when
the reference is present: CPU tests only); the host TX path must reproduce the
reference TX golden; on the GPU its RX loop must reproduce the reference output
file of preamble_qpsk_8k.raw."""
import hashlib
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import singlecarrier_amd as sc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLER = os.path.join(ROOT, "tests", "callers", "ref_caller.c")
REF_HEADERS = "/root/reference/headers"


def _build(tmp_path, include, extra=()):
    exe = str(tmp_path / ("ref_caller" + ("_c" if extra else "")))
    cmd = ["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-I", include, CALLER, "-o", exe, *extra]
    if not extra:
        libdir = os.path.dirname(sc.LIB_PATH)
        cmd += [sc.LIB_PATH, f"-Wl,-rpath,{libdir}"]   # QPSK_LIB: any file name
    cmd += ["-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    if not os.path.exists(sc.LIB_PATH):
        sc.build()
    return _build(tmp_path_factory.mktemp("caller"), os.path.join(ROOT, "include"))


def test_caller_compiles_unchanged_and_links(caller):
    r = subprocess.run([caller, "consts"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = dict(line.split(" ", 1) for line in r.stdout.splitlines())
    assert out["CYCLES"] == "5 sizeof 4" and out["FRAME_SIZE"] == "1880"
    assert out["TX_FILENAME"] == "/tmp/spectrum-filtered.raw"
    assert out["RXState"] == "0 1 4"


@pytest.mark.skipif(not os.path.isdir(REF_HEADERS), reason="reference not present")
def test_every_macro_equals_the_reference_header(caller, tmp_path):
    """Same values and expression types, printed by the same code compiled
    against each header (the reference build needs no library: consts only)."""
    ref = _build(tmp_path, REF_HEADERS, extra=("-DCONSTS_ONLY",))
    a = subprocess.run([caller, "consts"], capture_output=True, text=True, check=True).stdout
    b = subprocess.run([ref, "consts"], capture_output=True, text=True, check=True).stdout
    assert a == b


def test_header_is_cplusplus_clean(tmp_path):
    """A C++ caller sees the same prototypes with C linkage."""
    src = tmp_path / "cxx.cc"
    src.write_text('#include "qpsk_internal.h"\n'
                   "int main() { float _Complex z = 0; return (int)cnormf(z) + FRAME_SIZE - 1880 + hunt; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I",
                        os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_caller_tx_matches_reference_golden(caller, tmp_path, golden_dir):
    """qpsk_tx_frame called from C with complex float symbols == the TX golden
    the reference made (src/qpsk.c:278-322)."""
    g = np.load(os.path.join(golden_dir, "tx_golden.npz"))
    syms = np.split(g["symbols"], np.cumsum(g["lengths"])[:-1])
    blob = bytearray(struct.pack("<i", len(syms)))
    for s, p in zip(syms, g["preamble"]):
        blob += struct.pack("<ii", len(s), int(p))
        blob += np.stack([s.real, s.imag], axis=1).astype("<f4").tobytes()
    (tmp_path / "syms.bin").write_bytes(bytes(blob))
    subprocess.run([caller, "tx", str(tmp_path / "syms.bin"), str(tmp_path / "tx.raw")], check=True)
    got = np.fromfile(tmp_path / "tx.raw", dtype="<i2")
    np.testing.assert_array_equal(got, g["samples"])


@pytest.mark.gpu
def test_caller_rx_reproduces_reference_output_file(caller, tmp_path, golden_dir):
    """The reference RX loop in the caller, per-frame qpsk_rx_frame on the GPU,
    writes the reference's output file for the sample capture (md5 b56a4d36...)."""
    exp = json.load(open(os.path.join(golden_dir, "sample_expected.json")))
    out = tmp_path / "databits.bin"
    r = subprocess.run([caller, "rx", os.path.join(golden_dir, "preamble_qpsk_8k.raw"), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert hashlib.md5(out.read_bytes()).hexdigest() == exp["output_md5"]
