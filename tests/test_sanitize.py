"""ASan + UBSan build of the host C on the path: the
oracle restatement oracle/cpu_ref.c, the host generator csrc/qpsk_synth.c,
the reference surface csrc/qpsk_surface.c and the record writer
csrc/qpsk_records.c, driven by tests/sanitize/san_harness.c.  The sanitized
binary must run clean (any report aborts it: -fno-sanitize-recover=all) and
produce exactly what the unsanitized builds produce.  CPU only.

The unmodified reference (oracle/_ref) is never built with -fsanitize: its
answer depends on its static layout."""
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
import singlecarrier_amd as sc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "singlecarrier_amd", "csrc")
SAN = ["-fsanitize=address,undefined,float-cast-overflow", "-fno-sanitize-recover=all",
       "-fno-omit-frame-pointer"]
# the same IEEE contract as the product and oracle builds
FP = ["-std=gnu11", "-O1", "-g", "-ffp-contract=off", "-fno-fast-math"]

TRACE = np.dtype([("max_index", "<i4"), ("matches", "<i4"), ("valid", "<i4"),
                  ("rx_timing", "<i4"), ("soft", "<f4", (31, 2))])


@pytest.fixture(scope="module")
def san_out(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    d = tmp_path_factory.mktemp("san")
    exe = str(d / "san_harness")
    srcs = [os.path.join(ROOT, "tests", "sanitize", "san_harness.c"),
            os.path.join(ROOT, "oracle", "cpu_ref.c"), os.path.join(CSRC, "qpsk_synth.c"),
            os.path.join(CSRC, "qpsk_surface.c"), os.path.join(CSRC, "qpsk_records.c")]
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-I" + os.path.join(ROOT, "oracle")]
    subprocess.run(["gcc", *FP, *SAN, *inc, "-o", exe, *srcs, "-lm", "-lpthread"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(d), os.path.join(ROOT, "tests", "golden", "preamble_qpsk_8k.raw")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"sanitizer run failed ({r.returncode}):\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return d


def _rd(d, name, dtype):
    return np.fromfile(os.path.join(d, name), dtype=dtype)


def test_sanitized_generator_matches(san_out):
    x = _rd(san_out, "synth.bin", np.int16).reshape(24, 12, 1880)
    np.testing.assert_array_equal(x, oracle.synth(7, 24, 12, 4.0, c0=100))
    np.testing.assert_array_equal(x, sc.synth(7, 24, 12, 4.0, c0=100))


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_sanitized_oracle_matches(san_out, mode):
    x = oracle.synth(7, 24, 12, 4.0, c0=100)
    bits, valid, tr = oracle.cpu_rx(x, trace=True, mode=mode)
    np.testing.assert_array_equal(_rd(san_out, f"rx_bits_m{mode}.bin", np.uint8).reshape(bits.shape), bits)
    np.testing.assert_array_equal(_rd(san_out, f"rx_valid_m{mode}.bin", np.uint8).reshape(valid.shape), valid)
    t = _rd(san_out, f"rx_trace_m{mode}.bin", TRACE).reshape(valid.shape)
    for k in ("max_index", "matches", "valid", "rx_timing"):
        np.testing.assert_array_equal(t[k], tr[k])
    vm = valid.astype(bool)
    assert (t["soft"][vm].view(np.uint32) == tr["soft"][vm].view(np.uint32)).all()


def test_sanitized_surface_rx_records(san_out):
    """qpsk_rx_frame's host logic + qpsk_records over the sample file: the
    reference output file (md5 of SURVEY.md App. B)."""
    exp = json.load(open(os.path.join(ROOT, "tests", "golden", "sample_expected.json")))
    recs = open(os.path.join(san_out, "surface_records.bin"), "rb").read()
    assert hashlib.md5(recs).hexdigest() == exp["output_md5"]


def test_sanitized_tx_and_surface_helpers(san_out):
    lcg = 12345
    sc.qpsk_tx_init()
    out = []
    for k in range(4):
        syms = []
        for _ in range(128 if k == 0 else 31):
            lcg = (lcg * 1664525 + 1013904223) & 0xFFFFFFFF
            syms.append(sc.qpsk_mod([(lcg >> 16) & 1, (lcg >> 17) & 1], 0))
        out.append(sc.qpsk_tx_frame(np.array(syms, np.complex64), k == 0))
    np.testing.assert_array_equal(_rd(san_out, "tx.bin", np.int16), np.concatenate(out))
    vals = [-2.5, -1.0, -0.0, 0.0, 1e-30, 3.0]
    dm = _rd(san_out, "demod.bin", np.uint8).reshape(36, 2)
    cn = _rd(san_out, "cnormf.bin", np.float32)
    for i, a in enumerate(vals):
        for j, b in enumerate(vals):
            s = complex(np.float32(a), np.float32(b))
            assert list(dm[6 * i + j]) == sc.qpsk_demod(s)
            assert cn[6 * i + j] == np.float32(sc.cnormf(s))
