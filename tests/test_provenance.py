"""Counter provenance (CPU): the counters bench.py reports next to a live
measurement (roofline.traffic from FETCH_SIZE/WRITE_SIZE, valu from
SQ_INSTS_VALU) are read from committed rocprofv3 records, so they must belong
to the library being timed.  The Makefile compiles a hash of the receive
kernels' sources and build rules into the library (qpsk_kernel_hash());
profiles/summarize.py stores the profiled library's hash in each record and
bench.pmc_record() drops a record whose hash differs from the running one."""
import json
import os
import re
import shutil

import pytest

import bench
import singlecarrier_amd as sc

CSRC = os.path.join(os.path.dirname(sc.__file__), "csrc")


def _lib_built():
    if not os.path.exists(sc.LIB_PATH):
        pytest.skip("library not built")


def test_library_hash_is_the_sources_hash():
    _lib_built()
    assert re.fullmatch(r"[0-9a-f]{16}", sc.kernel_hash())
    assert sc.kernel_hash() == sc.kernel_source_hash()


def test_makefile_hashes_the_listed_sources():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    body = re.search(r"^KSRC\s*:=((?:.*\\\n)*.*)$", mk, re.M).group(1)
    assert tuple(body.replace("\\\n", " ").split()) == sc.KERNEL_SOURCES


def _write_records(root, khash, nch=65536, nf=32):
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    json.dump({"channels": nch, "frames": nf, "hbm_bytes_per_launch": 123, "kernel_hash": khash,
               "source": "test"}, open(os.path.join(root, "profiles", "pmc_traffic.json"), "w"))
    json.dump({"channels": nch, "frames": nf, "valu_insts_per_launch": 456, "kernel_hash": khash,
               "source": "test"}, open(os.path.join(root, "profiles", "pmc_valu.json"), "w"))


def test_one_flipped_source_byte_drops_the_counters(tmp_path):
    """Records profiled with the current kernels are reported; after one byte
    of qpsk_rx.hip changes, the rebuilt library's hash differs and both
    records are dropped (traffic null, no measured valu)."""
    cur = sc.kernel_source_hash()
    _write_records(str(tmp_path), cur)
    p = bench.pmc_record("pmc_traffic.json", 65536, 32, "reference", cur, root=str(tmp_path))
    assert p is not None and p["hbm_bytes_per_launch"] == 123
    v = bench.valu_from_counters(bench.pmc_record("pmc_valu.json", 65536, 32, "reference", cur,
                                                  root=str(tmp_path)), 6e-3)
    assert v is not None and v["valu_insts_per_launch"] == 456 and v["kernel_hash"] == cur
    # the same sources with one byte flipped
    src = tmp_path / "csrc"
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    f = src / "qpsk_rx.hip"
    b = bytearray(f.read_bytes())
    b[len(b) // 2] ^= 1
    f.write_bytes(bytes(b))
    new = sc.kernel_source_hash(str(src))
    assert new != cur
    for name in ("pmc_traffic.json", "pmc_valu.json"):
        assert bench.pmc_record(name, 65536, 32, "reference", new, root=str(tmp_path)) is None
    assert bench.valu_from_counters(None, 6e-3) is None
    # a record without a hash (older profiles) is never reported either
    _write_records(str(tmp_path), None)
    assert bench.pmc_record("pmc_traffic.json", 65536, 32, "reference", cur, root=str(tmp_path)) is None


def test_record_of_another_workload_is_dropped(tmp_path):
    cur = sc.kernel_source_hash()
    _write_records(str(tmp_path), cur, nch=8192)
    assert bench.pmc_record("pmc_traffic.json", 65536, 32, "reference", cur, root=str(tmp_path)) is None
    assert bench.pmc_record("pmc_traffic.json", 8192, 32, "dec752", cur, root=str(tmp_path)) is None


def _make(*args):
    import subprocess
    inc = os.path.join(os.path.dirname(CSRC), "..", "include")
    return subprocess.run(["make", "-s", "--no-print-directory", "-C", CSRC, f"INCDIR={os.path.abspath(inc)}",
                           *args], capture_output=True, text=True)


def test_variant_flags_change_the_hash_and_force_a_rebuild():
    """a QPSK_VARIANT build must never keep the product's
    hash, a plain `make` after it must rebuild the product object, and knobs
    with quotes or spaces must hash as written (the flags reach the hash
    through a file, not the shell's quoting)."""
    _lib_built()
    base = _make("khash").stdout.strip()
    assert base == sc.kernel_hash()
    var = _make("khash", "QPSK_VARIANT=-DQPSK_FIR_NOMASK=1").stdout.strip()
    quoted = _make("khash", "QPSK_VARIANT=-DQPSK_RX_ATTR='__attribute__((amdgpu_num_vgpr(128)))'")
    assert quoted.returncode == 0 and re.fullmatch(r"[0-9a-f]{16}", quoted.stdout.strip())
    assert len({base, var, quoted.stdout.strip()}) == 3
    # the object depends on a per-hash stamp: with the variant's flags the
    # product object is out of date (dry run: nothing is built here)
    dry = _make("-n", "QPSK_VARIANT=-DQPSK_FIR_NOMASK=1")
    assert "qpsk_rx.hip" in dry.stdout and "QPSK_FIR_NOMASK" in dry.stdout
    assert "qpsk_rx.hip" not in _make("-n").stdout
