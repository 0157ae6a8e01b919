"""Exhaustive check of the kernel's fast reciprocal (singlecarrier_amd/csrc/
qpsk_rcp.h): bit-identical to IEEE fp32 1.0f/x for every positive finite
float, so using it in kalman_calculate (src/kalman.c:162,173) keeps parity."""
import ctypes as C
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kernels")


def test_rcp_rn_is_correctly_rounded_everywhere():
    lib_path = os.path.join(HERE, "librcp_check.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE], check=True)
    lib = C.CDLL(lib_path)
    lib.rcp_check.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_ulonglong),
                              C.POINTER(C.c_uint32)]
    bad, first = C.c_ulonglong(0), C.c_uint32(0)
    # every positive float from the smallest denormal to +inf, plus NaNs
    assert lib.rcp_check(0x00000000, 0x7FFFFFFF, C.byref(bad), C.byref(first)) == 0
    assert bad.value == 0, f"{bad.value} mismatches, first at 0x{first.value:08x}"
    # and the negative ones
    assert lib.rcp_check(0x80000000, 0xFFFFFFFF, C.byref(bad), C.byref(first)) == 0
    assert bad.value == 0, f"{bad.value} mismatches, first at 0x{first.value:08x}"
