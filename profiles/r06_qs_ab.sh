#!/bin/bash
# Round 6: quad backs split into gain + equalizer waves (QPSK_QSPLIT, 1x4 at
# W = 32): the GPU suite on the variant, the W = 32 exact-retrain and quad tests
# forced through it, then 3 interleaved rounds at 8,192 channels against HEAD.
set -o pipefail
L=singlecarrier_amd/csrc/build
O=gpurun_out/r6c31
mkdir -p $O
QPSK_LIB=$L/lib_qs.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_qs.log 2>&1 || exit 1
QPSK_LIB=$L/lib_qs.so QPSK_WIDTH=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "exact_division or quad or random or edge" --timeout 120 --timeout-method thread > $O/pytest_qs_w32.log 2>&1 || exit 1
bash profiles/libs_ab.sh 3 8192 $O/qs_ab.txt $L/lib_head.so $L/lib_qs.so > $O/qs_ab.log 2>&1
