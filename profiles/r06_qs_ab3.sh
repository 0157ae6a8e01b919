#!/bin/bash
# Round 6: QPSK_QSPLIT with the gain wave's ring checks off its chain (the
# equalizer's count read 4 steps ahead, a 16-step ring, signals without waits)
# and the equalizer waves at issue priority 0: the -m gpu suite and the W = 32
# forced tests on it, then 3 interleaved rounds at 8,192 channels.
set -o pipefail
L=singlecarrier_amd/csrc/build
O=gpurun_out/r6c34
mkdir -p $O
QPSK_LIB=$L/lib_qs2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_qs2.log 2>&1 || exit 1
QPSK_LIB=$L/lib_qs2.so QPSK_WIDTH=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "exact_division or quad or random or edge" --timeout 120 --timeout-method thread > $O/pytest_qs2_w32.log 2>&1 || exit 1
bash profiles/libs_ab.sh 3 8192 $O/qs2_ab.txt $L/lib_head.so $L/lib_qsp0.so $L/lib_qs2.so > $O/qs2_ab.log 2>&1
