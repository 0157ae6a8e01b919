#!/bin/bash
# call 3: early decisions with the rt acquire fix -- parity subset, stamps at
# 8192, A/B vs lib_base incl. back issue priority
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_dec752.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/c3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python profiles/stamps_dual.py 8192 > gpurun_out/c3_stamps8192.txt 2>&1; echo "stamps rc=$?" >&2
export QPSK_PRIO=back
timeout -k 10 120 python profiles/stamps_dual.py 8192 > gpurun_out/c3_stamps8192_backprio.txt 2>&1; echo "stamps rc=$?" >&2
unset QPSK_PRIO
for r in 1 2; do
  timeout -k 10 300 bash profiles/ab_shards.sh 1 "8192 16384" singlecarrier_amd/csrc/build/lib_base.so singlecarrier_amd/libqpsk_hip.so >> gpurun_out/c3_ab.txt 2>&1 || exit 1
  QPSK_PRIO=back timeout -k 10 300 bash profiles/ab_shards.sh 1 "8192 16384" singlecarrier_amd/libqpsk_hip.so >> gpurun_out/c3_ab_backprio.txt 2>&1 || exit 1
  QPSK_PRIO=none timeout -k 10 300 bash profiles/ab_shards.sh 1 "8192 16384" singlecarrier_amd/libqpsk_hip.so >> gpurun_out/c3_ab_noprio.txt 2>&1 || exit 1
done
