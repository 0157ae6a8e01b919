#!/bin/bash
# call 13: the FIR-head pre-pass (QPSK_HEADPASS=1) and the
# 1x10 shape at 16,384 channels -- parity, A/B against the defaults
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "head_prepass or workgroup_shape or dual_chain or c4_shards or 1x10" --timeout 300 --timeout-method thread > gpurun_out/r3c13_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
L=singlecarrier_amd/libqpsk_hip.so
for r in 1 2; do
  for n in 16384 8192 32768 65536; do
    timeout -k 10 300 bash profiles/ab_shards.sh 1 "$n" $L 2>&1 | sed "s/^/default /" >> gpurun_out/r3c13_ab.txt || exit 1
    QPSK_HEADPASS=1 timeout -k 10 300 bash profiles/ab_shards.sh 1 "$n" $L 2>&1 | sed "s/^/prepass /" >> gpurun_out/r3c13_ab.txt || exit 1
  done
  for pr in front back; do
    QPSK_SHAPE=1x10 QPSK_PRIO=$pr timeout -k 10 300 bash profiles/ab_shards.sh 1 "16384" $L 2>&1 | sed "s/^/1x10-$pr /" >> gpurun_out/r3c13_ab.txt || exit 1
  done
done
QPSK_SHAPE=1x10 timeout -k 10 120 python profiles/stamps_dual.py 16384 > gpurun_out/r3c13_stamps16384_1x10.txt 2>&1; echo "stamps rc=$?" >&2
