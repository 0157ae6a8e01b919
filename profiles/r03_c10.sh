#!/bin/bash
# call 10: front prefetch without 64-bit lane addresses (straddling items
# loaded from both frames, selected in the mixer) -- parity, stamps at 8192,
# A/B vs HEAD at every shard size
set -u
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dec752.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3c10_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python profiles/stamps_dual.py 8192 > gpurun_out/r3c10_stamps8192.txt 2>&1; echo "stamps rc=$?" >&2
L=singlecarrier_amd/libqpsk_hip.so
B=singlecarrier_amd/csrc/build/lib_base.so
for r in 1 2; do
  timeout -k 10 400 bash profiles/ab_shards.sh 1 "8192 16384 32768 65536 4096" $B $L >> gpurun_out/r3c10_ab.txt 2>&1 || exit 1
done
