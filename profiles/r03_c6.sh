#!/bin/bash
# call 6: per-block front batches in the dual-chain kernel -- parity, stamps at
# 8192, A/B vs the kernel before at the shard sizes (and C3 as a control)
set -u
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_dec752.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r3c6_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python profiles/stamps_dual.py 8192 > gpurun_out/r3c6_stamps8192.txt 2>&1; echo "stamps rc=$?" >&2
L=singlecarrier_amd/libqpsk_hip.so
B=singlecarrier_amd/csrc/build/lib_base.so
for r in 1 2; do
  timeout -k 10 400 bash profiles/ab_shards.sh 1 "8192 16384 4096 65536" $B $L >> gpurun_out/r3c6_ab.txt 2>&1 || exit 1
  QPSK_PRIO=back timeout -k 10 300 bash profiles/ab_shards.sh 1 "8192" $L 2>&1 | sed "s/^/prio-back /" >> gpurun_out/r3c6_ab.txt || exit 1
done
