#!/bin/bash
# call 5: decided-first channel order -- parity subset; A/B vs base at every
# shard size; issue-priority variants
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_dec752.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r3c5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ge 124 ] && exit $rc
L=singlecarrier_amd/libqpsk_hip.so
B=singlecarrier_amd/csrc/build/lib_base.so
for r in 1 2; do
  timeout -k 10 400 bash profiles/ab_shards.sh 1 "65536 32768 16384 8192" $B $L >> gpurun_out/r3c5_ab.txt 2>&1 || exit 1
  for pr in back none; do
    QPSK_PRIO=$pr timeout -k 10 300 bash profiles/ab_shards.sh 1 "65536 8192" $L 2>&1 | sed "s/^/prio-$pr /" >> gpurun_out/r3c5_ab.txt || exit 1
  done
done
