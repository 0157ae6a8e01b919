#!/bin/bash
# call 4: fcnt fix check (parity subset), then C3 A/B: base vs 4x2 vs 4x2d (prio variants)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_dec752.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/c4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ge 124 ] && exit $rc
L=singlecarrier_amd/libqpsk_hip.so
B=singlecarrier_amd/csrc/build/lib_base.so
for r in 1 2; do
  timeout -k 10 300 bash profiles/ab_shards.sh 1 "65536" $B $L >> gpurun_out/c4_ab.txt 2>&1 || exit 1
  for pr in front back none; do
    QPSK_SHAPE=4x2d QPSK_PRIO=$pr timeout -k 10 300 bash profiles/ab_shards.sh 1 "65536" $L 2>&1 | sed "s/^/4x2d-$pr /" >> gpurun_out/c4_ab.txt || exit 1
  done
done
