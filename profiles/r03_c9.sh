#!/bin/bash
# call 9: the 4x3 C3 shape (three front waves per group, compact front input,
# 4 waves per SIMD) -- parity, A/B against 4x2 at 65,536 channels
set -u
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "workgroup_shape or low_amplitude or full_size_c3 or synth_goldens or edge_inputs or streaming_split" --timeout 300 --timeout-method thread > gpurun_out/r3c9_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
L=singlecarrier_amd/libqpsk_hip.so
for r in 1 2 3; do
  QPSK_SHAPE=4x2 timeout -k 10 300 bash profiles/ab_shards.sh 1 "65536" $L 2>&1 | sed "s/^/4x2 /" >> gpurun_out/r3c9_ab.txt || exit 1
  QPSK_SHAPE=4x3 timeout -k 10 300 bash profiles/ab_shards.sh 1 "65536" $L 2>&1 | sed "s/^/4x3 /" >> gpurun_out/r3c9_ab.txt || exit 1
done
