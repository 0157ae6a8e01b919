#!/bin/bash
# call 8 (call 7: dead-lane indexing bug in LB = 32, fixed): lane-back blocks at 16,384 channels (QPSK_BLOCKS) -- parity, A/B with
# issue priorities; machine-scheduler variants at 8,192 and 65,536
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "lane_back_blocks or dual_chain or c4_shards or quad" --timeout 200 --timeout-method thread > gpurun_out/r3c8_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
L=singlecarrier_amd/libqpsk_hip.so
for r in 1 2; do
  timeout -k 10 300 bash profiles/ab_shards.sh 1 "16384" $L 2>&1 | sed "s/^/blocks0 /" >> gpurun_out/r3c8_ab.txt || exit 1
  for pr in front back none; do
    QPSK_BLOCKS=1 QPSK_PRIO=$pr timeout -k 10 300 bash profiles/ab_shards.sh 1 "16384" $L 2>&1 | sed "s/^/blocks1-$pr /" >> gpurun_out/r3c8_ab.txt || exit 1
  done
  timeout -k 10 400 bash profiles/ab_shards.sh 1 "8192 65536" $L singlecarrier_amd/csrc/build/lib_sdef.so singlecarrier_amd/csrc/build/lib_smaxilp.so >> gpurun_out/r3c8_ab.txt 2>&1 || exit 1
done
