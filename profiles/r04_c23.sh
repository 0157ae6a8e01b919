#!/bin/bash
# Round 4, call 23: 1x4 quad shapes (4 back + 4 front waves, one of each per
# SIMD, 178 VGPRs at 2 waves/SIMD) vs 1x8 at the quad shard sizes; parity of
# the quad/C4 tests with QPSK_FRONTS=4 first.
set -u
O=gpurun_out/r4c23
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
QPSK_FRONTS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "quad or c4_shards or dual" -x -v \
  --timeout 200 --timeout-method thread > ${O}_pytest.log 2>&1; check pytest $?
for n in 4096 8192; do
  timeout -k 10 300 bash profiles/knob_ab.sh 2 $n QPSK_FRONTS=8 QPSK_FRONTS=4 >> ${O}_ab.txt 2>&1; check ab$n $?
done
