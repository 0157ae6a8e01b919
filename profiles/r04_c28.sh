#!/bin/bash
# Round 4, call 28 (rerun of 26, whose QPSK_FRONTS=4 runs still picked the lane-back shape at W = 64): 1x4 with quad backs at W = 64 (16,384 channels: 8 quad back
# waves in 4 blocks + 4 fronts) vs the default lane-back 1x8 W = 64
set -u
O=gpurun_out/r4c28
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
QPSK_FRONTS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "quad or c4_shards or dual or one_front" -x -v \
  --timeout 200 --timeout-method thread > ${O}_pytest.log 2>&1; check pytest $?
timeout -k 10 300 bash profiles/knob_ab.sh 2 16384 QPSK_FRONTS=8 QPSK_FRONTS=4 >> ${O}_ab.txt 2>&1; check ab $?
QPSK_FRONTS=4 timeout -k 10 120 python profiles/stamps_dual.py 16384 > ${O}_stamps_16384_f4.txt 2>&1; check stamps $?
