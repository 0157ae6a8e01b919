#!/bin/bash
# Double-quad back waves (QPSK_QUAD=2, 32 channels per back wave) at the
# 16,384-channel shard, interleaved A/B, R rounds: HEAD's library (default
# shape), the working library with and without QPSK_QUAD=2, and the
# default-scheduler build (lib_noilp: the double-quad kernel without spills).
# Each line: label, channels, ms per step, kernel us, verified vs oracle.
R=${1:-3}
run() { # label nch lib [env...]
  local label=$1 nch=$2 lib=$3; shift 3
  env "$@" QPSK_LIB=$lib timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', $nch, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
B=singlecarrier_amd/csrc/build
for r in $(seq 1 $R); do
  run base 16384 $B/lib_base.so || exit 1
  run cur-q2 16384 singlecarrier_amd/libqpsk_hip.so QPSK_QUAD=2 || exit 1
  run noilp-q2 16384 $B/lib_noilp.so QPSK_QUAD=2 || exit 1
  run noilp 16384 $B/lib_noilp.so || exit 1
  run cur 16384 singlecarrier_amd/libqpsk_hip.so || exit 1
  run base 8192 $B/lib_base.so || exit 1
  run cur 8192 singlecarrier_amd/libqpsk_hip.so || exit 1
done
