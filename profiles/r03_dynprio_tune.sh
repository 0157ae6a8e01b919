#!/bin/bash
# Dynamic back priority variants vs the product (QPSK_DYNPRIO=1, poll every
# 4 quad steps, waiting-time priority 0), interleaved, R rounds:
#   poll1 / poll2: priority updated every 1 / 2 quad steps (-DQPSK_DYNPOLL);
#   low1: the training backs drop to 1 (the fronts' level) instead of 0;
#   all2low1: every dual shape, drop to 1 (-DQPSK_DYNPRIO=2 -DQPSK_DYNLOW=1).
# Each line: label, channels, ms per step, kernel us, verified.
R=${1:-2}
B=singlecarrier_amd/csrc/build
run() { # label nch lib
  QPSK_LIB=$3 timeout -k 10 300 python bench.py --channels $2 --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', $2, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  for nch in 8192 4096; do
    run cur $nch singlecarrier_amd/libqpsk_hip.so || exit 1
    for v in poll1 poll2 low1; do run $v $nch $B/lib_$v.so || exit 1; done
  done
  for nch in 16384 32768; do
    run cur $nch singlecarrier_amd/libqpsk_hip.so || exit 1
    run all2low1 $nch $B/lib_all2low1.so || exit 1
  done
done
