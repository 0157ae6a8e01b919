#!/bin/bash
# Progress-balanced issue priority in the 4x2 (C3) kernel (-DQPSK_BALANCE=1):
# the back wave publishes its training step every 4 steps and runs at issue
# priority 1; each front wave runs at 2 but drops to 0 while it is further
# through its channels than the back through its 128 steps (+ margin steps,
# -DQPSK_BALANCE_MARGIN: bal0 0, bal8 8, balm8 -8).  Interleaved with the
# product library, R rounds, 65,536 channels.  Each line: label, channels,
# ms per step, kernel us, verified vs oracle (64 channels).
R=${1:-3}
B=singlecarrier_amd/csrc/build
run() { # label nch lib
  QPSK_LIB=$3 timeout -k 10 300 python bench.py --channels $2 --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', $2, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  run cur 65536 singlecarrier_amd/libqpsk_hip.so || exit 1
  for v in bal0 bal8 balm8; do run $v 65536 $B/lib_$v.so || exit 1; done
done
