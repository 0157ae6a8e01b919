#!/bin/bash
# Dynamic back priority (-DQPSK_DYNPRIO=1, lib_dyn.so): dual-chain back waves
# train at issue priority 2 (fronts 1) and drop to 0 every 4 steps while
# another back wave waits for its fronts; vs the product library, interleaved,
# R rounds, at the dual-chain shard sizes.  Each line: label, channels, ms per
# step, kernel us, verified vs oracle (64 channels).
R=${1:-3}
run() { # label nch lib
  QPSK_LIB=$3 timeout -k 10 300 python bench.py --channels $2 --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', $2, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  for nch in 8192 16384 32768 4096; do
    run base $nch singlecarrier_amd/libqpsk_hip.so || exit 1
    run dyn $nch singlecarrier_amd/csrc/build/lib_dyn.so || exit 1
  done
done
