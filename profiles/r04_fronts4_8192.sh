#!/bin/bash
# 8,192 channels: default 1x8 quad vs QPSK_FRONTS=4 (1x4), interleaved, 3 rounds
for r in 1 2 3; do
  for fr in 8 4; do
    QPSK_FRONTS=$fr timeout -k 10 300 python bench.py --channels 8192 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --verify 64 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('8192', 'fronts=$fr', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
  done
done
