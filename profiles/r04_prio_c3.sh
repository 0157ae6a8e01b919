#!/bin/bash
# C3 with each static issue priority (QPSK_PRIO), interleaved, R rounds
for r in 1 2; do
  for pr in front back none; do
    QPSK_PRIO=$pr timeout -k 10 300 python bench.py --channels 65536 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --verify 64 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('65536', '$pr', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
  done
done
