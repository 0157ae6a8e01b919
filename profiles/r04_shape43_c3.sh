#!/bin/bash
# C3 with the default 4x2 shape and the 4x3 kernel (QPSK_SHAPE), interleaved, 2 rounds
for r in 1 2; do
  for sh in 4x2 4x3; do
    QPSK_SHAPE=$sh timeout -k 10 300 python bench.py --channels 65536 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --verify 64 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('65536', '$sh', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
  done
done
