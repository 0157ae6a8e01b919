#!/bin/bash
# 65536 channels: 4x2 (default) vs the dual-chain shapes 4x1d and 2x4d, R rounds interleaved.
set -o pipefail
for r in 1 2; do for S in 4x2 4x1d 2x4d; do
  QPSK_SHAPE=$S timeout -k 10 300 python bench.py --channels ${NCH:-65536} \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('${NCH:-65536} $S', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
