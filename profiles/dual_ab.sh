#!/bin/bash
# A/B of the one-group-per-workgroup shapes: 1x8 (dual-chain back waves) vs
# 1x8s (single back wave), at the channel counts that select them, plus the
# default 4x2 point.  Run on the GPU box from the repo root.
set -o pipefail
for nch in 2048 4096 8192 16384 65536; do for S in 1x8 1x8s default; do
  [ $nch = 65536 ] && [ $S != default ] && continue
  QPSK_SHAPE=$([ $S = default ] || echo $S) timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $S', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
for nch in 4096 8192 16384; do for W in 16 32 64; do
  QPSK_WIDTH=$W timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch W=$W', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
