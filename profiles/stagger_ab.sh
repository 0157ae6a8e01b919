#!/bin/bash
# Front-wave stagger A/B (QPSK_STAGGER = units of 512 cycles the second half of
# the front waves sleeps at each frame start), 65536 channels, 4x2.
set -o pipefail
for r in 1 2; do for S in 0 4 10 16; do
  QPSK_STAGGER=$S timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 \
    --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('stagger $S', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
