#!/bin/bash
# 2x4 (one back wave per group) vs 2x4d (dual-chain backs, 2 groups per
# workgroup) at the channel counts that select 2x4, plus 16384 and 65536.
set -o pipefail
for nch in 16384 24576 32768 65536; do for S in 2x4 2x4d; do
  QPSK_SHAPE=$S timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $S', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
