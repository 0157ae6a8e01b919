#!/bin/bash
# Issue priority in the dual-chain kernel (1x8): front (default), back, none.
set -o pipefail
for nch in 8192 16384; do for PR in front back none; do
  QPSK_PRIO=$PR timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 0 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $PR', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'])" || exit 1
done; done
