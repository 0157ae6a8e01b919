#!/bin/bash
# C4 strong-scaling shard sizes on ONE GPU: the 65,536-channel batch split N
# ways (no collective exists on the data path, so an N-GPU run's job time is
# the slowest shard's time; this measures each shard size's time per step).
set -o pipefail
for N in 1 2 4 8; do
  nch=$((65536 / N))
  timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 --cpu-all-channels 0 \
    --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('N=$N shard $nch', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done
