#!/bin/bash
# rx_data_kernel launch geometry A/B at C3 (QPSK_DATA_GRID x QPSK_DATA_BLOCK).
set -o pipefail
for r in 1 2; do for cfg in ${CFGS:-"1024:256" "2048:128" "4096:64" "2048:256" "768:256" "512:256"}; do
  g=${cfg%%:*}; b=${cfg#*:}
  QPSK_DATA_GRID=$g QPSK_DATA_BLOCK=$b timeout -k 10 300 python bench.py --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('grid $g block $b', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
