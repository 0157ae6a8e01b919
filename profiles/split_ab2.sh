#!/bin/bash
# 16384 channels (1x8 dual, W=64): front split sweep with back priority.
set -o pipefail
for r in 1 2; do for cfg in "0:front" "2:back" "3:back" "4:back" "5:back" "3:none"; do
  sp=${cfg%%:*}; pr=${cfg#*:}
  QPSK_SPLIT=$sp QPSK_PRIO=$pr timeout -k 10 300 python bench.py --channels 16384 --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('16384 split=$sp prio=$pr', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
