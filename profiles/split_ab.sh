#!/bin/bash
# Dual-chain kernel: uneven front channel split (QPSK_SPLIT) x issue priority
# (QPSK_PRIO), at the C4 N=8 and N=4 shard sizes.
set -o pipefail
for nch in 8192 16384; do for cfg in "0:front" "1:front" "1:back" "2:back" "2:front"; do
  sp=${cfg%%:*}; pr=${cfg#*:}
  [ $nch = 16384 ] && [ $sp = 1 ] && sp=2 && [ $pr = front ] && continue
  QPSK_SPLIT=$sp QPSK_PRIO=$pr timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch split=$sp prio=$pr', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
