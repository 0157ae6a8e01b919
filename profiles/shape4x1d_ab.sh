#!/bin/bash
# 65,536 channels: 4x2 (default) vs 4x1d (two back waves per group, one per
# frame chain, and one front wave per group) under each issue priority.
set -o pipefail
one() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 \
    --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lab', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for rep in 1 2; do
  one 4x2 X=1 || exit 1
  one 4x1d QPSK_SHAPE=4x1d || exit 1
  one 4x1d-back QPSK_SHAPE=4x1d QPSK_PRIO=back || exit 1
  one 4x1d-none QPSK_SHAPE=4x1d QPSK_PRIO=none || exit 1
done
