#!/bin/bash
# Flow kernel at small batches (the back recursion bounds each frame there):
# 1x8f (one group per workgroup, per-lane frames, early-terminated training)
# vs the default dual-chain shapes.  Repo root, GPU box.
set -o pipefail
one() {  # label, channels, env...
  local lab=$1 nch=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $lab', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for rep in 1 2; do
  for nch in 16384 8192 4096; do
    one default $nch X=1 || exit 1
    one 1x8f $nch QPSK_SHAPE=1x8f || exit 1
    one 1x8f-noearly $nch QPSK_SHAPE=1x8f QPSK_EARLY=0 || exit 1
  done
done
