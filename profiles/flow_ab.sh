#!/bin/bash
# A/B of the flow kernel (rx_kernel<.., FLOW>: per-lane frames, early-terminated
# training, per-channel LDS counters) against the default shapes, at the bench
# workload (65,536 channels) and at 32,768 (2 groups per CU).  Repo root, GPU box.
set -o pipefail
one() {  # label, channels, env...
  local lab=$1 nch=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $lab', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for rep in 1 2; do
  one default 65536 X=1 || exit 1
  one 4x2f 65536 QPSK_SHAPE=4x2f || exit 1
  one 4x2f-noearly 65536 QPSK_SHAPE=4x2f QPSK_EARLY=0 || exit 1
done
one default 32768 X=1 || exit 1
one 2x4f 32768 QPSK_SHAPE=2x4f || exit 1
one 4x2f 32768 QPSK_SHAPE=4x2f || exit 1
