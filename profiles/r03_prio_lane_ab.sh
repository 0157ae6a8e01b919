#!/bin/bash
# Static issue priority of the lane-back dual shapes (QPSK_PRIO: front / back /
# none) against the product's choice (32,768: front priority; 16,384: back
# priority with split 2), interleaved, R rounds.  Each line: label, channels,
# ms per step, kernel us, verified.
R=${1:-2}
run() { # label nch [env...]
  local label=$1 nch=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', $nch, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  for nch in 32768 16384; do
    run default $nch || exit 1
    for pr in front back none; do run prio-$pr $nch QPSK_PRIO=$pr || exit 1; done
  done
done
