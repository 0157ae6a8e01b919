#!/bin/bash
# Pair-of-lanes back waves (QPSK_QUAD=2: two lanes per channel, 32 channels
# per back wave) against the default shapes, interleaved, R rounds, one device:
# 16,384 channels (default: lane backs, W = 64) and 8,192 (default: quad
# backs, W = 32).  Each line: label, channels, ms per step, kernel us, verified.
R=${1:-3}
run() { # label nch [env...]
  local label=$1 nch=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', $nch, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  run lane 16384 || exit 1
  run pair 16384 QPSK_QUAD=2 || exit 1
  run quad 8192 || exit 1
  run pair 8192 QPSK_QUAD=2 || exit 1
done
