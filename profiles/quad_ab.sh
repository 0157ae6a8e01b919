#!/bin/bash
# A/B of the dual-chain back layouts at the C4 shard sizes: a lane per channel
# (QPSK_QUAD=0) vs a quad of lanes per channel (QPSK_QUAD=1, back_frame_quad),
# each at pick_shape's group width, plus forced widths where they differ.
# Run on the GPU box from the repo root.
set -o pipefail
run() {  # label, env..., -- nch
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --channels $NCH --cpu-channels 0 --cpu-all-channels 0 \
    --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$NCH $label', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for NCH in 4096 8192 16384 32768; do
  run lane QPSK_QUAD=0 || exit 1
  run quad QPSK_QUAD=1 || exit 1
done
NCH=16384; run quad-W32 QPSK_QUAD=1 QPSK_WIDTH=32 || exit 1
NCH=16384; run quad-W64 QPSK_QUAD=1 QPSK_WIDTH=64 || exit 1
