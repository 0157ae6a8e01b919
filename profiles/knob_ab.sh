#!/bin/bash
# A/B of environment knobs on one device, interleaved, R rounds, at one batch size.
#   usage: bash profiles/knob_ab.sh R CHANNELS "QPSK_X=a" "QPSK_X=b" ...
R=$1; NCH=$2; shift 2
for r in $(seq 1 $R); do
  for kv in "$@"; do
    env $kv timeout -k 10 300 python bench.py --channels $NCH --cpu-channels 0 --cpu-all-channels 0 \
      --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$NCH $kv', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" \
      || exit 1
  done
done
