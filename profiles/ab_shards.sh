#!/bin/bash
# A/B of library variants over the C4 shard sizes (and C3), interleaved,
# R rounds, one device: ms per step (rx + data kernel) at each size.
#   bash profiles/ab_shards.sh R "65536 32768 16384 8192" lib1 lib2 ...
R=$1; SIZES=$2; shift 2
for r in $(seq 1 $R); do
  for nch in $SIZES; do
    for lib in "$@"; do
      QPSK_LIB=$lib timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 \
        --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
        | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch', '$(basename $lib)', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" \
        || exit 1
    done
  done
done
