#!/bin/bash
# A/B on one device: bench each library variant, interleaved, R rounds.
#   usage: bash profiles/ab.sh R lib1 lib2 ...
# Variant libraries: bash profiles/variant.sh NAME SRC.hip [extra hipcc flags]
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    QPSK_LIB=$lib timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 \
      --stream-chunks 0 --verify 0 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['roofline']['kernels_us'])" \
      || exit 1
  done
done
