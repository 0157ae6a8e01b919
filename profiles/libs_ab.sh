#!/bin/bash
# A/B of library variants on one box, interleaved, R rounds, at one batch size;
# every run also verifies its first 64 channels against the oracle.
#   bash profiles/libs_ab.sh R CHANNELS OUTFILE lib1 lib2 ...   ("prod" = the product library)
set -o pipefail
R=$1; NCH=$2; OUT=$3; shift 3
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 $R); do
  for lib in "$@"; do
    L=$lib; [ "$lib" = prod ] && L=
    env ${L:+QPSK_LIB=$L} timeout -k 10 300 python bench.py --channels $NCH --cpu-channels 0 --cpu-all-channels 0 \
      --stream-chunks 0 --frame-latency 0 --verify 64 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$NCH', '$(basename $lib)', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" \
      || exit 1
  done
done | tee "$OUT"
