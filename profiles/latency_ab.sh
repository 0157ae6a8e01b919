#!/bin/bash
# Drop-in latency A/B: qpsk_rx_frame() per call (bench.py's drop_in_frame_latency),
# library variants interleaved, R rounds, one box.
#   bash profiles/latency_ab.sh R OUTFILE lib1 lib2 ...   ("prod" = the product library)
set -o pipefail
R=$1; OUT=$2; shift 2
for r in $(seq 1 $R); do
  for lib in "$@"; do
    L=$lib; [ "$lib" = prod ] && L=
    env ${L:+QPSK_LIB=$L} timeout -k 10 300 python bench.py --channels 4096 --steps 2 --warmup 1 --cpu-channels 0 \
      --cpu-all-channels 0 --stream-chunks 0 --verify 0 --frame-latency 1024 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1])['drop_in_frame_latency']; print('$(basename $lib)', d['p50_us'], d['p99_us'], d['mean_us'], d['sample_file_md5_ok'])" \
      || exit 1
  done
done | tee "$OUT"
