#!/bin/bash
# FIR products first, then the sums (no wait state between a packed multiply and the
# dependent packed add): the product
# library vs the previous HEAD (lib_base.so), interleaved, R rounds, at every
# shard size.  Each line: label, channels, ms per step, kernel us, verified.
R=${1:-3}
run() { # label nch lib
  QPSK_LIB=$3 timeout -k 10 300 python bench.py --channels $2 --cpu-channels 0 \
    --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', $2, d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for r in $(seq 1 $R); do
  for nch in 8192 4096 16384 32768 65536; do
    run base $nch singlecarrier_amd/csrc/build/lib_base.so || exit 1
    run new $nch singlecarrier_amd/libqpsk_hip.so || exit 1
  done
done
