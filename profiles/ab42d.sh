#!/bin/bash
set -o pipefail
for r in 1 2; do for cfg in "prod:" "v42d:" "v42d:4x1d"; do
  lib=${cfg%%:*}; sh=${cfg#*:}
  L=singlecarrier_amd/libqpsk_hip.so; [ $lib = v42d ] && L=singlecarrier_amd/csrc/build/lib_v42d.so
  QPSK_LIB=$L QPSK_SHAPE=$sh timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 128 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
