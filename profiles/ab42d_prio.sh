#!/bin/bash
# 4x2 dual (16 waves, 128 VGPRs; v42d build, QPSK_SHAPE=4x1d selects it there) under
# each issue priority, against the product 4x2.
set -o pipefail
for r in 1 2; do for cfg in "prod::" "v42d:4x1d:front" "v42d:4x1d:back" "v42d:4x1d:none"; do
  IFS=: read lib sh pr <<< "$cfg"
  L=singlecarrier_amd/libqpsk_hip.so; [ $lib = v42d ] && L=singlecarrier_amd/csrc/build/lib_v42d.so
  QPSK_LIB=$L QPSK_SHAPE=$sh QPSK_PRIO=$pr timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done
