#!/bin/bash
# Round 6, item 6: one stamps run of the 4x2 kernel at C3 (diagnostic build,
# singlecarrier_amd/csrc/build/libqpsk_hip_stamps.so: make stamps), both roles
# and fronts alone: per-phase cycles and the back wave's tail after the last
# front of its SIMD reached the frame barrier (profiles/stamps.py).
#   bash profiles/r06_stamps.sh OUTDIR
set -o pipefail
OUT=$1
mkdir -p $OUT
timeout -k 10 300 python profiles/stamps.py both > $OUT/stamps_both.json 2> $OUT/stamps_both.err || exit 1
timeout -k 10 300 python profiles/stamps.py front > $OUT/stamps_front.json 2> $OUT/stamps_front.err || exit 1
echo done > $OUT/DONE
