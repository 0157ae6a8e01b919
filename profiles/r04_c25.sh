#!/bin/bash
# Round 4, call 25: the quad step's gain half alone (-DQPSK_ABL_EQ, timing only:
# output invalid) beside the fronts, 1x4 and 1x8 at 8,192 channels
set -u
O=gpurun_out/r4c25
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for f in 4 8; do
  QPSK_STAMPS_LIB=singlecarrier_amd/csrc/build/libqpsk_hip_stamps_ableq.so QPSK_FRONTS=$f timeout -k 10 120 \
    python profiles/stamps_dual.py 8192 > ${O}_ableq_8192_f$f.txt 2>&1; check ableq$f $?
done
