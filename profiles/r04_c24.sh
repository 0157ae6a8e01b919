#!/bin/bash
# Round 4, call 24: back/front stamps of the 1x4 and 1x8 quad shapes at 8,192 channels
set -u
O=gpurun_out/r4c24
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for f in 4 8; do
  QPSK_FRONTS=$f timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192_f$f.txt 2>&1; check stamps$f $?
  QPSK_FRONTS=$f QPSK_ABLATE=frontidle timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192_f${f}_idle.txt 2>&1; check idle$f $?
done
