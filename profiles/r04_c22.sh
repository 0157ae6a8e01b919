#!/bin/bash
# Round 4, call 22: stamps + guessed/redone channel counts of the speculative fronts
set -u
O=gpurun_out/r4c22
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for n in 8192 16384; do
  timeout -k 10 120 python profiles/stamps_dual.py $n > ${O}_stamps_$n.txt 2>&1; check stamps$n $?
done
