#!/bin/bash
# Round 4, call 30: where the 4x3 kernel loses: each role alone (QPSK_ABLATE,
# timing only) in 4x2 and 4x3 at C3
set -u
O=gpurun_out/r4c30
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for ab in front back; do
  for sh in 4x2 4x3; do
    QPSK_ABLATE=$ab QPSK_SHAPE=$sh timeout -k 10 200 python bench.py --channels 65536 --cpu-channels 0 --cpu-all-channels 0 \
      --stream-chunks 0 --frame-latency 0 --verify 0 --steps 5 --warmup 2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$ab $sh', d['ms_per_step'], d['roofline']['kernels_us'])" >> ${O}_ablate.txt 2>&1
    check $ab$sh $?
  done
done
