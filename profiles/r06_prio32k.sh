#!/bin/bash
# Round 6: issue priority in the 2x4 dual-chain kernel at 32,768 channels (the
# N = 2 shard): default (none) / front / back, 3 interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/r6c43
for r in 1 2 3; do for PR in default front back; do
  env $([ $PR = default ] || echo QPSK_PRIO=$PR) timeout -k 10 300 python bench.py --channels 32768 \
    --cpu-channels 0 --cpu-all-channels 0 --cpu-procs 0 --stream-chunks 0 --frame-latency 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('32768 $PR', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" || exit 1
done; done > gpurun_out/r6c43/prio32k.txt 2> gpurun_out/r6c43/prio32k.err
