#!/bin/bash
# Round 6: the split FIR in the dual-chain shapes too (QPSK_FIR_SPLIT=2), now
# with round 6's conflict-free pass 1 and anchored batches (round 5, without
# them: +0.2..1%), against the product at the C4 shard sizes, 2 rounds.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c17
bash profiles/ab_shards.sh 2 "32768 16384 8192 4096" singlecarrier_amd/libqpsk_hip.so $L/lib_split2.so 2>/dev/null \
  > gpurun_out/r6c17/split2_ab.txt
