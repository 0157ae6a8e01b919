#!/bin/bash
# Round 6: the FIRs' LDS batches.  LLVM had sunk every multiply-add of a
# batched FIR below its last LDS wait (the batches ran as load rounds, all the
# arithmetic after them, 59 samples live).  Variants: anc = accumulators
# anchored per batch (QPSK_FIR_ANCHOR, every shape); pip7 / pip5a / pip7a =
# the split FIR software-pipelined (QPSK_FIR_PIPE, batches of 7 or 5; "a": the
# dual shapes' FIRs anchored too).  C3 and the 16,384 / 8,192 shards,
# interleaved, verified against the oracle each run.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c5
bash profiles/libs_ab.sh 3 65536 gpurun_out/r6c5/pipe_ab_65536.txt prod $L/lib_anc.so $L/lib_pip7.so $L/lib_pip7a.so $L/lib_pip5a.so \
  > gpurun_out/r6c5/pipe_ab_65536.log 2>&1 || exit 1
bash profiles/ab_shards.sh 2 "16384 8192" singlecarrier_amd/libqpsk_hip.so $L/lib_anc.so $L/lib_pip7a.so \
  > gpurun_out/r6c5/pipe_ab_shards.txt 2>&1
