#!/bin/bash
# Round 6: confirm QPSK_FIR_ANCHOR=1 (every batched FIR's accumulators pinned
# per LDS batch; 0 VGPR spills in every shape) against the product: 5
# interleaved rounds at C3, 2 at 32,768 and 4,096 channels.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c6
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c6/anc_ab_65536.txt prod $L/lib_anc.so > gpurun_out/r6c6/anc_ab.log 2>&1 || exit 1
bash profiles/ab_shards.sh 2 "32768 4096" singlecarrier_amd/libqpsk_hip.so $L/lib_anc.so 2>/dev/null > gpurun_out/r6c6/anc_ab_shards.txt
