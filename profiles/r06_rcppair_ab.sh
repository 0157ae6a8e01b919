#!/bin/bash
# Round 6: the lane back's reciprocal Newton steps on packed pairs
# (QPSK_RCP_PAIR=1; round 5 measured +0.8% with 4 more spilled VGPRs; round 6's
# anchored FIR freed registers: the back loop 943 -> 929 instructions per 4
# steps) against the product, 5 interleaved rounds at C3, 2 at 16,384.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c13
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c13/rcppair_ab.txt prod $L/lib_rcppair.so > gpurun_out/r6c13/ab.log 2>&1 || exit 1
bash profiles/ab_shards.sh 2 "16384" singlecarrier_amd/libqpsk_hip.so $L/lib_rcppair.so 2>/dev/null > gpurun_out/r6c13/rcppair_ab_16384.txt
