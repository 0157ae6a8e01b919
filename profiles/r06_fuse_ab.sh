#!/bin/bash
# Round 6: the split FIR's two passes fused into one batched loop
# (QPSK_FIR_FUSE=1: 4 waits instead of 4 + 7, four interleaved accumulation
# chains, 68 s_nop per channel instead of 115) against the product (anchored
# passes), 5 interleaved rounds at C3, verified each run.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c9
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c9/fuse_ab.txt prod $L/lib_fuse.so > gpurun_out/r6c9/fuse_ab.log 2>&1
