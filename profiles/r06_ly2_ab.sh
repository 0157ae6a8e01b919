#!/bin/bash
# Round 6: confirm QPSK_LATE_YIELD=1 / 2 (5 rounds: K=2 -0.5%, K=4 +-0, K=8 +2.4%), 7 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c21
bash profiles/libs_ab.sh 7 65536 gpurun_out/r6c21/ly2_ab.txt prod $L/lib_ly1.so $L/lib_ly2.so > gpurun_out/r6c21/ly2_ab.log 2>&1
