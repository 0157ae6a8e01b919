#!/bin/bash
# Round 6: with the anchored FIR the 4x2 back wave is the frame's last wave
# (4.4% tail, r06_c19_stamps).  QPSK_LATE_YIELD=K: the fronts run their last K
# channels of each frame at the back's issue priority.  5 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c20
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c20/ly_ab.txt prod $L/lib_ly2.so $L/lib_ly4.so $L/lib_ly8.so > gpurun_out/r6c20/ly_ab.log 2>&1
