#!/bin/bash
# Round 6: the 4x2 back wave (the frame's last wave) at the highest issue
# priority from training step S on (QPSK_BACK_BOOST = 96 / 112 / 120), on top
# of the fronts' late yield, 5 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c24
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c24/bb_ab.txt prod $L/lib_bb96.so $L/lib_bb112.so $L/lib_bb120.so > gpurun_out/r6c24/bb_ab.log 2>&1
