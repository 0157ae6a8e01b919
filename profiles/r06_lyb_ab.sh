#!/bin/bash
# Round 6: the 4x2 back at issue priority 1 (above the fronts' late yield to 0,
# below their 2 before it), with the yield over the last 2 or 3 channels,
# against the product, 5 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c42
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c42/lyb_ab.txt prod $L/lib_lyb1.so $L/lib_lyb1k3.so > gpurun_out/r6c42/lyb_ab.log 2>&1
