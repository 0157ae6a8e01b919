#!/bin/bash
# Round 6: the lane back's packed Newton steps again, on the final tree (the
# back is the frame's last wave since the anchoring; late yield in both arms),
# 7 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c25
bash profiles/libs_ab.sh 7 65536 gpurun_out/r6c25/rp2_ab.txt prod $L/lib_rp2.so > gpurun_out/r6c25/rp2_ab.log 2>&1
