#!/bin/bash
# Round 6: confirm QPSK_FB=20 (pass 1 in 3 LDS batches: 20, 20, 19) against the
# product (15: 15, 15, 15, 14), with pass 2 at 8 / 13 / 7, 5 interleaved rounds at C3.
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c4
bash profiles/libs_ab.sh 5 65536 gpurun_out/r6c4/fb20_ab.txt prod $L/lib_fb_20.so $L/lib_fb20_13.so $L/lib_fb20_7.so \
  > gpurun_out/r6c4/fb20_ab.log 2>&1
