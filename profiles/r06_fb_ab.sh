#!/bin/bash
# Round 6: the split FIR's LDS batch sizes (QPSK_FB: pass 1, 15; QPSK_FB1: pass 2,
# 8) at C3, variant libraries beside the product, 3 interleaved rounds
# (profiles/libs_ab.sh).  Then one full-kernel parity check of the best
# variants (test_full_size_c3 under QPSK_LIB).
set -o pipefail
L=singlecarrier_amd/csrc/build
mkdir -p gpurun_out/r6c3
bash profiles/libs_ab.sh 3 65536 gpurun_out/r6c3/fb_ab.txt prod $L/lib_fb1_7.so $L/lib_fb1_13.so $L/lib_fb1_25.so \
  $L/lib_fb_20.so $L/lib_fb_30.so $L/lib_fb30_25.so > gpurun_out/r6c3/fb_ab.log 2>&1
