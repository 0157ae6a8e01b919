#!/bin/bash
# Round 6: QPSK_QSPLIT (qs2) against the same with static priorities (gain
# waves 2, fronts 0, equalizer waves 0: QPSK_DYNPRIO=0 with QPSK_PRIO=2, qs3),
# and HEAD (QPSK_PRIO=2 leaves the dynamic-priority kernels unchanged),
# 3 interleaved rounds at 8,192 channels.
set -o pipefail
L=singlecarrier_amd/csrc/build
O=gpurun_out/r6c35
mkdir -p $O
QPSK_PRIO=2 bash profiles/libs_ab.sh 3 8192 $O/qs3_ab.txt $L/lib_head.so $L/lib_qs2.so $L/lib_qs3.so > $O/qs3_ab.log 2>&1
