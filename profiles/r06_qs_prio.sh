#!/bin/bash
# Round 6: QPSK_QSPLIT's equalizer waves at issue priority 2 / 1 / 0 against
# HEAD, 2 interleaved rounds at 8,192 channels.
set -o pipefail
L=singlecarrier_amd/csrc/build
O=gpurun_out/r6c33
mkdir -p $O
bash profiles/libs_ab.sh 2 8192 $O/qs_prio_ab.txt $L/lib_head.so $L/lib_qs.so $L/lib_qsp1.so $L/lib_qsp0.so > $O/qs_prio_ab.log 2>&1
