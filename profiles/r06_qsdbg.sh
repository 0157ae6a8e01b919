#!/bin/bash
# Round 6: where QPSK_QSPLIT's W = 32 kernel stalls (diagnostic build printing
# the timed-out wait's LDS counter), one small ragged call.
set -o pipefail
mkdir -p gpurun_out/r6c29
QPSK_LIB=singlecarrier_amd/csrc/build/lib_qsdbg.so QPSK_WIDTH=32 timeout -k 10 120 python -c "
import oracle, singlecarrier_amd as sc
x = oracle.synth(64, 333, 15, 4.0)
try:
    sc.Receiver(333).demod(x)
    print('no stall')
except Exception as e:
    print('error', e)
" > gpurun_out/r6c29/dbg.txt 2>&1
