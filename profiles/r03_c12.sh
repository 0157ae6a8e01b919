#!/bin/bash
# call 12: stamps of the 16,384- and 32,768-channel shards (lane backs)
set -u
export TMPDIR=/tmp
timeout -k 10 120 python profiles/stamps_dual.py 16384 > gpurun_out/r3c12_stamps16384.txt 2>&1; echo "rc=$?" >&2
QPSK_PRIO=front timeout -k 10 120 python profiles/stamps_dual.py 16384 > gpurun_out/r3c12_stamps16384_front.txt 2>&1; echo "rc=$?" >&2
timeout -k 10 120 python profiles/stamps_dual.py 32768 > gpurun_out/r3c12_stamps32768.txt 2>&1; echo "rc=$?" >&2
