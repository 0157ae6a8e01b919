#!/bin/bash
# Round 4, call 1: instruction-cost calibration for the quad Kalman step
# (calib/dpp_rate) and the back-step stamps at the N = 8 shard, with the
# fronts working and with them idle (QPSK_ABLATE=frontidle), on HEAD.
set -u
O=gpurun_out/r4c1
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 120 ./profiles/calib/dpp_rate > ${O}_dpp.txt 2>&1; check dpp $?
timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192.txt 2>&1; check stamps8192 $?
QPSK_ABLATE=frontidle timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192_idle.txt 2>&1; check idle8192 $?
QPSK_ABLATE=frontidle timeout -k 10 120 python profiles/stamps_dual.py 4096 > ${O}_stamps_4096_idle.txt 2>&1; check idle4096 $?
