#!/bin/bash
# Builds the round-4 probes (run from anywhere; outputs next to this script):
#   simd_probe      which SIMD each wave of a workgroup lands on (HW_ID)
#   fir_probe       fir_dec / fir_head issue rates at 1..4 waves per SIMD, the
#                   product source's FIRs as they are (QPSK_FIR_WAIT default)
#   fir_probe_h15   the same with the batch waits forced on (-DQPSK_FIR_WAIT=1)
# Add -DQPSK_FIR_WAIT=0 to compare with the per-sample waits.
set -eu
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
B=../../singlecarrier_amd/csrc/build
make -s -C ../../singlecarrier_amd/csrc >/dev/null
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
 -I../../include -I../../singlecarrier_amd/csrc -mllvm -amdgpu-sched-strategy=iterative-ilp"
$H --offload-arch=gfx950 -O2 -o simd_probe simd_probe.hip
$H $F -c -o /tmp/fir_probe.o fir_probe.hip
$H --offload-arch=gfx950 -o fir_probe /tmp/fir_probe.o $B/qpsk_fft_host.o $B/qpsk_fft.o -lm -lpthread
$H $F -DQPSK_FIR_WAIT=1 -c -o /tmp/fir_probe_h15.o fir_probe.hip
$H --offload-arch=gfx950 -o fir_probe_h15 /tmp/fir_probe_h15.o $B/qpsk_fft_host.o $B/qpsk_fft.o -lm -lpthread
