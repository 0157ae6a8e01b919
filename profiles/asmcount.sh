#!/bin/bash
# Instruction mix of the C3 (4x2) kernel's loops for a variant's -D flags
# (device assembly only, no GPU):  bash profiles/asmcount.sh [-DKNOB=..]
set -eu
cd "$(dirname "$0")/../singlecarrier_amd/csrc"
OUT=$(mktemp /tmp/asmcount.XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math \
  -I../../include -I. -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" --cuda-device-only -S -o $OUT qpsk_rx.hip
python3 ../../profiles/loopstat.py $OUT "${KERN:-rx_kernelILi4ELi2ELi0ELb0ELi64ELb0ELb0E}" | awk '$4 > 800'
rm -f $OUT
