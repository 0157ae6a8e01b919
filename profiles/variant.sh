#!/bin/bash
# Build a variant of the receive library from another qpsk_rx.hip source (A/B
# experiments only; the product is singlecarrier_amd/libqpsk_hip.so).
#   bash profiles/variant.sh NAME path/to/qpsk_rx.hip [extra hipcc flags]
set -euo pipefail
SCHED=${SCHED-iterative-ilp}   # machine scheduler; SCHED= for the default one
NAME=$1; SRC=$(realpath $2); shift 2
cd "$(dirname "$0")/../singlecarrier_amd/csrc"
make -s build/qpsk_surface.o build/qpsk_synth.o build/qpsk_synth_dev.o build/qpsk_stream.o build/qpsk_fft.o build/qpsk_fft_host.o build/qpsk_records.o
cp "$SRC" build/_variant_$NAME.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math \
  -I../../include -I. ${SCHED:+-mllvm -amdgpu-sched-strategy=$SCHED} "$@" \
  -c -o build/_variant_$NAME.o build/_variant_$NAME.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/lib_$NAME.so build/_variant_$NAME.o \
  build/qpsk_surface.o build/qpsk_synth.o build/qpsk_synth_dev.o build/qpsk_stream.o \
  build/qpsk_fft.o build/qpsk_fft_host.o build/qpsk_records.o -lm -lpthread
echo singlecarrier_amd/csrc/build/lib_$NAME.so
