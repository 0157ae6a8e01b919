#!/bin/bash
# Build an A/B variant of libqpsk_hip.so whose receive kernels come from another
# revision of qpsk_rx.hip (or extra -D knobs), next to the product library.
# Every other object is the product's.  The variant carries its own kernel hash
# ("variant-<name>"), never the product's (bench.pmc_record drops its counters).
#   bash profiles/build_variant.sh NAME REV [-DKNOB=..]     REV: a git revision or "work"
# Output: singlecarrier_amd/csrc/build/lib_NAME.so
set -eu
NAME=$1; REV=$2; shift 2
cd "$(dirname "$0")/../singlecarrier_amd/csrc"
make -s >/dev/null
B=build
if [ "$REV" = work ]; then cp qpsk_rx.hip $B/_variant_$NAME.hip
else git show "$REV:singlecarrier_amd/csrc/qpsk_rx.hip" > $B/_variant_$NAME.hip; fi
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
 -fno-gpu-flush-denormals-to-zero -fno-fast-math -I../../include -I. -mllvm -amdgpu-sched-strategy=iterative-ilp"
$HIPCC $FLAGS "$@" -DQPSK_KERNEL_HASH="\"variant-$NAME\"" -c -o $B/_variant_$NAME.o $B/_variant_$NAME.hip
OBJ="$B/qpsk_surface.o $B/qpsk_synth.o $B/qpsk_synth_dev.o $B/qpsk_stream.o $B/qpsk_records.o $B/qpsk_fft.o $B/qpsk_fft_host.o"
$HIPCC --offload-arch=gfx950 -shared -fPIC -o $B/lib_$NAME.so $B/_variant_$NAME.o $OBJ -lm -lpthread
echo "$B/lib_$NAME.so"
