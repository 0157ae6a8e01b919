#!/bin/bash
# Round 4, call 29: the 4x3 C3 kernel (rx43_kernel: 4 lane backs + 12 fronts,
# 4 waves per SIMD, roles as separate functions, compact front input): parity
# with QPSK_SHAPE=4x3 (incl. the full C3 size), then an A/B against 4x2 at C3.
# (First try: the role functions read the kernel arguments through the kernarg
# pointer, which a called function does not receive: illegal address; fixed by
# copying the arguments to LDS.)
set -u
O=gpurun_out/r4c29
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "every_workgroup_shape and 4x3" -x -v \
  --timeout 150 --timeout-method thread > ${O}_pytest_shapes.log 2>&1; check pytest_shapes $?
QPSK_SHAPE=4x3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu \
  -k "sample_file or c2_4096 or ragged or edge or streaming_split or full_size_c3 or random_batches or exact_division or long_stream or per_call_job" -x -v \
  --timeout 300 --timeout-method thread > ${O}_pytest_4x3.log 2>&1; check pytest_4x3 $?
timeout -k 10 400 bash profiles/knob_ab.sh 2 65536 QPSK_SHAPE=4x2 QPSK_SHAPE=4x3 > ${O}_ab.txt 2>&1; check ab $?
