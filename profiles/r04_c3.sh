#!/bin/bash
# Round 4, call 3: the quad step rewrite (packed d, ring window, preamble from
# scalar loads, one range check per frame) -- parity of the quad shapes and the
# fixed stream/bench paths, A/B against HEAD's kernels (lib_base.so) at the
# quad shards and 16,384, and back-step stamps at 8,192 with fronts on/idle.
set -u
O=gpurun_out/r4c3
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_bench.py \
  -k "quad or c4_shards or dual_chain or stream or bench or exact or c2 or sample" -v --timeout 200 \
  --timeout-method thread > ${O}_pytest.log 2>&1; check pytest $?
timeout -k 10 400 bash profiles/ab_shards.sh 2 "4096 8192 16384" singlecarrier_amd/csrc/build/lib_base.so \
  singlecarrier_amd/libqpsk_hip.so > ${O}_ab.txt 2>&1; check ab $?
timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192.txt 2>&1; check stamps $?
QPSK_ABLATE=frontidle timeout -k 10 120 python profiles/stamps_dual.py 8192 > ${O}_stamps_8192_idle.txt 2>&1; check idle $?
