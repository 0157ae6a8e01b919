#!/bin/bash
# Round 4, call 21: speculative fronts (QPSK_SPEC=1, dual-chain kernels): the
# whole -m gpu suite on the new default, then an A/B at the dual-chain shard
# sizes against HEAD's kernels (lib_base.so) and the same tree without
# speculation (lib_nospec.so, -DQPSK_SPEC=0).
set -u
O=gpurun_out/r4c21
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { echo "[$(date +%T)] $1 rc=$2" >&2; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > ${O}_pytest.log 2>&1; check pytest $?
timeout -k 10 500 bash profiles/ab_shards.sh 2 "4096 8192 16384 32768" singlecarrier_amd/csrc/build/lib_base.so \
  singlecarrier_amd/csrc/build/lib_nospec.so singlecarrier_amd/libqpsk_hip.so > ${O}_ab.txt 2>&1; check ab $?
