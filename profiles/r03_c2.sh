#!/bin/bash
# call 2: early-decision protocol -- parity subset, then A/B against HEAD~ (lib_base)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_dec752.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/c2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 bash profiles/ab_shards.sh 2 "65536 32768 16384 8192" singlecarrier_amd/csrc/build/lib_base.so singlecarrier_amd/libqpsk_hip.so > gpurun_out/c2_ab.txt 2>&1
echo "ab rc=$?" >&2
