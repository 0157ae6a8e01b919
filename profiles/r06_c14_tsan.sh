#!/bin/bash
# Round 6: the thread tests with the ThreadSanitizer build of the host code
# (tests/callers/Makefile tsan, prebuilt on the CPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 700 --timeout-method thread tests/test_gpu_threads.py \
  > gpurun_out/r6c14_pytest.log 2>&1
