#!/bin/bash
# Round 6: the thread tests, streams from three host threads included.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_threads.py \
  > gpurun_out/r6c12_pytest.log 2>&1
