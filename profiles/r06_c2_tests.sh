#!/bin/bash
# Round 6: the new state / thread tests (+ the stream, stall and snapshot tests
# they touch), then the C3 stamps run (profiles/r06_stamps.sh).
set -o pipefail
mkdir -p gpurun_out/r6c2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_state.py \
  tests/test_gpu_threads.py tests/test_gpu_stream.py tests/test_gpu_parity.py \
  -k "state or thread or stream or stall or independent" > gpurun_out/r6c2/pytest.log 2>&1 || exit 1
bash profiles/r06_stamps.sh gpurun_out/r6c2
