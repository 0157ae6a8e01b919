set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "low_amplitude or edge_inputs" -x -q --timeout 120 --timeout-method thread > gpurun_out/lowamp.log 2>&1
