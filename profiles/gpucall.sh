set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dec752.py -k "low_amplitude" -x -q --timeout 120 --timeout-method thread > gpurun_out/lowamp2.log 2>&1
