set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02_pytest_gpu_final.log 2>&1
