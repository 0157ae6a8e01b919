set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu_v8.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench_v8.json 2> gpurun_out/r02_bench_v8.err &&
bash profiles/profile.sh r02_v8 > gpurun_out/r02_v8_profile.log 2>&1
