set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu_v5.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r02_bench_v5.json 2> gpurun_out/r02_bench_v5.err &&
bash profiles/profile.sh r02_v5 > gpurun_out/r02_v5_profile.log 2>&1
