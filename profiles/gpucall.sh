set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02_pytest_gpu_v9.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench_v9.json 2> gpurun_out/r02_bench_v9.err &&
bash profiles/profile.sh r02_v9 > gpurun_out/r02_v9_profile.log 2>&1
