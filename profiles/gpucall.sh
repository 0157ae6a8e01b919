set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/c17_pytest.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/c17_bench.json 2> gpurun_out/c17_bench.err &&
bash profiles/strong_curve.sh > gpurun_out/c17_curve.txt 2>&1
