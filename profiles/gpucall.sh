set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/filt_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 > gpurun_out/filt_bench.json 2> gpurun_out/filt_bench.err &&
for n in 8192 16384 32768; do timeout -k 10 300 python bench.py --channels $n --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 > gpurun_out/filt_$n.json 2>/dev/null || exit 1; done
