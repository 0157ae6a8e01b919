set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_hunt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hunt_test.log 2>&1 &&
timeout -k 10 300 python -u profiles/hunt_fallback.py > gpurun_out/hunt_fallback.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 > gpurun_out/filt_bench2.json 2> gpurun_out/filt_bench2.err
