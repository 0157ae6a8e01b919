set -o pipefail
timeout -k 10 1000 python -u bench.py --sweep > gpurun_out/r02_awgn_sweep_v5.jsonl 2> gpurun_out/r02_awgn_sweep_v5.err
