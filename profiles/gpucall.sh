set -o pipefail
timeout -k 10 900 python -u bench.py --sweep > gpurun_out/c19_sweep.jsonl 2> gpurun_out/c19_sweep.err
