set -o pipefail
# default bench line (N = 1), then the N = 2 launcher rehearsal (two ranks on
# the one GPU: not a scaling figure)
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench_v6.json 2> gpurun_out/r02_bench_v6.err &&
timeout -k 10 300 python -u bench.py --gpus 2 --cpu-channels 256 --cpu-all-channels 0 --stream-chunks 0 > gpurun_out/r02_launch_n2.json 2> gpurun_out/r02_launch_n2.err
