set -o pipefail
timeout -k 10 300 python -u profiles/hunt_h_margin.py > gpurun_out/hunt_h_margin.txt 2>&1
