set -o pipefail
timeout -k 10 120 python -u profiles/stamps_lp.py 65536 > gpurun_out/c15_stamps_lp.txt 2>&1 &&
timeout -k 10 120 python -u profiles/stamps_lp.py 16384 >> gpurun_out/c15_stamps_lp.txt 2>&1
