set -o pipefail
timeout -k 10 120 ./profiles/calib/mfma_mix > gpurun_out/mfma_mix3.txt 2>&1
