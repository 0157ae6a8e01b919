set -o pipefail
timeout -k 10 120 ./profiles/calib/mfma_mix > gpurun_out/mfma_mix2.txt 2>&1 &&
bash profiles/profile.sh r02s3 && echo profiled
