set -o pipefail
QPSK_ESPLIT=1 QPSK_WIDTH=64 timeout -k 10 120 python -u profiles/lp_check.py > gpurun_out/c20_es_check.txt 2>&1 &&
QPSK_ESPLIT=1 QPSK_WIDTH=64 QPSK_FORCE_EXACT=1 timeout -k 10 120 python -u profiles/lp_check.py >> gpurun_out/c20_es_check.txt 2>&1 &&
bash profiles/knob_ab.sh 2 16384 QPSK_ESPLIT=0 QPSK_ESPLIT=1 > gpurun_out/c20_es_ab.txt 2>&1
