set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "speculative or dual_chain or quad or progress" > gpurun_out/c5_pytest.log 2>&1 &&
bash profiles/knob_ab.sh 2 8192 "QPSK_SPEC=0 QPSK_ISO=0" "QPSK_SPEC=0 QPSK_ISO=1" "QPSK_SPEC=1 QPSK_ISO=1" > gpurun_out/c5_iso_ab.txt 2>&1 &&
bash profiles/knob_ab.sh 2 4096 "QPSK_SPEC=0 QPSK_ISO=0" "QPSK_SPEC=0 QPSK_ISO=1" "QPSK_SPEC=1 QPSK_ISO=1" >> gpurun_out/c5_iso_ab.txt 2>&1
