set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "every_workgroup_shape" > gpurun_out/c8_pytest.log 2>&1 &&
bash profiles/knob_ab.sh 3 65536 QPSK_SHAPE=4x2 QPSK_SHAPE=4x2l > gpurun_out/c8_ls_ab.txt 2>&1
