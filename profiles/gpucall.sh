set -o pipefail
V=singlecarrier_amd/csrc/build/lib_hvalu.so
QPSK_LIB=$PWD/$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not c_driver" > gpurun_out/c2_pytest_hvalu.log 2>&1 &&
bash profiles/ab.sh 3 singlecarrier_amd/libqpsk_hip.so $PWD/$V > gpurun_out/c2_ab_c3.txt 2>&1 &&
QPSK_LIB=$PWD/$V bash profiles/strong_curve.sh > gpurun_out/c2_curve_hvalu.txt 2>&1 &&
bash profiles/strong_curve.sh > gpurun_out/c2_curve_prod.txt 2>&1
