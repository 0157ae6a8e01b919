set -o pipefail
L=singlecarrier_amd/csrc/build
bash profiles/ab.sh 3 $L/lib_cur.so $L/lib_dm3.so $L/lib_dm4.so $L/lib_dm0.so > gpurun_out/dmin_ab.txt 2>&1
