set -o pipefail
L=singlecarrier_amd/csrc/build
bash profiles/ab.sh 2 $L/lib_cur.so $L/lib_nostore.so > gpurun_out/nostore_ab.txt 2>&1
