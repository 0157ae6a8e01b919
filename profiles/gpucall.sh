set -o pipefail
L=singlecarrier_amd/csrc/build
bash profiles/ab.sh 3 $L/lib_bb0.so $L/lib_bb64.so $L/lib_bb96.so $L/lib_bb112.so > gpurun_out/boost_ab.txt 2>&1
