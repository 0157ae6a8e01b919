set -o pipefail
L=singlecarrier_amd/csrc/build
bash profiles/ab.sh 3 $L/lib_hf1.so $L/lib_st0.so $L/lib_st6.so $L/lib_st20.so > gpurun_out/stagger2_ab.txt 2>&1
