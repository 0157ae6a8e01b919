set -o pipefail
L=singlecarrier_amd/csrc/build
bash profiles/ab.sh 2 $L/lib_hf1.so $L/lib_sch_dflt.so $L/lib_sch_maxilp.so $L/lib_sch_lowocc.so > gpurun_out/sched2_ab.txt 2>&1 &&
for r in 1 2; do for lib in hf1 sch_dflt sch_maxilp sch_lowocc; do
  QPSK_LIB=$L/lib_$lib.so timeout -k 10 300 python bench.py --channels 8192 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 10 --warmup 2 \
   | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('8192 $lib', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" >> gpurun_out/sched2_ab.txt || exit 1
done; done
