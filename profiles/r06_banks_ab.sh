#!/bin/bash
# Round 6, item 1: the split FIR's LDS bank mapping (QPSK_SPLIT_BANKS) against
# the round-5 mapping, on one box: the parity tests that cover the split FIR,
# then 3 interleaved rounds of C3 (whole kernel, verified; fronts alone), then
# one rocprofv3 LDS counter pass per library.
#   bash profiles/r06_banks_ab.sh OUTDIR LIB_A LIB_B   ("prod" = the product library)
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  -k "split_fir or full_size_c3 or every_workgroup or synth_goldens or sample_file" > $OUT/pytest.log 2>&1 || exit 1
B="bench.py --channels 65536 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --steps 5 --warmup 2"
for r in 1 2 3; do
  for lib in "$@"; do
    L=$lib; [ "$lib" = prod ] && L=
    for abl in none front; do
      if [ $abl = none ]; then V="--verify 64"; E=; else V="--verify 0"; E=QPSK_ABLATE=front; fi
      env ${L:+QPSK_LIB=$L} $E timeout -k 10 300 python $B $V > $OUT/run.json 2>$OUT/run.err || exit 1
      python -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print('$r', '$(basename $lib)', '$abl', d['ms_per_step'], d['roofline']['kernels_us'], d.get('verified_vs_oracle'))" || exit 1
    done
  done
done | tee $OUT/ab.txt || exit 1
for lib in "$@"; do
  L=$lib; [ "$lib" = prod ] && L=
  n=$(basename $lib .so)
  env ${L:+QPSK_LIB=$L} timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU \
    --output-format csv -d $OUT/lds_$n -o lds -- python3 $B --verify 0 > $OUT/lds_$n.log 2>&1 || exit 1
done
echo done > $OUT/DONE
