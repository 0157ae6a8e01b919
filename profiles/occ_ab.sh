#!/bin/bash
# C3 occupancy A/B: the 4x2 front at 2 vs 3 front
# waves per SIMD with the SAME front body.  The unchanged body (11.1 KB of M +
# two dec buffers per front) does not fit 12 fronts into one CU's LDS (190 KB
# > 160 KB), so both arms use the compact front input (item_c: 9.1 KB) with one
# dec buffer -- the only change to the front's instruction stream is the
# mixer's item map (569 items instead of 696) and the first channel's prefetch
# after the frame barrier:
#   prod      the product library (4x2)
#   ab1       QPSK_FRONT_AB=1: 4x2 with the compact front (output exact: verified)
#   prod_f    product, QPSK_ABLATE=front (8 fronts, 2/SIMD; back waves idle)
#   ab1_f     ab1, QPSK_ABLATE=front (8 compact fronts, 2/SIMD)
#   ab2       QPSK_FRONT_AB=2: 12 compact fronts, 3/SIMD, no back waves
# Timing: bench.py's HIP events, R interleaved rounds; then one rocprofv3
# counter pass per arm (LDS and wait counters).
# The A/B kernels live in commit 868e9f0 (moved out of the product source after
# the A/B); build the two variant libraries from it first:
#   bash profiles/build_variant.sh ab1 868e9f0 -DQPSK_FRONT_AB=1
#   bash profiles/build_variant.sh ab2 868e9f0 -DQPSK_FRONT_AB=2
#   bash profiles/occ_ab.sh R TAG
set -o pipefail
R=${1:-3}; TAG=${2:-occ}
L=singlecarrier_amd/csrc/build
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
arms=("prod::" "ab1:$L/lib_ab1.so:" "prod_f::QPSK_ABLATE=front" "ab1_f:$L/lib_ab1.so:QPSK_ABLATE=front" "ab2:$L/lib_ab2.so:")
B="bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --steps 5 --warmup 2"
for r in $(seq 1 $R); do
  for a in "${arms[@]}"; do
    IFS=: read name lib kv <<< "$a"
    ver=0; [ -z "$kv" ] && [ "$name" != ab2 ] && ver=64
    env ${lib:+QPSK_LIB=$lib} $kv timeout -k 10 300 python $B --verify $ver \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['roofline']['kernels_us'], d['verified_vs_oracle'])" \
      || exit 1
  done
done | tee $OUT/timing.txt
PMC="SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU"
for a in "${arms[@]}"; do
  IFS=: read name lib kv <<< "$a"
  env ${lib:+QPSK_LIB=$lib} $kv timeout -k 10 120 rocprofv3 --kernel-trace --pmc $PMC --output-format csv \
    -d $OUT/pmc_$name -o pmc -- python3 $B --verify 0 > $OUT/pmc_$name.log 2>&1 || exit 1
done
echo done > $OUT/DONE
