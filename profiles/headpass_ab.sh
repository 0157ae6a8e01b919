#!/bin/bash
# Head pre-pass (head_kernel, then the dual-chain fronts load
# the rt-independent FIR heads) vs the fronts computing them (QPSK_HEADPASS=0),
# at the batch sizes that select the dual-chain shapes.  Repo root, GPU box.
set -o pipefail
one() {  # label, channels, env...
  local lab=$1 nch=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --channels $nch \
    --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $lab', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for rep in 1 2; do
  for nch in 32768 16384 8192 4096 2048; do
    one prepass $nch X=1 || exit 1
    one fronts $nch QPSK_HEADPASS=0 || exit 1
  done
done
