#!/bin/bash
# quad vs lane backs at the C4 shard sizes that use the dual-chain kernel
set -o pipefail
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --channels $NCH --cpu-channels 0 --cpu-all-channels 0 \
    --stream-chunks 0 --verify 64 --steps 5 --warmup 2 \
    | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$NCH $label', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'], d['verified_vs_oracle'])"
}
for NCH in 4096 8192; do
  run lane QPSK_QUAD=0 || exit 1
  run quad QPSK_QUAD=1 || exit 1
done
