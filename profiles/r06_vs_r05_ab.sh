#!/bin/bash
# Round 6 against round 5 on one box: the product (round 6's final tree) and
# round 5's final qpsk_rx.hip (commit dca1c5f, hash 6e637a89 as shipped; built
# beside the product with a no-op qpsk_rx_mark_stalled, the one symbol round
# 6's stream code adds), 7 interleaved rounds at C3 (verified), then 3 of the
# fronts alone (QPSK_ABLATE=front) and 2 of the C4 shard sizes.
set -o pipefail
L=singlecarrier_amd/csrc/build
O=gpurun_out/r6c18
mkdir -p $O
bash profiles/libs_ab.sh 7 65536 $O/c3.txt prod $L/lib_r05final.so > $O/c3.log 2>&1 || exit 1
B="bench.py --channels 65536 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --steps 5 --warmup 2 --verify 0"
for r in 1 2 3; do
  for lib in prod $L/lib_r05final.so; do
    Lb=$lib; [ "$lib" = prod ] && Lb=
    env ${Lb:+QPSK_LIB=$Lb} QPSK_ABLATE=front timeout -k 10 300 python $B > $O/f.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/f.json').read().strip().splitlines()[-1]); print('front', '$(basename $lib)', d['ms_per_step'], d['roofline']['kernels_us'])" || exit 1
  done
done > $O/fronts.txt
bash profiles/ab_shards.sh 2 "32768 16384 8192 4096" singlecarrier_amd/libqpsk_hip.so $L/lib_r05final.so 2>/dev/null > $O/shards.txt
