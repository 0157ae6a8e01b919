#!/bin/bash
# Round 6: role breakdown of the 2x4 dual-chain kernel at 32,768 channels (the
# N = 2 shard) and, for comparison, the 1x8 quad kernel at 8,192 (diagnostic
# build, make stamps; profiles/stamps_dual.py).
set -o pipefail
O=gpurun_out/r6c44
mkdir -p $O
timeout -k 10 300 python profiles/stamps_dual.py 32768 > $O/stamps_32768.txt 2> $O/stamps_32768.err || exit 1
timeout -k 10 300 python profiles/stamps_dual.py 8192 > $O/stamps_8192.txt 2> $O/stamps_8192.err
