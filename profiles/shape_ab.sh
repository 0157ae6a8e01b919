for r in 1 2; do
for nch in 65536 8192 16384; do for S in 4x2 2x4 1x8; do
QPSK_SHAPE=$S timeout -k 10 300 python bench.py --channels $nch --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 0 --steps 5 --warmup 2 | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$nch $S', d['ms_per_step'], round(d['value']), d['roofline']['kernels_us'])" || exit 1
done; done; done
