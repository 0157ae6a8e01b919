for r in 1 2; do for P in front back none; do
QPSK_PRIO=$P timeout -k 10 300 python bench.py --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --verify 0 --steps 5 --warmup 2 | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$P', d['ms_per_step'], d['roofline']['kernels_us'])" || exit 1
done; done
