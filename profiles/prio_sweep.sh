for p in front back none; do QPSK_PRIO=$p timeout -k 10 300 python bench.py --cpu-channels 0 --verify 0 --steps 3 > gpurun_out/prio_$p.log 2>&1 || exit 1; done
