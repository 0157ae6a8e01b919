set -o pipefail
# launcher rehearsal on a one-GPU box: two ranks share the GPU (timing is not a
# scaling figure; the check is the spawn, the gloo reduction and per-rank parity)
B="--steps 3 --warmup 1 --cpu-channels 256 --cpu-all-channels 0 --stream-chunks 0"
timeout -k 10 300 python -u bench.py --gpus 2 $B > gpurun_out/r02_launch_n2.json 2> gpurun_out/r02_launch_n2.err &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $B > gpurun_out/r02_torchrun_n2.json 2> gpurun_out/r02_torchrun_n2.err
