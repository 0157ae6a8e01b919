set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c11_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r6c11_bench.json 2> gpurun_out/r6c11_bench.err
