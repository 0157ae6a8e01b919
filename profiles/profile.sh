#!/bin/bash
# Kernel timing + PMC passes for the C3 bench (run on the GPU box from the
# repo root).  Separate rocprofv3 runs: kernel-trace stats, then one counter
# group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   bash profiles/profile.sh TAG [extra bench args]
set -euo pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# provenance of the profiled kernels (summarize.py -> pmc_*.json -> bench.py)
python3 -c "import singlecarrier_amd as sc; print(sc.kernel_hash())" > $OUT/kernel_hash.txt
B="bench.py --steps 5 --warmup 2 --cpu-channels 0 --cpu-all-channels 0 --stream-chunks 0 --frame-latency 0 --verify 0 $*"
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 $B \
    > $OUT/$name.log 2>&1
}
run stats --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS
run lds --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
export QPSK_ABLATE=back; run abl_back --kernel-trace --stats
export QPSK_ABLATE=front; run abl_front --kernel-trace --stats; unset QPSK_ABLATE
echo done > $OUT/DONE
