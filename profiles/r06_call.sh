#!/bin/bash
# One GPU call of round 6: the -m gpu suite, the default bench line and the
# rocprofv3 passes of profile.sh, every step under its own time limit; a crash,
# abort or time-out (exit status >= 124) ends the call there.  Outputs go to
# gpurun_out/c<N>_* (suffixed by call number, never overwritten).
#   bash profiles/r06_call.sh N [tests|bench|prof|curve|env]...
set -u
N=$1; shift
O=gpurun_out/r6c${N}
mkdir -p gpurun_out
export TMPDIR=/tmp
check() { # name rc
  echo "[$(date +%T)] $1 rc=$2" >&2
  if [ "$2" -ge 124 ]; then echo "stopping: $1 rc=$2" >&2; exit "$2"; fi
}
for what in "$@"; do
  echo "[$(date +%T)] $what" >&2
  case $what in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 \
             --timeout-method thread > ${O}_pytest.log 2>&1; check pytest $? ;;
    bench) timeout -k 10 400 python bench.py > ${O}_bench.json 2> ${O}_bench.err; check bench $? ;;
    prof)  timeout -k 10 900 bash profiles/profile.sh r06_c${N}; check prof $? ;;
    curve) timeout -k 10 600 bash profiles/ab_shards.sh 1 "65536 32768 16384 8192 4096" singlecarrier_amd/libqpsk_hip.so > ${O}_curve.txt 2>&1; check curve $? ;;
    sweep) timeout -k 10 1100 python bench.py --sweep --cpu-procs 16 > ${O}_sweep.jsonl 2> ${O}_sweep.err; check sweep $? ;;
    env)   { nproc; cat /sys/fs/cgroup/cpu.max; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > ${O}_env.txt 2>&1 ;;
    *) echo "unknown step $what" >&2; exit 2 ;;
  esac
done
