#!/bin/bash
# Profiles of the bench workload for profiles/ (run on the GPU box through gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc runs; MI355X_MICROARCH.md §HBM)
#   4. SQ instruction-mix pass (VALU vs MFMA vs LDS instructions)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
# the bench defaults (5 timed steps, 2 warmup), headline workload only (no secondary lines)
ARGS="--secondary= ${BENCH_ARGS:---no-cpu-baseline}"
mkdir -p $OUT
# one rank only: bench.py --gpus N > 1 would start a launcher under the profiler
case " $ARGS " in *" --gpus "[2-9]*|*" --gpus="[2-9]*) echo "profile a single rank (--gpus 1)"; exit 2;; esac
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step trace timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS
step fetch timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS
step write timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 bench.py $ARGS
step insts timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES -f csv -d $OUT/insts -o run -- python3 bench.py $ARGS
find $OUT -name "*.csv" | sort
