#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of one c5 chain launch (separate --pmc passes) + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof_c5}
ARGS="--workload c5 --rows ${ROWS:-20000000} --no-cpu-baseline --secondary= --prewarm-s 0.3 --steps 2 --warmup 1"
mkdir -p $OUT
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step trace timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS
step fetch timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS
step write timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 bench.py $ARGS
find $OUT -name "*.csv" | sort
