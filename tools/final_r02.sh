#!/bin/bash
# round-2 close-out: the default bench (as the driver runs it), then c4 rocprof trace + PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_default.log; echo
[ $rc -eq 0 ] || exit $rc
PROF_OUT=gpurun_out/prof_c4 BENCH_ARGS="--workload c4 --no-cpu-baseline" bash tools/profile_round.sh > gpurun_out/prof_c4.log 2>&1
rc=$?; tail -5 gpurun_out/prof_c4.log; exit $rc
