#!/bin/bash
# chain_split with 2 compute waves (PSGD_SPLIT_HMAX=2 build) against the default 4 at c3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --secondary= --no-cpu-baseline --workload c3 --steps 3 --warmup 1"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*\|"kernel": "[^"(]*' gpurun_out/_run.log | tail -2 | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc; }
for lib in "" "PSGD_LIB=$PWD/tools/libpsgd_h2.so"; do
  for u in adagrad adam; do for c in f32 f64; do run env $lib $B --updater $u --compute $c; done; done
done
