#!/bin/bash
# c4: speculation depth SK = 4 vs 8 (PSGD_SPARSE_SK) for fp32 and fp64, with wave stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --secondary= --no-cpu-baseline --workload c4 --steps 2 --warmup 1 --prewarm-s 0.3"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/_run.log | tail -1; grep "psgd stamps" gpurun_out/_run.log | tail -6; [ $rc -eq 0 ] || exit $rc; }
for sk in 4 8; do for c in f32 f64; do run env PSGD_SPARSE_SK=$sk $B --compute $c; done; done
export PSGD_STAMPS=1
run env PSGD_SPARSE_SK=4 $B --compute f64
run env PSGD_SPARSE_SK=8 $B --compute f64
