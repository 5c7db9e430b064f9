#!/bin/bash
# c4 (chain_sparse_lds, tail in HBM) cost probes: the product kernel and builds whose tail stores
# (PSGD_LDS_EXP=1), gathers (2) or both (3) touch no memory; chain / loader / tagger stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --secondary= --no-cpu-baseline --workload c4 --steps 2 --warmup 1 --prewarm-s 0.3"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/_run.log | tail -1; grep "psgd stamps" gpurun_out/_run.log | tail -6; [ $rc -eq 0 ] || exit $rc; }
run $B
for e in 1 2 3; do run env PSGD_LIB=$PWD/tools/libpsgd_e$e.so $B; done
export PSGD_STAMPS=1
run $B
for e in 1 2 3; do run env PSGD_LIB=$PWD/tools/libpsgd_e$e.so $B; done
