#!/bin/bash
# chain_split probes: time per sample vs d, chains, and chain_dense (PSGD_SPLIT=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --secondary= --no-cpu-baseline --workload c3 --steps 3 --warmup 1 --prewarm-s 0.3"
run() { echo "== $*"; timeout -k 10 200 "$@" 2>&1 | grep -o '"avg_kernel_ms": [0-9.]*\|"rows_per_gpu": [0-9]*\|"d": [0-9]*\|"chains_per_gpu": [0-9]*' | tr '\n' ' '; rc=${PIPESTATUS[0]}; echo; [ $rc -eq 0 ] || exit $rc; }
run $B --updater adagrad --features 512
run $B --updater adagrad --features 2048
run $B --updater adagrad --chains 512
run $B --updater adagrad --chains 128
run $B --updater adagrad --compute f64 --features 256
PSGD_SPLIT=0 run $B --updater adagrad --features 512
run $B --updater adagrad --rows 2500000
