#!/bin/bash
# chain_sparse_lds with 32-bit row bookkeeping: sparse / config GPU tests, then the c4 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
B="python bench.py --secondary= --no-cpu-baseline --workload c4 --steps 3 --warmup 1"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/_run.log | tail -1; [ $rc -eq 0 ] || exit $rc; }
run $B --compute f32
run $B --compute f64
