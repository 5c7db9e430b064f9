#!/bin/bash
# chain_split: its GPU tests, then the four c3 stateful lines (kernel ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
B="python bench.py --secondary= --no-cpu-baseline --workload c3 --steps 3 --warmup 1"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/_run.log | tail -1; [ $rc -eq 0 ] || exit $rc; }
for u in adagrad adam; do for c in f32 f64; do run $B --updater $u --compute $c; done; done
