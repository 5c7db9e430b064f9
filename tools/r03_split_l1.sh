#!/bin/bash
# chain_split with L1: GPU tests of the split / stateful paths, then the c3 L1 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or stateful or throughput_updaters" 2>&1 | tail -3
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
B="python bench.py --secondary= --no-cpu-baseline --workload c3 --steps 3 --warmup 1"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*\|"kernel": "[^"(]*' gpurun_out/_run.log | tail -2 | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc; }
run $B --updater l1 --compute f32
run $B --updater l1 --compute f64
PSGD_SPLIT=0 run $B --updater l1 --compute f32
