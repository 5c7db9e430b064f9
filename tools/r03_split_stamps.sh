#!/bin/bash
# chain_split: GPU tests, per-phase cycle stamps (diagnostic library, PSGD_STAMPS=1) and the c3
# AdaGrad / Adam lines (fp32 / fp64).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or stateful or throughput_updaters" 2>&1 | tail -3
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
B="python bench.py --secondary= --no-cpu-baseline --workload c3 --steps 3 --warmup 1"
run() { echo "== $*"; timeout -k 10 200 "$@" > gpurun_out/_run.log 2>&1; rc=$?; grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/_run.log | tail -1; grep "psgd stamps" gpurun_out/_run.log | tail -16; [ $rc -eq 0 ] || exit $rc; }
for u in adagrad adam; do for c in f32 f64; do run $B --updater $u --compute $c; done; done
export PSGD_STAMPS=1 PSGD_LIB=$PWD/tools/libpsgd_stamps.so
run $B --rows 2500000 --updater adagrad
run $B --rows 2500000 --updater adagrad --compute f64
