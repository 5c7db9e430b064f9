#!/bin/bash
# chain_split (AdaGrad / Adam feature-split chain): parity tests, then the c3 stateful bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
for u in adagrad adam; do
  for c in f32 f64; do
    step "bench c3 $c $u" timeout -k 10 300 python bench.py --secondary= --no-cpu-baseline --workload c3 --compute $c --updater $u --steps 3 --warmup 1
  done
done
