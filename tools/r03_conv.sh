#!/bin/bash
# chain_split with the per-sample convergence test: the GPU suite, then the c3 lines with tol > 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -15
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -m gpu -q -s -k "convergence and logistic and simple" 2>&1 | tail -5
