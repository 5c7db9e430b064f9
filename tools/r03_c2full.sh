#!/bin/bash
# C2 full-geometry parity test, then the c1 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_full.py -m gpu -x -v --timeout 380 --timeout-method thread 2>&1 | tail -5
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
bash tools/profile_r03.sh c1
