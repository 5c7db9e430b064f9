#!/bin/bash
# GPU suite + smoke + the default bench line (what the driver runs at round end), logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
step smoke timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 400 python bench.py
