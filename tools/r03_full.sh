#!/bin/bash
# Full GPU suite + smoke + the default bench line (what the driver runs at round end).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step smoke timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
