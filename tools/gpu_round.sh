#!/bin/bash
# One GPU-box session: parity tests, then a short bench. Stops at the first GPU fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q --timeout=300 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -20 gpurun_out/bench.log
  exit $brc
fi
exit $rc
