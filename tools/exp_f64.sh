#!/bin/bash
# GPU suite, then fp64 parity-mode bench lines (c3 shard, c2, c1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for w in c3 c2 c1; do
  timeout -k 10 200 python bench.py --workload $w --compute f64 --no-cpu-baseline --secondary= --steps 10 --warmup 2 > gpurun_out/f64_$w.log 2>&1 || exit $?
  python -c "
import json; o=json.loads([l for l in open('gpurun_out/f64_$w.log') if l.startswith('{')][-1])
print('$w f64', round(o['value']/1e6,1), 'M/s', round(o['roofline']['frac'],3), o['roofline']['kernel'][:30], round(o['roofline']['avg_kernel_ms'],3))"
done
