#!/bin/bash
# dense fp32 AdaGrad / Adam: parity tests, then the c3 secondary lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "updater or adam or adagrad or throughput" > gpurun_out/adam_tests.log 2>&1
rc=$?; tail -2 gpurun_out/adam_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for u in adagrad adam; do
  timeout -k 10 200 python bench.py --workload c3 --updater $u --no-cpu-baseline --secondary= --steps 3 --warmup 1 > gpurun_out/upd_$u.log 2>&1 || exit $?
  python -c "
import json; o=json.loads([l for l in open('gpurun_out/upd_$u.log') if l.startswith('{')][-1])
print('$u', round(o['value']/1e6,1), 'M/s', round(o['roofline']['avg_kernel_ms'],2), 'ms')"
done
