#!/bin/bash
# chain_sparse_lds: sparse GPU tests, then c4 stamps (4M rows) and the full c4 shard
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lds_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lds_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
VARIANTS=lds bash tools/exp_gram.sh || exit $?
timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --secondary= --steps 5 --warmup 2 > gpurun_out/lds_c4_full.log 2>&1 || exit $?
python -c "
import json; o=json.loads([l for l in open('gpurun_out/lds_c4_full.log') if l.startswith('{')][-1])
print('c4 full', round(o['value']/1e6,1), 'M/s', round(o['roofline']['avg_kernel_ms'],3), 'ms')"
