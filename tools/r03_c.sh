#!/bin/bash
# Round 3: the short-chain fp64 sigmoid (accuracy + A/B), fp64 AdaGrad/Adam speedups, parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step sigmoid timeout -k 10 60 tools/sigmoid_check
step c3_fast timeout -k 10 60 tools/chain_bench64 20000 256 1024 0 0 4 2
step c3_libm timeout -k 10 60 tools/chain_bench64_roles 20000 256 1024 0 0 4 2
step c3f64_fast timeout -k 10 60 tools/chain_bench64 20000 256 1024 0 0 8 2
step c3l2_fast timeout -k 10 60 tools/chain_bench64 20000 256 1024 0 1 4 2
step parity timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block.py -x -q --timeout 300 --timeout-method thread
step bench timeout -k 10 500 python -u bench.py --workload c3 --compute f64 --no-cpu-baseline --secondary "c3:f64::f64,c3:f64:adagrad,c3:f64:adam,c2:f64"
