#!/bin/bash
# Round 3: wave placement, the c5 request ceiling, the fp64 CSR kernel, the RCCL leg, C5 at 1,024
# chains, bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step placement timeout -k 10 60 tools/wave_placement 256
step roles_c3 timeout -k 10 60 tools/chain_bench64_roles 20000 256 1024 0 0 4 2
step roles_c3_f64 timeout -k 10 60 tools/chain_bench64_roles 20000 256 1024 0 0 8 2
step roles_c2 timeout -k 10 60 tools/chain_bench64_roles 39062 256 512 1 0 4 2
step roles_c2_h1 timeout -k 10 60 tools/chain_bench64_roles 39062 256 512 1 0 4 1
step gather timeout -k 10 300 tools/gather_bench 20000 1024
step sparse64 timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread -k "fp64"
step alpha timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "alpha_scaled or csr"
step configs timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 500 --timeout-method thread -k "rccl or c5_1024 or c4_rcv1_shape_fp64"
step bench timeout -k 10 500 python -u bench.py --workload c4 --compute f64 --no-cpu-baseline --secondary "c3:f64,c3:f64::f64,c2:f64,c3:f64:adagrad,c3:f64:adam"
