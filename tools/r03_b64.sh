#!/bin/bash
# Round 3: chain_block64 with two chain waves -- diagnostics, parity, bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B=tools/chain_bench64
# rows/chain chains d grad upd storage H
step c3_f32_h1 timeout -k 10 60 $B 20000 256 1024 0 0 4 1
step c3_f32_h2 timeout -k 10 60 $B 20000 256 1024 0 0 4 2
step c3_f64_h2 timeout -k 10 60 $B 20000 256 1024 0 0 8 2
step c2_f32_h1 timeout -k 10 60 $B 39062 256 512 1 0 4 1
step c2_f32_h2 timeout -k 10 60 $B 39062 256 512 1 0 4 2
step c3l2_f32_h2 timeout -k 10 60 $B 20000 256 1024 0 1 4 2
step gather timeout -k 10 120 tools/gather_bench 20000 1024
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "block_rows or kernel_selection or stateful_updaters_in_registers or fp32_storage"
step tests2 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 400 --timeout-method thread -k "rccl or c5_1024"
step bench timeout -k 10 400 python -u bench.py --workload c3 --compute f64 --no-cpu-baseline --secondary "c3:f64::f64,c2:f64,c3:f64:adagrad,c3:f64:adam"
