#!/bin/bash
# chain_block64: row reads issued before the conversions (CONV1) vs converted at use (c0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for g in 0 1; do
  step "conv1_grad$g" timeout -k 10 60 tools/chain_bench64 20000 256 1024 $g 0 4 2
  step "c0_grad$g" timeout -k 10 60 tools/chain_bench64_c0 20000 256 1024 $g 0 4 2
done
step conv1_c2 timeout -k 10 60 tools/chain_bench64 39062 256 512 1 0 4 2
step c0_c2 timeout -k 10 60 tools/chain_bench64_c0 39062 256 512 1 0 4 2
step c2_h1 timeout -k 10 60 tools/chain_bench64 39062 256 512 1 0 4 1
step f64rows timeout -k 10 60 tools/chain_bench64 20000 256 1024 0 0 8 2
