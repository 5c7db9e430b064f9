#!/bin/bash
# chain_block64: updates interleaved into the recurrence (A/B), and the recurrence's share by gradient
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for g in 0 1 2; do
  step "il_grad$g" timeout -k 10 60 tools/chain_bench64_il 20000 256 1024 $g 0 4 2
  step "seq_grad$g" timeout -k 10 60 tools/chain_bench64_seq 20000 256 1024 $g 0 4 2
done
step il_f64rows timeout -k 10 60 tools/chain_bench64_il 20000 256 1024 0 0 8 2
step il_c2 timeout -k 10 60 tools/chain_bench64_il 39062 256 512 1 0 4 2
step il_c2_h1 timeout -k 10 60 tools/chain_bench64_il 39062 256 512 1 0 4 1
