#!/bin/bash
# chain microbenchmark over build variants: VARIANTS="d0 d1" CFGS="512,1 512,0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in $VARIANTS; do for cfg in $CFGS; do
  IFS=, read d g u <<< "$cfg"
  echo "== $b d=$d grad=$g upd=${u:-0}"; timeout -k 10 60 tools/$b 39062 256 $d $g ${u:-0} || exit $?
done; done
