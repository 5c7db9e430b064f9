#!/bin/bash
# Bench variants in one GPU session: each line of $SWEEP is "ENV=... ENV2=... -- bench args".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra CASES <<< "$SWEEP"
for c in "${CASES[@]}"; do
  envs="${c%%--*}"; args="${c#*--}"
  echo "=== $c" | tee -a gpurun_out/sweep.log
  env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --no-cpu-baseline $args >> gpurun_out/sweep.log 2>&1
  rc=$?
  tail -1 gpurun_out/sweep.log | python -c "import sys,json; l=sys.stdin.read(); d=json.loads(l) if l.startswith('{') else None; print(f'rc=$rc', d and (round(d['value']/1e9,4), 'Gsamples/s', round(d['roofline']['achieved']), 'GB/s', round(d['roofline']['frac'],3)))"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after rc=$rc"; exit $rc; fi
done
