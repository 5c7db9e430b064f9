#!/bin/bash
# LDS / instruction counters of chain_sparse_gram on a c4-shaped 4M-row shard (one --pmc pass each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_gram
export TMPDIR=/tmp
B="python3 bench.py --workload c4 --rows 4000000 --no-cpu-baseline --secondary= --prewarm-s 0 --steps 1 --warmup 0"
i=0
for c in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  PSGD_SPARSE_KERNEL=${KERNEL:-gram} timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_gram/p$i -o p$i -- $B > gpurun_out/pmc_gram/run$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_gram/run$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_gram/p*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if 'chain_sparse' not in r.get('Kernel_Name', ''): continue
        agg[r['Counter_Name']] += float(r['Counter_Value'])
    print(f.split('/')[-1], dict(agg))
PY
