#!/bin/bash
# c4 chain kernel: one bench line, then FETCH_SIZE and WRITE_SIZE passes (separate --pmc runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof_c4x}
ARGS="--workload c4 --no-cpu-baseline --secondary= --steps 3 --warmup 1 --prewarm-s 0.3 ${EXTRA:-}"
mkdir -p $OUT
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench timeout -k 10 200 python3 bench.py $ARGS > $OUT/bench.log 2>&1
python3 -c "
import json; l=[x for x in open('$OUT/bench.log') if x.startswith('{')][-1]; o=json.loads(l)
print('c4', round(o['value']/1e6,1), 'M/s', round(o['roofline']['avg_kernel_ms'],2), 'ms', o['roofline']['kernel'][:30])"
step fetch timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS
step write timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 bench.py $ARGS
python3 - <<PY
import csv, collections
for kind in ("fetch", "write"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open("$OUT/%s/run_counter_collection.csv" % kind)):
        if "chain_sparse" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(kind, k, "KiB/launch", sum(v) / len(v), "B/sample", sum(v) / len(v) * 1024 / 20e6)
PY
