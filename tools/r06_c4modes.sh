# c4's two per-process modes: the same bench process repeated under PMC
# counters (cycles, clock, instruction counts), then which mode each process landed in; and the
# full 125M-row c5 shard as the N > 1 secondary runs it (time and memory)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06_c4modes; mkdir -p $O
P=/tmp/r06_pmc; mkdir -p $P
for i in 1 2 3 4 5; do
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -f csv -d $P/p$i -o run -- python3 bench.py --workload c4 --secondary= --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 - $P/p$i/run_counter_collection.csv > $O/pmc$i.json <<'PY'
import csv, json, sys, statistics
acc = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "chain_sparse_lds" not in r["Kernel_Name"]:
        continue
    acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
print(json.dumps({c: {"dispatches": len(v), "mean": statistics.mean(v.values()),
                      "median": statistics.median(v.values())} for c, v in acc.items()}))
PY
done
T0=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --workload c2 --secondary c5:f32 --secondary-rows 125000000 --no-cpu-baseline --steps 20 --warmup 5 --detail $O/c5full_detail.json > $O/c5full.json 2> $O/c5full.err || { tail -5 $O/c5full.err; exit 1; }
T1=$(date +%s.%N)
python3 -c "print('c5 full-shard bench process seconds:', $T1 - $T0)"
tail -c 700 $O/c5full.json
