# c4 cost probes: the chain_sparse_lds launch with one part of the chain
# wave's per-sample path removed at a time (tools/build_lds_probes.sh builds; wrong results):
# 4 = no wave reduction, 8 = the coefficient does not wait for the dot, 16 = no wait for the tail
# gathers, 24 = 8 + 16. The vector-set re-roll keeps every process in the same placement mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_c4_probe; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for lib in product 4 8 16 24; do
    if [ $lib = product ]; then L=spark-parallelized-sgd_amd/libpsgd.so; else L=tools/libpsgd_lds_exp$lib.so; fi
    CS="f32 f64"; case $lib in 16|24) CS=f32;; esac   # (16/24 in fp64: the chain's watchdog fires)
    for c in $CS; do
      PSGD_LIB=$L timeout -k 10 200 python3 bench.py --workload c4 --compute $c --secondary= --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/out.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/out.json').read().strip().splitlines()[-1]);print('rep $rep lib $lib $c', round(d['roofline']['avg_kernel_ms'],3))" >> $O/probe.log
    done
  done
done
cat $O/probe.log
