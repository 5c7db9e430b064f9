set -o pipefail
O=gpurun_out/r06_c5cal; mkdir -p $O
for v in 1 0 1 0 1 0; do
  for c in f32 f64; do
    PSGD_VMM=$v timeout -k 10 200 python bench.py --workload c5 --compute $c --rows 20000000 --secondary '' --no-cpu-baseline --steps 8 --warmup 2 --detail '' > $O/out.json 2>$O/err.log || { cat $O/err.log; exit 1; }
    python -c "import json;d=json.loads(open('$O/out.json').read().strip().splitlines()[-1]);print('vmm=$v $c', round(d['roofline']['avg_kernel_ms'],3), d['c5_store_probe'])" >> $O/cal.log
  done
done
cat $O/cal.log
