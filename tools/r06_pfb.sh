set -o pipefail
O=gpurun_out/r06_pfb; mkdir -p $O
for rep in 1 2; do
 for b in chain_bench_pf0 chain_bench_pf1; do
  for a in "39062 256 512 1 0" "39062 256 512 1 0 1e-30" "39062 256 512 1 1 1e-30"; do
   echo "== $b $a" >> $O/pf.log
   timeout -k 10 60 tools/$b $a > $O/tmp.out 2>&1 || { cat $O/tmp.out >> $O/pf.log; exit 1; }
   head -1 $O/tmp.out >> $O/pf.log
  done
 done
done
