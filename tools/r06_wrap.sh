set -o pipefail
O=gpurun_out/r06_wrap; mkdir -p $O; : > $O/wrap.log
for rep in 1 2 3; do
 for b in chain_bench64_wrap0 chain_bench64_wrap1; do
  for a in "48828 256 1024 0 0 8 2" "48828 256 1024 1 0 8 2" "48828 256 1024 0 0 8 2 1e-30"; do
   echo "== $b $a" >> $O/wrap.log
   timeout -k 10 60 tools/$b $a > $O/tmp.out 2>&1 || { cat $O/tmp.out >> $O/wrap.log; exit 1; }
   head -1 $O/tmp.out >> $O/wrap.log
  done
 done
done
