set -o pipefail
O=gpurun_out/r06_sig; mkdir -p $O; : > $O/sig.log
for rep in 1 2; do
 for b in chain_bench64_sig1 chain_bench64_sig2; do
  for a in "25000 4 128 0 0 8 1" "25000 256 128 0 0 8 1" "39062 256 512 0 0 4 2" "48828 256 1024 0 0 4 2" "48828 256 1024 0 0 8 2" "39062 256 512 0 0 4 2 1e-30"; do
   echo "== $b $a" >> $O/sig.log
   timeout -k 10 60 tools/$b $a > $O/tmp.out 2>&1 || { cat $O/tmp.out >> $O/sig.log; exit 1; }
   head -1 $O/tmp.out >> $O/sig.log
  done
 done
done
