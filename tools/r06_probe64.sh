set -o pipefail
O=gpurun_out/r06_probe64; mkdir -p $O
for b in ${BINS:-chain_bench64 chain_bench64_e1 chain_bench64_e2 chain_bench64_new}; do
 for a in "39062 256 512 1 0 4 2" "39062 256 512 1 0 4 2 1e-30" "39062 256 512 0 0 4 2" "48828 256 1024 0 0 4 2" "48828 256 1024 0 0 8 2"; do
  echo "== $b $a" >> $O/probe.log
  timeout -k 10 60 tools/$b $a > $O/tmp.out 2>&1 || { cat $O/tmp.out >> $O/probe.log; exit 1; }
  head -1 $O/tmp.out >> $O/probe.log
 done
done
