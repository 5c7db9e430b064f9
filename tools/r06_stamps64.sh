set -o pipefail
O=gpurun_out/r06_stamps64; mkdir -p $O
for a in "48828 256 1024 0 0 4 2" "48828 256 1024 1 0 4 2" "39062 256 512 1 0 4 2" "39062 256 512 0 0 4 2" "48828 256 1024 0 0 8 2"; do
  echo "== $a" >> $O/stamps.log
  timeout -k 10 60 tools/chain_bench64 $a >> $O/stamps.log 2>&1 || exit 1
done
