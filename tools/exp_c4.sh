#!/bin/bash
# c4 sparse-kernel variants (A/B): one bench line each on a 4M-row shard; PSGD_STAMPS=1 prints
# per-chain cycle counters per row (chain / loader / tagger total and wait) on stderr.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { tag=$1; shift; echo "== $tag"; env "$@" timeout -k 10 120 python bench.py --workload c4 --rows 4000000 --no-cpu-baseline --secondary= --prewarm-s 0.3 --steps 2 --warmup 1 ${EXTRA:-} > gpurun_out/exp_$tag.log 2>&1; rc=$?; python -c "
import json,sys
txt=open('gpurun_out/exp_$tag.log').read()
l=[x for x in txt.splitlines() if x.startswith('{')]
o=json.loads(l[-1]) if l else None
st=[x for x in txt.splitlines() if x.startswith('psgd stamps')][-6:]
print('$tag', 'rc=$rc', (round(o['value']/1e6,1), round(o['roofline']['avg_kernel_ms'],3), o['roofline']['kernel'][:24]) if o else txt[-800:])
print('\n'.join(st))"; [ $rc -eq 0 ] || exit $rc; }
for v in ${VARIANTS:-lds4 lds8 lds4_d4k lds8_d4k}; do
  case $v in
    lds4) run $v PSGD_SPARSE_KERNEL=lds PSGD_STAMPS=1 ;;
    lds8) run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_SK=8 PSGD_STAMPS=1 ;;
    lds4_d4k) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=lds PSGD_STAMPS=1 ;;
    lds8_d4k) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_SK=8 PSGD_STAMPS=1 ;;
    spec) run $v PSGD_SPARSE_KERNEL=spec PSGD_STAMPS=1 ;;
    lds4_h10k) run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_LDS_HEAD=10000 PSGD_STAMPS=1 ;;
    lds8_h10k) run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_LDS_HEAD=10000 PSGD_SPARSE_SK=8 PSGD_STAMPS=1 ;;
    lds4_d30k) EXTRA="--features 30000" run $v PSGD_SPARSE_KERNEL=lds PSGD_STAMPS=1 ;;
    lds4_d4k_h1364) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_LDS_HEAD=1364 PSGD_STAMPS=1 ;;
    lds4_d4k_h4000) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_LDS_HEAD=4000 PSGD_STAMPS=1 ;;
    lds4_h2000) run $v PSGD_SPARSE_KERNEL=lds PSGD_SPARSE_LDS_HEAD=2000 PSGD_STAMPS=1 ;;
  esac
done
