#!/bin/bash
# chain_sparse_gram A/B on c4-shaped shards: bench lines + PSGD_STAMPS per-wave cycles per row
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { tag=$1; shift; echo "== $tag"; env "$@" timeout -k 10 150 python bench.py --workload c4 --rows ${ROWS:-4000000} --no-cpu-baseline --secondary= --prewarm-s 0.3 --steps 2 --warmup 1 ${EXTRA:-} > gpurun_out/expg_$tag.log 2>&1; rc=$?; python -c "
import json
txt=open('gpurun_out/expg_$tag.log').read()
l=[x for x in txt.splitlines() if x.startswith('{')]
o=json.loads(l[-1]) if l else None
st=[x for x in txt.splitlines() if x.startswith('psgd stamps')][-8:]
print('$tag', 'rc=$rc', (round(o['value']/1e6,1), round(o['roofline']['avg_kernel_ms'],3)) if o else txt[-800:])
print('\n'.join(st))"; [ $rc -eq 0 ] || exit $rc; }
for v in ${VARIANTS:-gram gram_d4k lds}; do
  case $v in
    gram) run $v PSGD_SPARSE_KERNEL=gram PSGD_STAMPS=1 ;;
    gram_d4k) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=gram PSGD_STAMPS=1 ;;
    lds) run $v PSGD_SPARSE_KERNEL=lds PSGD_STAMPS=1 ;;
    lds_d4k) EXTRA="--features 4096" run $v PSGD_SPARSE_KERNEL=lds PSGD_STAMPS=1 ;;
  esac
done
