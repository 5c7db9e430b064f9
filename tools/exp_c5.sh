#!/bin/bash
# c5 (L2 logistic CSR, 2^22 features) experiments: one bench line per variant on a bounded shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { tag=$1; shift; echo "== $tag"; timeout -k 10 ${T:-150} env "$@" python bench.py --workload ${WL:-c5} --no-cpu-baseline --secondary= --prewarm-s 0.3 --steps 2 --warmup 1 ${EXTRA:-} > gpurun_out/exp5_$tag.log 2>&1; rc=$?; python -c "
import json
txt=open('gpurun_out/exp5_$tag.log').read()
l=[x for x in txt.splitlines() if x.startswith('{')]
o=json.loads(l[-1]) if l else None
st=[x for x in txt.splitlines() if x.startswith('psgd stamps')][-6:]
print('$tag', 'rc=$rc', (round(o['value']/1e6,1), round(o['roofline']['avg_kernel_ms'],3), round(o['roofline']['avg_epoch_ms'],3), o['roofline']['kernel'][:30]) if o else txt[-1500:])
print('\n'.join(st))"; [ $rc -eq 0 ] || exit $rc; }
for v in ${VARIANTS:-base}; do
  case $v in
    base) EXTRA="--rows 4000000" run $v PSGD_X=0 ;;
    p256) EXTRA="--rows 4000000 --chains 256" run $v PSGD_X=0 ;;
    p4096) EXTRA="--rows 4000000 --chains 4096" run $v PSGD_X=0 ;;
    d20) EXTRA="--rows 4000000 --features 1048576" run $v PSGD_X=0 ;;
    d16) EXTRA="--rows 4000000 --features 65536" run $v PSGD_X=0 ;;
    d16plain) EXTRA="--rows 4000000 --features 65536" run $v PSGD_SPARSE_KERNEL=plain ;;
    bs8) EXTRA="--rows 4000000" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_STAMPS=1 ;;
    bs4) EXTRA="--rows 4000000" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_SPARSE_SK=4 PSGD_STAMPS=1 ;;
    bs16) EXTRA="--rows 4000000" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_SPARSE_SK=16 PSGD_STAMPS=1 ;;
    bs8_20m) EXTRA="--rows 20000000" run $v PSGD_SPARSE_KERNEL=bsearch ;;
    bs16_20m) EXTRA="--rows 20000000" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_SPARSE_SK=16 ;;
    plain_20m) EXTRA="--rows 20000000" run $v PSGD_SPARSE_KERNEL=plain ;;
    c4lds) EXTRA="--rows 20000000" T=200 run $v PSGD_X=0 ;;
    m_plain) EXTRA="--rows 4000000 --features 262144 --chains 256" run $v PSGD_SPARSE_KERNEL=plain ;;
    m_bs8) EXTRA="--rows 4000000 --features 262144 --chains 256" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_STAMPS=1 ;;
    m_bs4) EXTRA="--rows 4000000 --features 262144 --chains 256" run $v PSGD_SPARSE_KERNEL=bsearch PSGD_SPARSE_SK=4 PSGD_STAMPS=1 ;;
    p256_plain) EXTRA="--rows 20000000 --chains 256" run $v PSGD_SPARSE_KERNEL=plain ;;
    p2048_plain) EXTRA="--rows 20000000 --chains 2048" run $v PSGD_SPARSE_KERNEL=plain ;;
  esac
done
