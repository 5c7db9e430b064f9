#!/bin/bash
# Cost-probe builds of chain_sparse_lds (PSGD_LDS_EXP bits, psgd_sparse_lds.hip; wrong results):
# tools/libpsgd_lds_exp<N>.so = the product objects with psgd_sparse_lds.hip built with
# -DPSGD_LDS_EXP=N. usage: tools/build_lds_probes.sh N1 N2 ...   (run after `make` in csrc)
cd "$(dirname "$0")/../spark-parallelized-sgd_amd/csrc"
F="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -ffp-contract=off -w"
for n in "$@"; do
  ( /opt/rocm/bin/hipcc $F -DPSGD_LDS_EXP=$n -c psgd_sparse_lds.hip -o /tmp/psgd_sparse_lds_exp$n.o &&
    /opt/rocm/bin/hipcc $F -shared -o ../../tools/libpsgd_lds_exp$n.so psgd_kernels.o psgd_split.o psgd_block.o \
      psgd_block64.o psgd_sparse.o /tmp/psgd_sparse_lds_exp$n.o psgd_multinomial.o psgd_probe.o psgd_libsvm.o psgd_capi.o &&
    echo "built libpsgd_lds_exp$n.so" ) &
done
wait
