#!/bin/bash
# chain_split per-sample cycle split at c3 for H = 1, 2, 4 compute waves:
# the diagnostic builds `make -C spark-parallelized-sgd_amd/csrc stamps_h` (PSGD_SPLIT_HMAX=1/2,
# and 4: stamps_h4 -- round 6; round 5 used tools/libpsgd_stamps.so), one bench epoch each with PSGD_STAMPS=1 (stderr: per compute
# wave, cycles per sample: total, dot + reduction, exchange wait, multiplier + update).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/split_h
mkdir -p $out
for lib in ${LIBS:-stamps_h1 stamps_h2 stamps_h4}; do
  for spec in "f32 adagrad" "f32 adam" "f64 adagrad" "f64 adam"; do
    set -- $spec
    f=$out/${lib}_$1_$2.log
    PSGD_STAMPS=1 PSGD_LIB=tools/libpsgd_$lib.so timeout -k 10 120 python bench.py --workload c3 --compute $1 \
        --updater $2 --steps 2 --warmup 1 --prewarm-s 0 --secondary= --no-cpu-baseline --detail '' > $f 2>&1 || exit 1
    echo "== $lib $1 $2: $(grep -o '"avg_kernel_ms":[0-9.]*' $f) $(grep -o '"variant":[0-9]*' $f)"
    grep "psgd stamps" $f | tail -16 | sort | uniq | head -16
  done
done
