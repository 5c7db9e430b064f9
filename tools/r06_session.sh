set -o pipefail
O=gpurun_out/r06s1; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_vmm.py "tests/test_gpu_configs.py::test_bench_two_ranks_gloo" -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do
  $T 200 python bench.py --workload c4 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c4_fence_$i.json 2>$O/c4_fence_$i.err &&
  PSGD_LIB=tools/libpsgd_nofence.so $T 200 python bench.py --workload c4 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c4_nofence_$i.json 2>$O/c4_nofence_$i.err || exit 1
done
$T 200 python bench.py --workload c4 --compute f64 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c4f64_fence.json 2>&1 &&
PSGD_LIB=tools/libpsgd_nofence.so $T 200 python bench.py --workload c4 --compute f64 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c4f64_nofence.json 2>&1 || exit 1
for v in 1 0 1 0; do
  PSGD_VMM=$v $T 200 python bench.py --workload c5 --rows 20000000 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c5_vmm${v}_$RANDOM.json 2>&1 || exit 1
done
$T 200 python bench.py --workload c5 --compute f64 --rows 20000000 --secondary '' --no-cpu-baseline --steps 10 --warmup 3 --detail '' > $O/c5f64.json 2>&1 || exit 1
echo ALL OK
