set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_fold2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k "fold or pipeline or two_ranks or rccl" > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python3 bench.py --secondary= --no-cpu-baseline --workload c2 --steps 20 --warmup 5 > $O/bench_c2_$r.out 2>&1 || exit 1
tail -c 1500 $O/bench_c2_$r.out | tr ',' '\n' | grep -E '"value"|ms_per_step|avg_kernel_ms|avg_epoch_ms|"frac'
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 bench.py --secondary= --no-cpu-baseline --workload c2 --steps 20 --warmup 5 --prewarm-s 0.3 > $O/bench_c2_trace.out 2>&1 || exit 1
