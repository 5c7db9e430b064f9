set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_fold; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $O/trace -o run -- python3 bench.py --secondary= --no-cpu-baseline --workload c2 --steps 20 --warmup 5 --prewarm-s 0.3 > $O/bench_c2.out 2>&1 || exit 1
tail -c 300 $O/bench_c2.out
