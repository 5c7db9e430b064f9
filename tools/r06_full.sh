set -o pipefail
O=gpurun_out/r06_full; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
