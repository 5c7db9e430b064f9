cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread -k "gram" > gpurun_out/gram_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gram_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
VARIANTS="gram gram_d4k" bash tools/exp_gram.sh
