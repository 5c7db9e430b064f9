#!/bin/bash
# One GPU-box session as a list of steps, run in order; the first failing step ends the session
# (a GPU fault, abort or time limit must not be followed by more GPU work). Every step runs under
# its own time limit and logs to gpurun_out/session/NN_KIND.log (its tail is echoed).
#
# usage (from gpurun): bash tools/gpu_session.sh 'STEP' ['STEP' ...]
#   test:EXPR          python -m pytest tests -m gpu -k EXPR  (EXPR 'all': the whole GPU suite)
#   smoke              __graft_entry__.smoke()
#   bench:ARGS         python bench.py ARGS
#   prof:NAME:ARGS     rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE PMC passes
#                      (one counter block per pass, MI355X_MICROARCH.md §HBM) of
#                      `bench.py --secondary= --no-cpu-baseline ARGS` into gpurun_out/prof/NAME
#                      (summarise with tools/pmc_summary.py)
#   pmc:NAME:CTRS:ARGS one rocprofv3 --pmc pass with the counters CTRS (comma-separated, within
#                      one pass's limits) of the same bench command
#   tool:BIN ARGS      a tools/ binary (gather_bench, chain_bench, ...)
#   run:CMD            any other command
# STEP_TIMEOUT (seconds, default 600) bounds each step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LOG=gpurun_out/session
mkdir -p $LOG gpurun_out/prof
T=${STEP_TIMEOUT:-600}
n=0
go() {   # go KIND CMD...: run one step under its limit, stop the session on failure
    local kind=$1; shift
    n=$((n + 1))
    local f=$LOG/$(printf %02d $n)_$kind.log
    echo "== step $n ($kind): $*"
    timeout -k 10 $T "$@" > $f 2>&1
    local rc=$?
    tail -25 $f
    echo "rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
bench_args() { echo "--secondary= --no-cpu-baseline $1"; }
for step in "$@"; do
    kind=${step%%:*}
    rest=${step#*:}
    case $kind in
    test)
        if [ "$rest" = all ]; then k=(); else k=(-k "$rest"); fi
        go test python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}";;
    smoke)
        go smoke python -u -c "import __graft_entry__ as g; g.smoke()";;
    bench)
        go bench python -u bench.py $rest;;
    prof)
        name=${rest%%:*}; args=$(bench_args "${rest#*:}"); D=gpurun_out/prof/$name
        go trace rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python3 bench.py $args
        go fetch rocprofv3 --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- python3 bench.py $args
        go write rocprofv3 --pmc WRITE_SIZE -f csv -d $D/write -o run -- python3 bench.py $args;;
    pmc)
        name=${rest%%:*}; rest=${rest#*:}; ctrs=${rest%%:*}; args=$(bench_args "${rest#*:}")
        go pmc rocprofv3 --pmc ${ctrs//,/ } -f csv -d gpurun_out/prof/$name/pmc -o run -- python3 bench.py $args;;
    tool)
        go tool tools/$rest;;
    run)
        go run bash -c "$rest";;
    *)
        echo "unknown step $step"; exit 2;;
    esac
done
