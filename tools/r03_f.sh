#!/bin/bash
# Where scattered 4-byte stores go: WRITE_SIZE per store for a footprint far beyond L2 (c5: 17 GB)
# and for one that fits the XCDs' L2 (1,024 chains x 4,096 floats = 16 MB), per store policy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/wr_r03
mkdir -p $OUT
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step counters timeout -k 10 120 rocprofv3 -L > $OUT/counters_avail.txt 2>&1
step valu timeout -k 10 60 tools/valu_rate
step big timeout -k 10 200 tools/gather_bench 4000 1024 4194304
step small timeout -k 10 200 tools/gather_bench 4000 1024 4096
step big_write timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/big_write -o run -- tools/gather_bench 4000 1024 4194304
step small_write timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/small_write -o run -- tools/gather_bench 4000 1024 4096
step small_fetch timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/small_fetch -o run -- tools/gather_bench 4000 1024 4096
