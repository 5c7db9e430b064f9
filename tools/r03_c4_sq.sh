#!/bin/bash
# c4 chain_sparse_lds: SQ instruction / LDS counters (one pass of <= 8 SQ counters each), tail vs
# all-LDS (d = 4,096) shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c4_sq
mkdir -p $OUT
A="--secondary= --no-cpu-baseline --workload c4 --steps 2 --warmup 1 --prewarm-s 0.2 --rows 4000000"
step() { echo "== $1"; shift; "$@" > /dev/null 2>&1; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step "tail lds" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAVES -f csv -d $OUT/tail -o run -- python3 bench.py $A
step "all-lds lds" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAVES -f csv -d $OUT/alllds -o run -- python3 bench.py $A --features 4096
step "tail lds2" timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -f csv -d $OUT/tail2 -o run -- python3 bench.py $A
