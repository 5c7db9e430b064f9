#!/bin/bash
# chain_split SQ instruction counters at c3 (fp32 / fp64 AdaGrad), one <= 8-counter pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/split_sq
mkdir -p $OUT
A="--secondary= --no-cpu-baseline --workload c3 --updater adagrad --steps 2 --warmup 1 --prewarm-s 0.2 --rows 2500000"
step() { echo "== $1"; shift; "$@" > /dev/null 2>&1; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step f32 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -f csv -d $OUT/f32 -o run -- python3 bench.py $A
step f64 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -f csv -d $OUT/f64 -o run -- python3 bench.py $A --compute f64
