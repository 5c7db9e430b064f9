#!/bin/bash
# Profiles for profiles/: per workload, one rocprofv3 kernel-trace + stats pass and
# separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md §HBM), of the bench command
# for that line (bench.py --secondary= ...). Summarised locally by tools/pmc_summary.py.
# usage: tools/profile.sh name1 name2 ...   (names below; default: all; PROF_OUT = output dir)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
declare -A ARGS=(
  [c2]="--workload c2"
  [c2_f64]="--workload c2 --compute f64"
  [c3_f32]="--workload c3"
  [c3_f64]="--workload c3 --compute f64"
  [c3_f64rows]="--workload c3 --compute f64 --storage f64"
  [c4_f32]="--workload c4"
  [c4_f64]="--workload c4 --compute f64"
  [c4_f64rows]="--workload c4 --compute f64 --storage f64"
  [c5]="--workload c5 --rows 20000000"
  [c5_f64]="--workload c5 --compute f64 --rows 20000000"
  [c5_f64rows]="--workload c5 --compute f64 --storage f64 --rows 20000000"
  [c3_f32_adagrad]="--workload c3 --updater adagrad"
  [c3_f32_adam]="--workload c3 --updater adam"
  [c3_f64_adagrad]="--workload c3 --compute f64 --updater adagrad"
  [c3_f64_adam]="--workload c3 --compute f64 --updater adam"
  [c1]="--workload c1 --compute f64"
)
NAMES=${@:-c2 c2_f64 c3_f32 c3_f64 c3_f64rows c4_f32 c4_f64 c5 c3_f32_adagrad c3_f32_adam c3_f64_adagrad c3_f64_adam}
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for n in $NAMES; do
  A="--secondary= --no-cpu-baseline ${ARGS[$n]}"
  D=$OUT/$n
  mkdir -p $D
  step "$n trace" timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python3 bench.py $A
  step "$n fetch" timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- python3 bench.py $A
  step "$n write" timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $D/write -o run -- python3 bench.py $A
done
# instruction mix (VALU vs MFMA vs LDS) of the headline and the fp64 c3 kernel
for n in c2 c3_f64; do
  case " $NAMES " in *" $n "*)
    step "$n insts" timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES -f csv -d $OUT/$n/insts -o run -- python3 bench.py --secondary= --no-cpu-baseline ${ARGS[$n]};;
  esac
done
find $OUT -name "*.csv" | sort | head -100
