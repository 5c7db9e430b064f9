# Round-6 last profiles of the shipped library (profiles/r06last_*): per workload, the
# rocprofv3 kernel-trace + stats pass and separate FETCH_SIZE / WRITE_SIZE PMC passes
# (tools/profile.sh), summarised on the box (tools/pmc_summary.py) so only small files come back.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06last; mkdir -p $O
export PROF_OUT=/tmp/r06prof
for n in ${NAMES:-c2 c3_f32 c4_f32 c5 c2_f64}; do
  timeout -k 10 900 bash tools/profile.sh $n > $O/$n.profile.log 2>&1 || { tail -20 $O/$n.profile.log; exit 1; }
  cp $PROF_OUT/$n/trace/run_kernel_stats.csv $O/r06last_${n}_kernel_stats.csv
  rows=""; case $n in c5*) rows="--rows 20000000";; esac
  python3 tools/pmc_summary.py $PROF_OUT/$n $O/r06last_${n}_pmc.json --workload ${n%%_*} $rows > /dev/null || exit 1
  rm -rf $PROF_OUT/$n
done
ls -la $O
