#!/bin/bash
# Diagnostic: sample the GPU's clocks, power and temperatures every half second while a command
# runs (is a workload's slowdown after the first seconds a power / thermal state, not the kernel?).
# usage: bash tools/clock_watch.sh OUT.log CMD...   (samples go to OUT.log, the command's output to stdout)
out=$1; shift
: > "$out"
(
    while :; do
        echo "== $(date +%s.%N)" >> "$out"
        timeout 5 amd-smi metric -p -c -t >> "$out" 2>&1
        sleep 0.5
    done
) &
watcher=$!
"$@"
rc=$?
kill $watcher 2>/dev/null
wait $watcher 2>/dev/null
exit $rc
