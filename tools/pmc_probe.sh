#!/bin/bash
# PMC passes over an arbitrary command (each pass its own rocprofv3 run, counters + kernel trace).
# usage: tools/pmc_probe.sh OUTDIR "CMD" "COUNTERS 1" "COUNTERS 2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=$1; cmd=$2; shift 2
mkdir -p "$out"
rocprofv3 -L > "$out/counters_list.txt" 2>&1 || true
i=0
for set in "$@"; do
    i=$((i+1))
    echo "== pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$out/p$i" -o run -- $cmd > "$out/p$i.log" 2>&1
    rc=$?
    echo "== pass $i rc=$rc"
    if [ "$rc" -ge 124 ]; then exit $rc; fi
done
