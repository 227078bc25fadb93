#!/bin/bash
# PMC passes on the align kernel (each pass its own rocprofv3 run, counters only + kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --pairs 512"
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "$@"; do
    i=$((i+1))
    echo "== pass $i: $set"
    timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- $BENCH > gpurun_out/pmc/p$i.log 2>&1
    rc=$?
    echo "== pass $i rc=$rc"
    if [ "$rc" -ge 124 ]; then exit $rc; fi
done
